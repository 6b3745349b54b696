// clustering.h — the stages of `categorization` after index construction
// (ReadClusteringEngine::run_clustering / export_components,
// src/clustering/ReadClusteringEngine.cpp:301-826).
//
// The engine starts from the state construct_indices leaves (one component per read with >= 1
// SDK hit; kmer_component_index; read metadata), which the GPU lookup produced.  The all-reads
// connection pass (get_all_connections / the filtered get_connections call at :750-755) runs on
// the GPU (hga_connections_run) on the device-resident indices; every later get_connections
// call works on merged components and the edited kmer_component_index and runs on the host.
//
// Determinism: the reference iterates tsl::robin_map / std::unordered_map containers and sorts
// connections with an unstable std::sort on the score only, so ties and container orders are
// unspecified there.  Here components are visited in ascending ComponentID order, connections
// are ordered by (score descending, x ascending, y ascending) — the GPU's order — and ties of
// max_element take the smallest id.  With those orders fixed, every rule below follows the
// reference statement by statement, including its edge behaviour (kmer_component_index
// removal drops the tail of a list once the removal list is exhausted, :405-416; unsigned BFS
// distances, :529; merged components carry de-duplicated KmerIDs, Utils.h merge_n_vectors).
// Spectral clustering uses a Jacobi eigensolver (Eigen2's SelfAdjointEigenSolver in the
// reference) and the Evrot rotation (src/lib/clustering/Evrot.cpp, method 1: true gradient):
// floating-point results can differ in degenerate eigenspaces, so the final read->component
// assignment is "parity unpinned" (SURVEY.md §8(c)).
#pragma once

#include <cstdint>
#include <map>
#include <ostream>
#include <set>
#include <string>
#include <utility>
#include <functional>
#include <vector>

#include "hga.h"
#include "seqio.h"

namespace hgah {

using ComponentID = uint32_t;
using KmerID = uint32_t;
using Score = uint64_t;

struct Connection {   // ComponentConnection, ReadClusteringEngine.h:127-136
    ComponentID x, y;
    Score score;
    bool is_good;
};
using SpanningTree = std::vector<std::pair<ComponentID, ComponentID>>;
using ComponentList = std::vector<ComponentID>;

struct ClusteringConfig {   // ReadClusteringConfig, ReadClusteringEngine.h:138-148
    int scaffold_component_min_size = 30;
    int scaffold_component_max_size = -1;
    double scaffold_forming_fraction = 0.15;
    Score scaffold_forming_score = 0;
    Score enrichment_connections_min_score = 20;
    Score tail_amplification_min_score = 40;
    int threads = 1;
    int spectral_dims = 16;
    bool force_spectral = false;
};

// (score desc, x asc, y asc) — the order of hga_connections_fetch.
void sort_connections(std::vector<Connection>& c);

// union_find (:424-489).  Components in ascending order of their root id.
std::vector<std::pair<ComponentList, SpanningTree>> union_find(const std::vector<Connection>& connections,
                                                               const std::set<ComponentID>& restricted,
                                                               int min_component_size, int max_component_size);

// spectral_clustering (:653-697) with SpectralClustering + ClusterRotate + Evrot.
std::vector<ComponentList> spectral_clustering(const std::vector<Connection>& connections, int dims);

// Symmetric eigen-decomposition (cyclic Jacobi): eigenvalues ascending, eigenvectors as columns
// of the row-major n x n `vectors`.
void sym_eigen(std::vector<double> a, int n, std::vector<double>& values, std::vector<double>& vectors);

class ClusteringEngine {
   public:
    // State after construct_indices (ReadClusteringEngine.cpp:234-299) from the lookup's CSR
    // outputs (hga_lookup_result): read i has ReadID first_read_id + i.  `gpu` (may be null)
    // holds the same lookup on the device for the first connection pass.
    ClusteringEngine(const ClusteringConfig& cfg, bool debug, const RecordSet& reads, uint32_t first_read_id,
                     std::vector<uint64_t> hit_ptr, std::vector<uint32_t> sorted_kid, std::vector<uint64_t> first_ptr,
                     std::vector<uint32_t> first_kid, std::vector<uint32_t> first_pos,
                     const std::vector<uint64_t>& kci_ptr, const std::vector<uint32_t>& kci_read, hga_ctx* gpu);

    // run_clustering after construct_indices (:737-801); the timing lines go to `out`.
    std::vector<ComponentID> run(std::ostream& out);

    // print_components (:189-198) under debug: ids sorted in place by size, largest first (ties by
    // ascending id; std::sort leaves them unspecified there), then one ReadComponent::to_string line
    // each (ReadClusteringEngine.h:52-112): "#<id> : <per-category read counts a/b/..> [<per-category
    // simulator-coordinate intervals>]".
    void print_components(std::vector<ComponentID>& ids, std::ostream& out) const;
    std::string component_string(ComponentID id) const;

    // export_components (:804-826).
    void export_components(const std::vector<ComponentID>& ids, const std::string& dir, std::ostream& out) const;

    // Stages, public for the tests.
    // keep_fraction >= 0: return only the first (size_t)(n * keep_fraction) entries of the sorted list
    // (the device path fetches just that prefix, hga_connections_fetch_range).
    std::vector<Connection> get_connections(const std::vector<ComponentID>& pivots, Score min_score,
                                            uint32_t min_kmers = 0, double keep_fraction = -1.0);
    std::vector<Connection> get_all_connections(Score min_score, double keep_fraction = -1.0);
    std::vector<ComponentID> merge_components(const std::vector<ComponentList>& components);
    void remove_merged_components();
    std::vector<ComponentID> component_ids(uint64_t threshold_size) const;

    struct Component {   // ReadComponent, ReadClusteringEngine.h:36-113
        std::vector<uint32_t> reads;   // contained_read_ids
        std::vector<KmerID> kmers;     // discriminative_kmer_ids (sorted)
        std::set<int32_t> categories;
    };
    const std::map<ComponentID, Component>& components() const { return index_; }
    const std::vector<std::vector<ComponentID>>& kmer_component_index() const { return kci_; }
    bool used_gpu() const { return gpu_calls_ > 0; }
    // Device connection pass over several ranks (categorization --gpus N): fn(pivots or empty for
    // "every read", min_score, min_kmers) -> connections in the reference order; replaces the
    // single-ctx call while the device indices describe the state.
    using DeviceConnections = std::function<std::vector<Connection>(const std::vector<ComponentID>&, Score, uint32_t)>;
    void set_device_connections(DeviceConnections fn) { dev_conn_ = std::move(fn); }

   private:
    std::vector<KmerID> accumulate_kmer_ids(const std::vector<ComponentID>& ids) const;
    uint32_t kmer_position(ComponentID read, KmerID kid) const;
    uint32_t read_length(ComponentID read) const;
    int approximate_read_overlap(ComponentID x, ComponentID y) const;
    std::pair<std::vector<ComponentID>, std::vector<ComponentID>> spanning_tree_tails(const SpanningTree& tree) const;
    std::vector<ComponentID> amplify_component(const std::vector<ComponentID>& comp, Score min_score);
    std::vector<Connection> core_component_connections(
        const std::vector<std::pair<ComponentList, SpanningTree>>& comps_and_trees);
    bool is_good(ComponentID x, ComponentID y) const;
    std::vector<Connection> host_connections(const std::vector<ComponentID>& pivots, Score min_score) const;

    ClusteringConfig cfg_;
    bool debug_;
    const RecordSet& reads_;
    uint32_t first_id_;
    std::vector<uint64_t> hit_ptr_, first_ptr_;
    std::vector<uint32_t> first_kid_, first_pos_;
    std::map<ComponentID, Component> index_;
    std::vector<std::vector<ComponentID>> kci_;
    hga_ctx* gpu_;
    DeviceConnections dev_conn_;
    bool pristine_ = true;   // no merge yet: the device indices still describe the state
    int gpu_calls_ = 0;
};

}  // namespace hgah
