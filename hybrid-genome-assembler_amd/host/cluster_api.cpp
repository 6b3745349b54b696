// cluster_api.cpp — C ABI of the host clustering stages (lib/libhga_cluster.so) for the ctypes
// mirror and the tests: the engine on construct_indices outputs, union_find, spectral
// clustering and the eigensolver.  Status 0 = ok, -1 = error (hgc_last_error()).
#include <cstdlib>
#include <cstring>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "clustering.h"

namespace {
thread_local std::string g_err;

template <class F>
int guard(F&& f) {
    try {
        g_err.clear();
        f();
        return 0;
    } catch (const std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

template <class T>
T* dup(const T* p, size_t n) {
    T* q = static_cast<T*>(std::malloc(n ? n * sizeof(T) : 1));
    if (!q) throw std::bad_alloc();
    if (n) std::memcpy(q, p, n * sizeof(T));
    return q;
}

std::vector<hgah::Connection> conns_of(const uint32_t* x, const uint32_t* y, const uint64_t* s, uint64_t n) {
    std::vector<hgah::Connection> c(n);
    for (uint64_t i = 0; i < n; ++i) c[i] = {x[i], y[i], s[i], false};
    return c;
}

// Components as a flat list: ids[] with ptr[] (CSR), caller frees both.
void put_components(const std::vector<hgah::ComponentList>& comps, uint64_t** ptr, uint32_t** ids, uint64_t* n) {
    std::vector<uint64_t> p{0};
    std::vector<uint32_t> v;
    for (auto& c : comps) {
        v.insert(v.end(), c.begin(), c.end());
        p.push_back(v.size());
    }
    *ptr = dup(p.data(), p.size());
    *ids = dup(v.data(), v.size());
    *n = comps.size();
}
}  // namespace

extern "C" {

struct hgc_config {   // ReadClusteringConfig (ReadClusteringEngine.h:138-148)
    int sc_min_size, sc_max_size;
    double sc_fraction;
    uint64_t sc_score, core_enrichment, tail_amplification;
    int threads, spectral_dims, force_spectral;
};

const char* hgc_last_error(void) { return g_err.c_str(); }
void hgc_free(void* p) { std::free(p); }

// run_clustering after construct_indices (host-only: no device state) on the lookup's CSR
// outputs; reads in reader order with ReadID = first_read_id + i.  Outputs: the returned
// component ids (ascending; under debug in print_components' order), per read the id of the returned
// component containing it (0 = none), the timing/log text (with print_components' blocks under debug).
// start / end: the reads' simulator-header coordinates (GenomeReadData start / end), null = 0.
int hgc_cluster(const char* bases, const uint64_t* offsets, const int32_t* category, const uint32_t* start,
                const uint32_t* end, uint64_t n_reads,
                uint64_t avg_read_length, uint32_t first_read_id, const uint64_t* hit_ptr, const uint32_t* sorted_kid,
                const uint64_t* first_ptr, const uint32_t* first_kid, const uint32_t* first_pos, const uint64_t* kci_ptr,
                const uint32_t* kci_read, uint32_t n_sdk, const hgc_config* cfg, int debug, uint32_t** ids_out,
                uint64_t* n_ids, uint32_t** comp_of_read, char** log_out) {
    return guard([&] {
        hgah::RecordSet rs;
        rs.bases.append(bases, n_reads ? offsets[n_reads] : 0);
        rs.offsets.assign(offsets, offsets + n_reads + 1);
        rs.category.assign(category, category + n_reads);
        if (start && end) {
            rs.start.assign(start, start + n_reads);
            rs.end.assign(end, end + n_reads);
        }
        rs.meta.avg_read_length = avg_read_length;
        hgah::ClusteringConfig c;
        c.scaffold_component_min_size = cfg->sc_min_size;
        c.scaffold_component_max_size = cfg->sc_max_size;
        c.scaffold_forming_fraction = cfg->sc_fraction;
        c.scaffold_forming_score = cfg->sc_score;
        c.enrichment_connections_min_score = cfg->core_enrichment;
        c.tail_amplification_min_score = cfg->tail_amplification;
        c.threads = cfg->threads;
        c.spectral_dims = cfg->spectral_dims;
        c.force_spectral = cfg->force_spectral != 0;
        const uint64_t H = hit_ptr[n_reads], U = first_ptr[n_reads], HK = kci_ptr[n_sdk];
        hgah::ClusteringEngine e(c, debug != 0, rs, first_read_id, std::vector<uint64_t>(hit_ptr, hit_ptr + n_reads + 1),
                                 std::vector<uint32_t>(sorted_kid, sorted_kid + H),
                                 std::vector<uint64_t>(first_ptr, first_ptr + n_reads + 1),
                                 std::vector<uint32_t>(first_kid, first_kid + U),
                                 std::vector<uint32_t>(first_pos, first_pos + U),
                                 std::vector<uint64_t>(kci_ptr, kci_ptr + n_sdk + 1),
                                 std::vector<uint32_t>(kci_read, kci_read + HK), nullptr);
        std::ostringstream log;
        const auto ids = e.run(log);
        std::vector<uint32_t> owner(n_reads, 0);
        for (auto id : ids)
            for (uint32_t r : e.components().at(id).reads) owner[r - first_read_id] = id;
        *ids_out = dup(ids.data(), ids.size());
        *n_ids = ids.size();
        *comp_of_read = dup(owner.data(), owner.size());
        const std::string s = log.str();
        *log_out = dup(s.c_str(), s.size() + 1);
    });
}

// union_find (ReadClusteringEngine.cpp:424-489) of an ordered connection list.
int hgc_union_find(const uint32_t* x, const uint32_t* y, const uint64_t* s, uint64_t n, const uint32_t* restricted,
                   uint64_t n_restricted, int min_size, int max_size, uint64_t** comp_ptr, uint32_t** comp_ids,
                   uint64_t* n_comp, uint64_t** tree_ptr, uint32_t** tree_xy) {
    return guard([&] {
        const std::set<hgah::ComponentID> r(restricted, restricted + n_restricted);
        const auto res = hgah::union_find(conns_of(x, y, s, n), r, min_size, max_size);
        std::vector<hgah::ComponentList> comps;
        std::vector<uint64_t> tp{0};
        std::vector<uint32_t> txy;
        for (auto& ct : res) {
            comps.push_back(ct.first);
            for (auto& e : ct.second) {
                txy.push_back(e.first);
                txy.push_back(e.second);
            }
            tp.push_back(txy.size() / 2);
        }
        put_components(comps, comp_ptr, comp_ids, n_comp);
        *tree_ptr = dup(tp.data(), tp.size());
        *tree_xy = dup(txy.data(), txy.size());
    });
}

// spectral_clustering (ReadClusteringEngine.cpp:653-697).
int hgc_spectral(const uint32_t* x, const uint32_t* y, const uint64_t* s, uint64_t n, int dims, uint64_t** comp_ptr,
                 uint32_t** comp_ids, uint64_t* n_comp) {
    return guard([&] { put_components(hgah::spectral_clustering(conns_of(x, y, s, n), dims), comp_ptr, comp_ids, n_comp); });
}

// Symmetric eigen-decomposition used by spectral_clustering (values ascending, vectors as
// columns of a row-major n x n matrix); caller-allocated outputs.
int hgc_sym_eigen(const double* a, int n, double* values, double* vectors) {
    return guard([&] {
        std::vector<double> v, w;
        hgah::sym_eigen(std::vector<double>(a, a + (size_t)n * n), n, v, w);
        std::memcpy(values, v.data(), (size_t)n * sizeof(double));
        std::memcpy(vectors, w.data(), (size_t)n * n * sizeof(double));
    });
}

}  // extern "C"
