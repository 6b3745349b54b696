// categorization — drop-in for the reference's `categorization` CLI
// (src/read_clustering.cpp:35-84) up to and including index construction, whose
// per-read SDK lookup (ReadClusteringEngine::construct_indices,
// src/clustering/ReadClusteringEngine.cpp:234-299) runs on the MI355X through libhga.
//
// Kept from the reference: argv (positional reads, -k/--kmers <path>, -o/--output,
// the clustering knobs, -s/--spectral, -d/--debug, -t/--threads), SDK loading with
// KmerIDs in std::unordered_set iteration order (read_clustering.cpp:18-33,
// ReadClusteringEngine.cpp:237-241), the SequenceRecordIterator metadata print,
// the default output folder "./<f1>__<f2>_clusters/" (read_clustering.cpp:78), the
// "Index construction took <ms>ms" timing line and, when every file is a category
// (ReadClusteringEngine.cpp:229), "X out of Y kmers are discriminative" (:285-297).
//
// The stages after index construction (ReadClusteringEngine.cpp:301-826) run in
// host/clustering.cpp: the first connection pass on the GPU (hga_connections_run on the
// lookup's device-resident indices), union-find, merging, spanning-tree tails, spectral
// clustering and the per-component FASTA/FASTQ export with the reference's timing lines.
// With --index-out <path> the constructed index is also written as a binary file.
//
// --gpus N (extension, default 1): N ranks in this process, one per GPU
// (ranks.h).  Every rank loads the whole SDK set and looks up a contiguous ReadID range of the
// reads; hga_lookup_gather gives every rank the whole input's index; the device connection pass
// splits its pivots over the ranks and hga_connections_gather joins them in the reference order.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <memory>
#include <set>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_set>
#include <vector>

#include "args.h"
#include "clustering.h"
#include "hga.h"
#include "phase_timer.h"
#include "ranks.h"
#include "seqio.h"

namespace {
void check(hga_status s, const char* what) {
    if (s != HGA_OK) throw std::runtime_error(std::string(what) + ": " + hga_last_error());
}

// load_text_file_kmers (src/read_clustering.cpp:18-33): KmerID = the iteration order of the
// std::unordered_set the reference fills line by line (hgah::load_kmer_text reproduces it without the
// per-key node allocations: 0.78 s -> see DESIGN.md §7 for the C2 export's 1.82 M lines).
std::pair<std::vector<uint64_t>, int> load_text_file_kmers(const std::string& path) {
    if (!std::ifstream(path)) return {{}, 0};   // (an unreadable file reads as empty there)
    int k = 0;
    std::vector<uint64_t> keys = hgah::load_kmer_text(path, &k);
    return {std::move(keys), k};
}
}  // namespace

int main(int argc, char* argv[]) {
    std::vector<std::string> read_paths;
    std::string kmer_path, output_folder_path, index_out;
    bool debug = false, force_spectral = false;
    int threads = 1, sc_min = 30, sc_max = -1, dims = 16;
    double sc_fraction = 0.15;
    uint64_t sc_score = 0, tail = 40, enrich = 20;
    hgah::ArgParser ap;
    ap.add("help", 'h', true, "Help screen", nullptr);
    ap.add("read_paths", 0, false, "Path to file with reads (FASTA or FASTQ)",
           [&](const std::string& v) { read_paths.push_back(v); });
    ap.add("kmers", 'k', false, "Path to text file with kmers", [&](const std::string& v) { kmer_path = v; });
    ap.add("output", 'o', false, "Path to folder with exported clusters",
           [&](const std::string& v) { output_folder_path = v; });
    ap.add("sc_max_size", 0, false, "Maximum size for a scaffold component", [&](const std::string& v) { sc_max = std::stoi(v); });
    ap.add("sc_min_size", 0, false, "Minimum size for a scaffold component", [&](const std::string& v) { sc_min = std::stoi(v); });
    ap.add("sc_fraction", 0, false, "Minimum score for a scaffold component forming connection",
           [&](const std::string& v) { sc_fraction = std::stod(v); });
    ap.add("sc_score", 0, false, "Minimum score for a scaffold component forming connection",
           [&](const std::string& v) { sc_score = std::stoull(v); });
    ap.add("tail_amplification", 0, false, "Minimal score for tail amplifying connections",
           [&](const std::string& v) { tail = std::stoull(v); });
    ap.add("core_enrichment", 0, false, "Minimal score for connections enriching core components",
           [&](const std::string& v) { enrich = std::stoull(v); });
    ap.add("spectral_dims", 0, false, "Number of dimensions for spectral embedding",
           [&](const std::string& v) { dims = std::stoi(v); });
    ap.add("spectral", 's', true, "Forces the usage of spectral clustering on the entire dataset",
           [&](const std::string&) { force_spectral = true; });
    ap.add("debug", 'd', true, "Debug flag. Treat read files as separate haplotype reads.",
           [&](const std::string&) { debug = true; });
    ap.add("threads", 't', false, "Number of threads to use", [&](const std::string& v) { threads = std::stoi(v); });
    ap.add("index-out", 0, false, "Write the constructed index (binary) to this path",
           [&](const std::string& v) { index_out = v; });
    int gpus = 1;
    ap.add("gpus", 0, false, "GPUs for the lookup and the first connection pass, one rank each (MI355X build "
           "extension; default 1)", [&](const std::string& v) { gpus = std::stoi(v); });
    ap.parse(argc, argv);
    for (auto& p : ap.positional) read_paths.push_back(p);
    if (ap.has("help")) {
        std::cout << ap.describe();
        return 0;
    }
    if (read_paths.empty()) throw std::invalid_argument("You need to specify paths to read files");
    if (kmer_path.empty()) throw std::invalid_argument("You need to specify path to kmers");
    hgah::PhaseTimer tm;
    const char* dev_env = std::getenv("HGA_DEVICE");
    // device set-up (HIP init, contexts) on a thread while the k-mer file and the reads are read
    std::unique_ptr<hgah::Ranks> ranks_p;
    std::exception_ptr init_err;
    std::thread init_th([&] {
        try {
            ranks_p = std::make_unique<hgah::Ranks>(gpus, dev_env ? std::atoi(dev_env) : 0);
        } catch (...) {
            init_err = std::current_exception();
        }
    });
    struct InitJoin {   // joined on every way out (an input error must not leave the thread running)
        std::thread& t;
        ~InitJoin() { if (t.joinable()) t.join(); }
    } init_join{init_th};
    auto kk = load_text_file_kmers(kmer_path);
    const int k = kk.second;
    if (k < 1 || k > 32) throw std::invalid_argument("Kmer size must be in [1, 32]");
    tm.mark("sdk_load");

    hgah::RecordSet rs = hgah::load_records(read_paths, debug, true);   // headers/qualities for the export
    for (auto& m : rs.file_meta) std::cout << m.repr();
    if (output_folder_path.empty()) output_folder_path = "./" + rs.meta.filename + "_clusters/";
    const bool engine_debug = rs.file_meta.size() == rs.categories;   // ReadClusteringEngine.cpp:229
    tm.mark("read_files");
    init_th.join();
    if (init_err) std::rethrow_exception(init_err);
    tm.mark("device_init_wait");
    hgah::Ranks& ranks = *ranks_p;
    hga_ctx* ctx = ranks.ctx[0];
    const int P = ranks.size();
    const uint64_t n_reads = rs.size();
    auto share = [&](int r) { return std::make_pair(n_reads * (uint64_t)r / P, n_reads * (uint64_t)(r + 1) / P); };
    const auto t0 = std::chrono::steady_clock::now();
    ranks.each([&](int r, hga_ctx* c) {   // rank r: the whole SDK set, its contiguous ReadID range
        const auto [a, b] = share(r);
        std::vector<uint64_t> offs(rs.offsets.begin() + (int64_t)a, rs.offsets.begin() + (int64_t)b + 1);
        for (auto& o : offs) o -= rs.offsets[a];
        check(hga_lookup_load(c, k, kk.first.data(), (uint32_t)kk.first.size()), "hga_lookup_load");
        check(hga_lookup_set_reads(c, rs.bases.data() + rs.offsets[a], offs.data(), b - a, (uint32_t)(1 + a)),
              "hga_lookup_set_reads");
        check(hga_lookup_run(c), "hga_lookup_run");
        if (P > 1) check(hga_lookup_gather(c), "hga_lookup_gather");   // every rank: the whole index
    });
    hga_lookup_sizes sz;
    check(hga_lookup_get_sizes(ctx, &sz), "hga_lookup_get_sizes");
    std::vector<uint64_t> hit_ptr(sz.n_reads + 1), first_ptr(sz.n_reads + 1), kci_ptr((size_t)sz.n_sdk + 1);
    std::vector<uint32_t> sorted_kid(sz.hits), first_kid(sz.firsts), first_pos(sz.firsts), kci_read(sz.hits);
    hga_lookup_result res{};
    res.hit_ptr = hit_ptr.data();
    res.sorted_kid = sorted_kid.data();
    res.first_ptr = first_ptr.data();
    res.first_kid = first_kid.data();
    res.first_pos = first_pos.data();
    res.kci_ptr = kci_ptr.data();
    res.kci_read = kci_read.data();
    check(hga_lookup_fetch(ctx, &res), "hga_lookup_fetch");
    const auto t1 = std::chrono::steady_clock::now();
    std::cout << "Index construction took "
              << std::chrono::duration_cast<std::chrono::milliseconds>(t1 - t0).count() << "ms\n";
    tm.mark("index_construction");

    if (engine_debug) {   // ReadClusteringEngine.cpp:285-297
        uint32_t discriminative = 0, total = 0;
        for (uint64_t id = 0; id < sz.n_sdk; ++id) {   // (the set of categories has one element iff all agree)
            const uint64_t a = kci_ptr[id], b = kci_ptr[id + 1];
            if (a == b) continue;
            const int32_t c0 = rs.category[kci_read[a] - 1];
            bool one = true;
            for (uint64_t j = a + 1; j < b && one; ++j) one = rs.category[kci_read[j] - 1] == c0;
            discriminative += one ? 1u : 0u;
            ++total;
        }
        std::cout << discriminative << " out of " << total << " kmers are discriminative \n";
        tm.mark("discriminative_check");
    }
    if (!index_out.empty()) {
        std::FILE* f = std::fopen(index_out.c_str(), "wb");
        if (!f) throw std::runtime_error("cannot write " + index_out);
        const uint64_t hdr[5] = {sz.n_reads, sz.hits, sz.firsts, sz.n_sdk, (uint64_t)k};
        std::fwrite(hdr, 8, 5, f);
        std::fwrite(hit_ptr.data(), 8, hit_ptr.size(), f);
        std::fwrite(sorted_kid.data(), 4, sorted_kid.size(), f);
        std::fwrite(first_ptr.data(), 8, first_ptr.size(), f);
        std::fwrite(first_kid.data(), 4, first_kid.size(), f);
        std::fwrite(first_pos.data(), 4, first_pos.size(), f);
        std::fwrite(kci_ptr.data(), 8, kci_ptr.size(), f);
        std::fwrite(kci_read.data(), 4, kci_read.size(), f);
        std::fclose(f);
    }
    hgah::ClusteringConfig cfg;   // ReadClusteringConfig (ReadClusteringEngine.h:138-148)
    cfg.scaffold_component_min_size = sc_min;
    cfg.scaffold_component_max_size = sc_max;
    cfg.scaffold_forming_fraction = sc_fraction;
    cfg.scaffold_forming_score = sc_score;
    cfg.enrichment_connections_min_score = enrich;
    cfg.tail_amplification_min_score = tail;
    cfg.threads = threads;
    cfg.spectral_dims = dims;
    cfg.force_spectral = force_spectral;
    hgah::ClusteringEngine engine(cfg, engine_debug, rs, 1, std::move(hit_ptr), std::move(sorted_kid),
                                  std::move(first_ptr), std::move(first_kid), std::move(first_pos), kci_ptr, kci_read,
                                  ctx);
    if (P > 1) {   // the device connection pass with the pivots split over the ranks
        std::vector<int32_t> cats;
        if (engine_debug) cats.assign(rs.category.begin(), rs.category.end());
        engine.set_device_connections([&](const std::vector<hgah::ComponentID>& pivots, hgah::Score min_score,
                                          uint32_t min_kmers) {
            std::vector<uint64_t> ns(P, 0);
            ranks.each([&](int r, hga_ctx* c) {
                std::vector<uint32_t> piv;
                if (min_kmers > 0) {   // "every read with >= min_kmers KmerIDs": this rank's ReadID range
                    const auto [a, b] = share(r);
                    for (uint64_t i = a; i < b; ++i) piv.push_back((uint32_t)(1 + i));
                } else {
                    piv.assign(pivots.begin() + (int64_t)(pivots.size() * r / P),
                               pivots.begin() + (int64_t)(pivots.size() * (r + 1) / P));
                }
                uint64_t n = 0;
                uint32_t none = 0;   // an empty list is not NULL (NULL would mean every read)
                check(hga_connections_run(c, piv.empty() ? &none : piv.data(), piv.size(), min_kmers > 0 ? min_kmers : 1, min_score,
                                          engine_debug ? cats.data() : nullptr, &n), "hga_connections_run");
                check(hga_connections_gather(c, &ns[r]), "hga_connections_gather");
            });
            const uint64_t n = ns[0];
            std::vector<uint32_t> x(n), y(n);
            std::vector<uint64_t> sc(n);
            std::vector<uint8_t> g(n);
            check(hga_connections_fetch(ctx, x.data(), y.data(), sc.data(), g.data()), "hga_connections_fetch");
            std::vector<hgah::Connection> out(n);
            for (uint64_t i = 0; i < n; ++i) out[i] = {x[i], y[i], sc[i], g[i] != 0};
            return out;
        });
    }
    tm.mark("engine_setup");
    const std::vector<hgah::ComponentID> cluster_ids = engine.run(std::cout);   // run_clustering (:699-802)
    tm.mark("run_clustering");
    engine.export_components(cluster_ids, output_folder_path, std::cout);       // read_clustering.cpp:82
    tm.mark("export_components");
    tm.total();
    return 0;
}
