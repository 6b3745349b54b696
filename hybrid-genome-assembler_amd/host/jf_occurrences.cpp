// jf_occurrences — drop-in for the reference's `jf_occurrences` CLI
// (src/jellyfish_occurrences.cpp:14-59), with the jellyfish count + dump + sort
// (src/occurrences/run_jellyfish.sh) and both string k-way merge passes of
// JellyfishOccurrenceReader (src/occurrences/JellyfishOccurrenceReader.cpp:63-135)
// replaced by the MI355X pipeline of libhga (include/hga.h).
//
// Kept from the reference: argv (positional read files, -k/--k-size, -o/--output,
// -h/--help), the specificity thresholds {70,85,90,95,99,100,100.01} (:47), the
// plot pipe to `python scripts/plotting.py --plot kmer_histogram_with_spec` with the
// Python-literal wire format (src/common/Plotting.cpp:20-37) and its "0" echo, the
// stdin prompt (:54-55), the default export name "{k}-mers_{lower}_{upper}_{p*100}%.txt"
// (:57), one k-mer per line in ascending order, and the final
// "{d} out of {e} exported kmers are discriminative" line without newline (:133).
//
// Dump cache (JellyfishOccurrenceReader.cpp:19-24): a file whose "<reads>_<k>-mers_sorted"
// exists is not read at all, its dump rows are merged verbatim (hga_count_add_rows); for every
// other file the GPU count is written back as that dump, "KMER COUNT" lines in LC_ALL=C order,
// as run_jellyfish.sh:5-6 would leave it.  HGA_DUMP_CACHE=0 skips writing.
//
// Without -k, k is chosen as the reference does (:40-44, KmerAnalysis.cpp:41-56): HyperLogLog
// estimates for k = 11, 13, ... filled on the GPU (hga_hll_registers), printed per k.
//
// HGA_DEVICE selects the GPU (default 0); HGA_PLOT_CMD overrides the plot command; HGA_TIMING=1 prints
// the wall time of each phase to stderr ("hga-timing <phase> <ms>"; stdout stays the reference's).
//
// Overlap (same outputs): the HIP / device set-up runs on a thread while the read files are parsed,
// and the dump caches are formatted and written on a thread while the histogram, the plot, the prompt
// and the export proceed (joined before exit).
//
// --gpus N (extension, default 1): N ranks in this process, one per GPU (ranks.h), each counting a
// contiguous share of every file's reads with min 1; hga_count_exchange moves the rows to their owner
// ranks (RCCL over xGMI, or a host transport when ranks share a GPU) and applies the --bc drop; the
// histogram, dumps and export are then the whole input's, written by rank 0 exactly as with one GPU.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <filesystem>
#include <iostream>
#include <map>
#include <memory>
#include <random>
#include <set>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "args.h"
#include "hga.h"
#include "kmer_analysis.h"
#include "phase_timer.h"
#include "ranks.h"
#include "seqio.h"

namespace {

void check(hga_status s, const char* what) {
    if (s != HGA_OK) throw std::runtime_error(std::string(what) + ": " + hga_last_error());
}

// run_command_with_input (src/common/Utils.cpp:24-45): popen(cmd, "w"), write, pclose.
int run_command_with_input(const std::string& cmd, const std::string& in) {
    std::FILE* p = popen(cmd.c_str(), "w");
    if (!p) {
        std::fprintf(stderr, "incorrect parameters or too many files.\n");
        return EXIT_FAILURE;
    }
    std::fprintf(p, "%s", in.c_str());
    if (std::ferror(p)) {
        std::fprintf(stderr, "Output to stream failed.\n");
        std::exit(EXIT_FAILURE);
    }
    if (pclose(p) != 0) std::fprintf(stderr, "Could not run more or other error.\n");
    return EXIT_SUCCESS;
}

using hgah::PhaseTimer;

using KmerSpecificity = std::map<double, std::map<int, int>>;

// plot_kmer_specificity (src/common/Plotting.cpp:20-37)
std::string plot_wire(const std::map<int, KmerSpecificity>& specs, int max_coverage) {
    std::string ks;
    bool first_k = true;
    for (const auto& k_specs : specs) {
        std::string bounds;
        bool first_b = true;
        for (const auto& bound : k_specs.second) {
            std::string counts;
            bool first_c = true;
            for (const auto& cc : bound.second) {
                if (cc.second < 50) continue;
                counts += (first_c ? "" : ", ") + std::string("(") + std::to_string(cc.first) + ", " +
                          std::to_string(cc.second) + ")";
                first_c = false;
            }
            bounds += (first_b ? "" : ", ") + std::string("(") + hgah::fmt_double(bound.first) + ", [" + counts + "])";
            first_b = false;
        }
        ks += (first_k ? "" : "\n") + std::string("(") + std::to_string(k_specs.first) + ", [" + bounds + "])";
        first_k = false;
    }
    return std::to_string(specs.size()) + " " + std::to_string(max_coverage) + "\n" + ks;
}

}  // namespace

int main(int argc, char* argv[]) {
    std::vector<std::string> read_paths;
    std::string output_path;
    int k = 11;
    hgah::ArgParser ap;
    ap.add("help", 'h', true, "Help screen", nullptr);
    ap.add("read_paths", 0, false, "Path to file with reads (FASTA or FASTQ)",
           [&](const std::string& v) { read_paths.push_back(v); });
    ap.add("k-size", 'k', false, "Size of kmer to analyze & select", [&](const std::string& v) { k = std::stoi(v); });
    ap.add("output", 'o', false, "Output path for the counting bloom filter",
           [&](const std::string& v) { output_path = v; });
    int gpus = 1;
    ap.add("gpus", 0, false, "GPUs to count on, one rank each (MI355X build extension; default 1)",
           [&](const std::string& v) { gpus = std::stoi(v); });
    ap.parse(argc, argv);
    for (auto& p : ap.positional) read_paths.push_back(p);
    if (ap.has("help")) {
        std::cout << ap.describe();
        return 0;
    }
    if (read_paths.empty()) throw std::invalid_argument("You need to specify paths to read files");

    PhaseTimer tm;
    const char* dev_env = std::getenv("HGA_DEVICE");
    // device set-up (HIP init, contexts) on a thread while the files are read, when k is given
    std::unique_ptr<hgah::Ranks> ranks_p;
    std::exception_ptr init_err;
    std::thread init_th([&] {
        try {
            ranks_p = std::make_unique<hgah::Ranks>(gpus, dev_env ? std::atoi(dev_env) : 0);
        } catch (...) {
            init_err = std::current_exception();
        }
    });
    auto join_init = [&] {
        if (init_th.joinable()) init_th.join();
        if (init_err) std::rethrow_exception(init_err);
    };
    if (!ap.has("k-size")) {   // :40-44 — SequenceRecordIterator(read_paths, true) + get_unique_k_length
        const hgah::RecordSet rs = hgah::load_records(read_paths, true, false);
        join_init();
        hga_ctx* c0 = ranks_p->ctx[0];
        check(hga_lookup_set_reads(c0, rs.bases.data(), rs.offsets.data(), rs.size(), 1), "hga_lookup_set_reads");
        k = hgah::unique_k_length(c0, std::cout).first;
    }
    // dump caches (JellyfishOccurrenceReader.cpp:19-24) and the other files' bases
    std::vector<std::vector<uint64_t>> cache_k(read_paths.size());
    std::vector<std::vector<uint32_t>> cache_c(read_paths.size());
    std::vector<hgah::Bytes> streams(read_paths.size());
    std::vector<bool> cached(read_paths.size(), false);
    std::vector<uint32_t> counted;
    for (uint32_t f = 0; f < read_paths.size(); ++f) {
        const std::string cache = hgah::dump_cache_path(read_paths[f], k);
        if (std::filesystem::exists(cache)) {   // the dump's rows enter once, on rank 0
            hgah::read_kmer_dump(cache, k, cache_k[f], cache_c[f]);
            cached[f] = true;
            continue;
        }
        streams[f] = hgah::jf_stream(read_paths[f]);
        counted.push_back(f);
    }
    tm.mark("read_files");
    join_init();
    tm.mark("device_init_wait");
    hgah::Ranks& ranks = *ranks_p;
    hga_ctx* ctx = ranks.ctx[0];
    const int P = ranks.size();
    for (auto* c : ranks.ctx) {
        check(hga_count_begin(c, k, (uint32_t)read_paths.size()), "hga_count_begin");
        // --gpus N: the dumps and the export reach rank 0 only (one writer, one copy in this process,
        // as the reference's single export pass writes them, JellyfishOccurrenceReader.cpp:110-135)
        if (P > 1) check(hga_comm_set_root(c, 0), "hga_comm_set_root");
    }
    for (uint32_t f = 0; f < read_paths.size(); ++f) {
        if (cached[f]) {
            check(hga_count_add_rows(ctx, f, cache_k[f].data(), cache_c[f].data(), cache_k[f].size()),
                  "hga_count_add_rows");
            std::vector<uint64_t>().swap(cache_k[f]);
            std::vector<uint32_t>().swap(cache_c[f]);
            continue;
        }
        const hgah::Bytes& sb = streams[f];
        for (int r = 0; r < P; ++r) {
            const auto [a, b] = hgah::shard_of(sb.data(), sb.size(), r, P);
            check(hga_count_add(ranks.ctx[r], f, sb.data() + a, b - a), "hga_count_add");
        }
        streams[f] = hgah::Bytes();   // freed once uploaded
    }
    tm.mark("upload");
    if (P == 1) {
        check(hga_count_run(ctx, 2), "hga_count_run");   // jellyfish --bc: per-file singletons dropped
        if (tm.on) {   // (the count is asynchronous; the stats wait for it)
            hga_count_stats st;
            check(hga_count_get_stats(ctx, &st), "hga_count_get_stats");
            tm.mark("count");
        }
    } else {
        ranks.each([](int, hga_ctx* c) {
            check(hga_count_run(c, 1), "hga_count_run");   // no drop before the global sum
            check(hga_count_exchange(c, 2), "hga_count_exchange");
        });
    }
    // the dumps come off the device here; they are formatted and written on a thread meanwhile
    struct DumpJob {
        std::string path;
        uint32_t file = 0;
        std::vector<uint64_t*> k;   // one rank's dump of `file` (--gpus N), or null: the merged rows
        std::vector<uint32_t*> c;
        uint64_t n = 0;
    };
    std::vector<DumpJob> dumps;
    uint64_t* all_k = nullptr;   // one GPU: every dump from one fetch of the merged rows
    uint32_t* all_c = nullptr;
    uint64_t all_n = 0;
    const uint32_t F = (uint32_t)read_paths.size();
    const char* cache_env = std::getenv("HGA_DUMP_CACHE");
    if (!(cache_env && std::string(cache_env) == "0") && !counted.empty()) {
        if (P == 1) check(hga_count_rows(ctx, &all_k, &all_c, &all_n), "hga_count_rows");
        for (uint32_t f : counted) {
            DumpJob j;
            j.path = hgah::dump_cache_path(read_paths[f], k);
            j.file = f;
            if (P > 1) {
                j.k.assign(P, nullptr);
                j.c.assign(P, nullptr);
                std::vector<uint64_t> n_d(P, 0);
                ranks.each([&](int r, hga_ctx* c) { check(hga_count_dump(c, f, &j.k[r], &j.c[r], &n_d[r]), "hga_count_dump"); });
                j.n = n_d[0];
            }
            dumps.push_back(std::move(j));
        }
    }
    tm.mark("count_and_dump_fetch");
    std::exception_ptr dump_err;
    std::thread dump_th([&] {
        try {
            for (auto& j : dumps) {
                if (j.k.empty()) hgah::write_kmer_dump_rows(j.path, k, all_k, all_c, F, j.file, all_n);
                else hgah::write_kmer_dump(j.path, k, j.k[0], j.c[0], j.n);
            }
        } catch (...) {
            dump_err = std::current_exception();
        }
    });
    struct DumpJoin {   // joined on every way out of main, the outputs complete before exit
        std::thread& t;
        ~DumpJoin() { if (t.joinable()) t.join(); }
    } dump_join{dump_th};

    const std::set<double> thresholds = {70, 85, 90, 95, 99, 100, 100.01};
    const std::vector<double> thr(thresholds.begin(), thresholds.end());
    std::vector<int64_t*> tris(P, nullptr);
    std::vector<uint64_t> n_tris(P, 0);
    ranks.each([&](int r, hga_ctx* c) {
        check(hga_count_spec_hist(c, thr.data(), (uint32_t)thr.size(), &tris[r], &n_tris[r]), "hga_count_spec_hist");
    });
    for (int r = 1; r < P; ++r) hga_free(tris[r]);
    int64_t* tri = tris[0];
    const uint64_t n_tri = n_tris[0];
    KmerSpecificity spec;
    for (double t : thr) spec.insert({t, {}});
    for (uint64_t i = 0; i < n_tri; ++i)
        spec[thr[(size_t)tri[3 * i]]][(int)tri[3 * i + 1]] += (int)tri[3 * i + 2];
    hga_free(tri);
    std::map<int, KmerSpecificity> spec_map = {{k, spec}};
    tm.mark("spec_hist");
    const char* plot_env = std::getenv("HGA_PLOT_CMD");
    const std::string plot_cmd = plot_env ? plot_env : "python scripts/plotting.py --plot kmer_histogram_with_spec";
    std::cout << run_command_with_input(plot_cmd, plot_wire(spec_map, 200)) << std::endl;
    tm.mark("plot");

    int lower = 0, upper = 0;
    double percent = 0;
    std::cout << "Enter lower and upper bounds for exported kmers as well as percentage\n";
    std::cin >> lower >> upper >> percent;
    tm.mark("prompt");
    if (output_path.empty())
        output_path = std::to_string(k) + "-mers_" + std::to_string(lower) + "_" + std::to_string(upper) + "_" +
                      hgah::fmt_double(percent * 100) + "%.txt";

    // export_kmers (JellyfishOccurrenceReader.cpp:110-135)
    std::vector<uint64_t*> keys_r(P, nullptr);
    std::vector<uint8_t*> disc_r(P, nullptr);
    std::vector<uint64_t> n_r(P, 0), nd_r(P, 0);
    ranks.each([&](int r, hga_ctx* c) {
        check(hga_count_select_ex(c, lower, upper, &keys_r[r], &disc_r[r], &n_r[r], &nd_r[r]), "hga_count_select_ex");
    });
    for (int r = 1; r < P; ++r) {
        hga_free(keys_r[r]);
        hga_free(disc_r[r]);
    }
    uint64_t* keys = keys_r[0];
    uint8_t* disc = disc_r[0];
    const uint64_t n = n_r[0];
    std::random_device dev;
    std::mt19937 rng(dev());
    std::uniform_real_distribution<> dis(0.0, 1.0);
    std::FILE* out = std::fopen(output_path.c_str(), "wb");
    if (!out) throw std::runtime_error("cannot open " + output_path);
    std::vector<char> buf;
    buf.reserve(1 << 20);
    uint32_t exported = 0, discriminative = 0;
    std::vector<char> line((size_t)k + 1, '\n');
    for (uint64_t i = 0; i < n; ++i) {
        if (!(dis(rng) < percent)) continue;
        hgah::kmer_to_chars(keys[i], k, line.data());
        buf.insert(buf.end(), line.begin(), line.end());
        if (buf.size() > (1u << 20)) { std::fwrite(buf.data(), 1, buf.size(), out); buf.clear(); }
        ++exported;
        discriminative += disc[i] ? 1u : 0u;
    }
    std::fwrite(buf.data(), 1, buf.size(), out);
    std::fclose(out);
    hga_free(keys);
    hga_free(disc);
    tm.mark("select_and_export");
    std::cout << discriminative << " out of " << exported << " exported kmers are discriminative";
    std::cout.flush();
    dump_th.join();
    for (auto& j : dumps)
        for (size_t r = 0; r < j.k.size(); ++r) {
            hga_free(j.k[r]);
            hga_free(j.c[r]);
        }
    hga_free(all_k);
    hga_free(all_c);
    tm.mark("dump_write_wait");
    tm.total();
    if (dump_err) std::rethrow_exception(dump_err);
    // Every output is written and closed: leave without the orderly teardown (freeing each device
    // buffer, the HIP runtime's exit) — the OS reclaims the process and its device memory, and the
    // teardown was about a quarter of the CLI's wall time.  HGA_CLI_FULL_EXIT=1 keeps it.
    const char* full = std::getenv("HGA_CLI_FULL_EXIT");
    if (!(full && std::string(full) == "1")) {
        std::cout.flush();
        std::fflush(nullptr);
        std::_Exit(0);
    }
    return 0;
}
