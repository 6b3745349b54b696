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
// HGA_DEVICE selects the GPU (default 0); HGA_PLOT_CMD overrides the plot command.
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
#include <random>
#include <set>
#include <stdexcept>
#include <string>
#include <vector>

#include "args.h"
#include "hga.h"
#include "kmer_analysis.h"
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

    const char* dev_env = std::getenv("HGA_DEVICE");
    hgah::Ranks ranks(gpus, dev_env ? std::atoi(dev_env) : 0);
    hga_ctx* ctx = ranks.ctx[0];
    const int P = ranks.size();
    if (!ap.has("k-size")) {   // :40-44 — SequenceRecordIterator(read_paths, true) + get_unique_k_length
        const hgah::RecordSet rs = hgah::load_records(read_paths, true, false);
        check(hga_lookup_set_reads(ctx, rs.bases.data(), rs.offsets.data(), rs.size(), 1), "hga_lookup_set_reads");
        k = hgah::unique_k_length(ctx, std::cout).first;
    }
    for (auto* c : ranks.ctx) check(hga_count_begin(c, k, (uint32_t)read_paths.size()), "hga_count_begin");
    std::vector<uint32_t> counted;
    for (uint32_t f = 0; f < read_paths.size(); ++f) {
        const std::string cache = hgah::dump_cache_path(read_paths[f], k);
        if (std::filesystem::exists(cache)) {   // the dump's rows enter once, on rank 0
            std::vector<uint64_t> dk;
            std::vector<uint32_t> dc;
            hgah::read_kmer_dump(cache, k, dk, dc);
            check(hga_count_add_rows(ctx, f, dk.data(), dc.data(), dk.size()), "hga_count_add_rows");
            continue;
        }
        const hgah::Bytes s = hgah::jf_stream(read_paths[f]);
        for (int r = 0; r < P; ++r) {
            const auto [a, b] = hgah::shard_of(s.data(), s.size(), r, P);
            check(hga_count_add(ranks.ctx[r], f, s.data() + a, b - a), "hga_count_add");
        }
        counted.push_back(f);
    }
    if (P == 1) {
        check(hga_count_run(ctx, 2), "hga_count_run");   // jellyfish --bc: per-file singletons dropped
    } else {
        ranks.each([](int, hga_ctx* c) {
            check(hga_count_run(c, 1), "hga_count_run");   // no drop before the global sum
            check(hga_count_exchange(c, 2), "hga_count_exchange");
        });
    }
    const char* cache_env = std::getenv("HGA_DUMP_CACHE");
    if (!(cache_env && std::string(cache_env) == "0"))
        for (uint32_t f : counted) {
            std::vector<uint64_t*> dk(P, nullptr);
            std::vector<uint32_t*> dc(P, nullptr);
            std::vector<uint64_t> n_d(P, 0);
            ranks.each([&](int r, hga_ctx* c) { check(hga_count_dump(c, f, &dk[r], &dc[r], &n_d[r]), "hga_count_dump"); });
            hgah::write_kmer_dump(hgah::dump_cache_path(read_paths[f], k), k, dk[0], dc[0], n_d[0]);
            for (int r = 0; r < P; ++r) {
                hga_free(dk[r]);
                hga_free(dc[r]);
            }
        }

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
    const char* plot_env = std::getenv("HGA_PLOT_CMD");
    const std::string plot_cmd = plot_env ? plot_env : "python scripts/plotting.py --plot kmer_histogram_with_spec";
    std::cout << run_command_with_input(plot_cmd, plot_wire(spec_map, 200)) << std::endl;

    int lower = 0, upper = 0;
    double percent = 0;
    std::cout << "Enter lower and upper bounds for exported kmers as well as percentage\n";
    std::cin >> lower >> upper >> percent;
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
    std::cout << discriminative << " out of " << exported << " exported kmers are discriminative";
    std::cout.flush();
    return 0;
}
