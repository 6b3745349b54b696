// host_api.cpp — C ABI of libhga_host.so: the host-side readers and the synthetic
// generators, for the Python test / bench plumbing (ctypes).  Buffers returned through
// out-pointers are malloc'ed; release them with hgh_free.
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "gen.h"
#include "kmer_analysis.h"
#include "seqio.h"

namespace {
thread_local std::string g_err;

template <class T>
T* dup(const T* p, size_t n) {
    T* q = static_cast<T*>(std::malloc(n ? n * sizeof(T) : 1));
    if (n) std::memcpy(q, p, n * sizeof(T));
    return q;
}

template <class F>
int guard(F&& f) {
    try {
        g_err.clear();
        f();
        return 0;
    } catch (const std::exception& e) {
        g_err = e.what();
        return 1;
    }
}

void export_batch(const hgah::ReadBatch& b, char** seq, uint64_t* seq_len, char** bases, uint64_t** offsets,
                  uint64_t* n_reads) {
    if (seq) { *seq = dup(b.seq.data(), b.seq.size()); *seq_len = b.seq.size(); }
    if (bases) *bases = dup(b.bases.data(), b.bases.size());
    if (offsets) *offsets = dup(b.offsets.data(), b.offsets.size());
    *n_reads = b.offsets.size() - 1;
}
}  // namespace

extern "C" {

const char* hgh_last_error(void) { return g_err.c_str(); }

// The dump cache writer of jf_occurrences (seqio.cpp write_kmer_dump), for the tests.
int hgh_write_kmer_dump(const char* path, int k, const uint64_t* keys, const uint32_t* counts, uint64_t n) {
    return guard([&] { hgah::write_kmer_dump(path, k, keys, counts, n); });
}
void hgh_free(void* p) { std::free(p); }

int hgh_gen_genome(uint64_t len, uint64_t seed, char** out) {
    return guard([&] {
        std::string g = hgah::gen_genome(len, seed);
        *out = dup(g.data(), g.size());
    });
}

int hgh_gen_haplotype(const char* src, uint64_t len, double d, uint64_t extra, uint64_t seed, char** out,
                      uint64_t* out_len) {
    return guard([&] {
        std::string h = hgah::gen_haplotype(std::string(src, len), d, extra, seed);
        *out = dup(h.data(), h.size());
        *out_len = h.size();
    });
}

// Reads as a '\n'-joined stream (seq) and/or CSR (bases, offsets); any out may be null.
int hgh_gen_art(const char* genome, uint64_t glen, uint64_t n_reads, int read_len, uint64_t seed, char** seq,
                uint64_t* seq_len, char** bases, uint64_t** offsets, uint64_t* n_out) {
    return guard([&] {
        auto b = hgah::gen_art(std::string(genome, glen), "r", n_reads, read_len, seed, false);
        export_batch(b, seq, seq_len, bases, offsets, n_out);
    });
}

int hgh_gen_nanosim(const char* genome, uint64_t glen, uint64_t n_reads, uint64_t seed, char** seq,
                    uint64_t* seq_len, char** bases, uint64_t** offsets, uint64_t* n_out) {
    return guard([&] {
        auto b = hgah::gen_nanosim(std::string(genome, glen), "r", n_reads, seed, false);
        export_batch(b, seq, seq_len, bases, offsets, n_out);
    });
}

// Writes FASTQ (ART-like) or single-line FASTA (Nanosim-like) files.
int hgh_write_art_fastq(const char* genome, uint64_t glen, const char* name, uint64_t n_reads, int read_len,
                        uint64_t seed, const char* path) {
    return guard([&] {
        auto b = hgah::gen_art(std::string(genome, glen), name, n_reads, read_len, seed, true);
        std::FILE* f = std::fopen(path, "wb");
        if (!f) throw std::runtime_error(std::string("cannot write ") + path);
        for (size_t i = 0; i + 1 < b.offsets.size(); ++i) {
            std::fprintf(f, "@%s\n", b.headers[i].c_str());
            std::fwrite(b.bases.data() + b.offsets[i], 1, b.offsets[i + 1] - b.offsets[i], f);
            std::fprintf(f, "\n+\n%s\n", b.quals[i].c_str());
        }
        std::fclose(f);
    });
}

int hgh_write_nanosim_fasta(const char* genome, uint64_t glen, const char* name, uint64_t n_reads,
                            uint64_t seed, const char* path) {
    return guard([&] {
        auto b = hgah::gen_nanosim(std::string(genome, glen), name, n_reads, seed, true);
        std::FILE* f = std::fopen(path, "wb");
        if (!f) throw std::runtime_error(std::string("cannot write ") + path);
        for (size_t i = 0; i + 1 < b.offsets.size(); ++i) {
            std::fprintf(f, ">%s\n", b.headers[i].c_str());
            std::fwrite(b.bases.data() + b.offsets[i], 1, b.offsets[i + 1] - b.offsets[i], f);
            std::fputc('\n', f);
        }
        std::fclose(f);
    });
}

// SequenceRecordIterator-semantics load.  meta_out: [files+1][5] u64
// (records, total_bases, min, max, avg); file 0..n-1 then the all-files meta.
int hgh_load_records(const char** paths, int n_paths, int annotate, char** bases, uint64_t** offsets,
                     int32_t** category, uint32_t** start, uint32_t** end, uint64_t* n_reads,
                     uint64_t** meta_out, char** filename_out) {
    return guard([&] {
        std::vector<std::string> p(paths, paths + n_paths);
        auto rs = hgah::load_records(p, annotate != 0, false);
        *bases = dup(rs.bases.data(), rs.bases.size());
        *offsets = dup(rs.offsets.data(), rs.offsets.size());
        *category = dup(rs.category.data(), rs.category.size());
        *start = dup(rs.start.data(), rs.start.size());
        *end = dup(rs.end.data(), rs.end.size());
        *n_reads = rs.size();
        std::vector<uint64_t> m;
        auto put = [&](const hgah::FileMeta& x) {
            m.push_back(x.records); m.push_back(x.total_bases); m.push_back(x.min_read_length);
            m.push_back(x.max_read_length); m.push_back(x.avg_read_length);
        };
        for (auto& x : rs.file_meta) put(x);
        put(rs.meta);
        *meta_out = dup(m.data(), m.size());
        std::string fn = rs.meta.filename;
        *filename_out = dup(fn.c_str(), fn.size() + 1);
    });
}

int hgh_jf_stream(const char* path, char** out, uint64_t* len, uint64_t* n_records) {
    return guard([&] {
        const hgah::Bytes s = hgah::jf_stream(path, n_records);
        *out = dup(s.data(), s.size());
        *len = s.size();
    });
}

int hgh_fmt_double(double v, char* buf, int cap) {
    std::string s = hgah::fmt_double(v);
    if ((int)s.size() + 1 > cap) return -1;
    std::memcpy(buf, s.c_str(), s.size() + 1);
    return (int)s.size();
}

// Reader threads of load_records / jf_stream (1 = the sequential readers).
void hgh_set_threads(int n) { hgah::set_host_threads(n); }

// load_text_file_kmers (read_clustering.cpp:18-33): canonical codes in KmerID order, k.
int hgh_load_kmer_text(const char* path, uint64_t** keys, uint64_t* n, int* k) {
    return guard([&] {
        const std::vector<uint64_t> v = hgah::load_kmer_text(path, k);
        *keys = dup(v.data(), v.size());
        *n = v.size();
    });
}

// The iteration order of a std::unordered_set<uint64_t> filled with keys[0..n) in order.
int hgh_unordered_set_order(const uint64_t* keys, uint64_t n, uint64_t** out, uint64_t* m) {
    return guard([&] {
        const std::vector<uint64_t> v = hgah::unordered_set_order(keys, n);
        *out = dup(v.data(), v.size());
        *m = v.size();
    });
}

// hll::HyperLogLog::estimate of 2^b registers (kmer_analysis.h).
double hgh_hll_estimate(const uint8_t* regs, int b) { return hgah::hll_estimate(regs, b); }

}  // extern "C"
