// gen.h — seeded synthetic inputs standing in for the reference's read simulators
// (src/scripts/read_generator.py drives art_illumina / nanosim-h, neither of which is
// available here).  Deterministic for a given seed, independent of thread count.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace hgah {

struct Rng {   // xoshiro256**, seeded through splitmix64
    uint64_t s[4];
    explicit Rng(uint64_t seed);
    uint64_t next();
    double uniform() { return (next() >> 11) * 0x1.0p-53; }
    uint64_t below(uint64_t n) { return n ? next() % n : 0; }
};
uint64_t mix_seed(uint64_t a, uint64_t b);

// i.i.d. uniform ACGT genome.
std::string gen_genome(uint64_t len, uint64_t seed);
// Per-base substitution with probability d by one of the other three bases
// (read_generator.py:158-162), then `extra` random bases inserted as 10 kb blocks.
std::string gen_haplotype(const std::string& src, double d, uint64_t extra, uint64_t seed);

struct ReadBatch {
    std::string seq;                 // sequences joined by '\n'
    std::vector<uint64_t> offsets;   // CSR over the sequences (without separators)
    std::vector<char> bases;         // concatenated sequences (no separators)
    std::vector<std::string> headers;
    std::vector<std::string> quals;
};

// ART-like short reads (stand-in for `art_illumina -ss HS25 -l 150 -f C -na`,
// read_generator.py:58): uniform start, strand 50/50, substitution rate rising from
// 0.1 % to 0.3 % along the read.  Header "<name>-<n>".
ReadBatch gen_art(const std::string& genome, const std::string& name, uint64_t n_reads, int read_len,
                  uint64_t seed, bool with_text);
// Nanosim-H-like long reads (read_generator.py:135-138): log-normal lengths (mean
// ~7.8 kb, clipped to [85, 59500]), ~10 % errors (sub:ins:del 1:1:1), header
// "<ref>_<start>_aligned_<idx>_<F|R>_0_<len>_0" so the nanosim-h regex parses.
ReadBatch gen_nanosim(const std::string& genome, const std::string& name, uint64_t n_reads, uint64_t seed,
                      bool with_text);

}  // namespace hgah
