// hga_gen — writes the seeded synthetic datasets of SURVEY.md §8(d) as read files.
//   hga_gen art     <out_prefix> <genome_len> <divergence> <coverage> <seed> [read_len]
//       -> <prefix>_A.fq, <prefix>_B.fq   (ART-like, 2 haplotypes)
//   hga_gen nanosim <out_prefix> <genome_len> <divergence> <coverage> <seed>
//       -> <prefix>_A.fa, <prefix>_B.fa   (Nanosim-H-like)
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "gen.h"

extern "C" int hgh_write_art_fastq(const char*, uint64_t, const char*, uint64_t, int, uint64_t, const char*);
extern "C" int hgh_write_nanosim_fasta(const char*, uint64_t, const char*, uint64_t, uint64_t, const char*);
extern "C" const char* hgh_last_error(void);

int main(int argc, char** argv) {
    if (argc < 7) {
        std::fprintf(stderr, "usage: %s art|nanosim <prefix> <genome_len> <divergence> <coverage> <seed> [read_len]\n",
                     argv[0]);
        return 2;
    }
    const std::string mode = argv[1], prefix = argv[2];
    const uint64_t L = std::strtoull(argv[3], nullptr, 10);
    const double d = std::atof(argv[4]), cov = std::atof(argv[5]);
    const uint64_t seed = std::strtoull(argv[6], nullptr, 10);
    const int rl = argc > 7 ? std::atoi(argv[7]) : 150;
    const std::string A = hgah::gen_genome(L, seed);
    const std::string B = hgah::gen_haplotype(A, d, 0, seed + 1);
    int rc = 0;
    if (mode == "art") {
        const uint64_t n = (uint64_t)(cov * (double)L / rl);
        rc |= hgh_write_art_fastq(A.data(), A.size(), "hapA", n, rl, seed + 10, (prefix + "_A.fq").c_str());
        rc |= hgh_write_art_fastq(B.data(), B.size(), "hapB", n, rl, seed + 11, (prefix + "_B.fq").c_str());
    } else if (mode == "nanosim") {
        const uint64_t n = (uint64_t)std::llround((double)L / 7777.0 * cov);
        rc |= hgh_write_nanosim_fasta(A.data(), A.size(), "hapA", n, seed + 10, (prefix + "_A.fa").c_str());
        rc |= hgh_write_nanosim_fasta(B.data(), B.size(), "hapB", n, seed + 11, (prefix + "_B.fa").c_str());
    } else {
        std::fprintf(stderr, "unknown mode %s\n", mode.c_str());
        return 2;
    }
    if (rc) std::fprintf(stderr, "hga_gen: %s\n", hgh_last_error());
    return rc;
}
