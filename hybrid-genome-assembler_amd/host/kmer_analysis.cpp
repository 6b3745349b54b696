// kmer_analysis.cpp — see kmer_analysis.h.
#include "kmer_analysis.h"

#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

namespace hgah {

uint64_t approximate_kmer_count(hga_ctx* ctx, int k) {
    std::vector<uint8_t> regs(1u << 10);
    if (hga_hll_registers(ctx, k, 10, regs.data()) != HGA_OK)
        throw std::runtime_error(std::string("hga_hll_registers: ") + hga_last_error());
    return (uint64_t)hll_estimate(regs.data(), 10);
}

std::pair<int, uint64_t> unique_k_length(hga_ctx* ctx, std::ostream& out) {
    int k = 11;
    long long previous_count = (long long)approximate_kmer_count(ctx, k);
    out << "k=11 : ~" << previous_count << " kmers" << std::endl;
    while (k < 33) {
        const long long count = (long long)approximate_kmer_count(ctx, k + 2);
        out << "k=" << k + 2 << " : ~" << count << " kmers" << std::endl;
        if (((double)std::llabs(count - previous_count) / ((double)(count + previous_count) / 2.0)) < 0.1)
            return {k, (uint64_t)previous_count};
        k += 2;
        previous_count = count;
    }
    return {k, (uint64_t)previous_count};
}

}  // namespace hgah
