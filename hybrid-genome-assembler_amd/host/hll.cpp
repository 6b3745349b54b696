// hll.cpp — hll::HyperLogLog::estimate on the host (src/lib/HyperLogLog.hpp:66-87, 113-132);
// the registers come from the GPU (hga_hll_registers).
#include <cmath>
#include <cstdint>

#include "kmer_analysis.h"

namespace hgah {

double hll_estimate(const uint8_t* regs, int b) {
    const uint32_t m = 1u << b;
    double alpha;   // HyperLogLog.hpp:70-84
    switch (m) {
        case 16: alpha = 0.673; break;
        case 32: alpha = 0.697; break;
        case 64: alpha = 0.709; break;
        default: alpha = 0.7213 / (1.0 + 1.079 / m); break;
    }
    const double alphaMM = alpha * m * m;
    double sum = 0.0;
    for (uint32_t i = 0; i < m; i++) sum += 1.0 / (1 << regs[i]);
    double estimate = alphaMM / sum;
    if (estimate <= 2.5 * m) {
        uint32_t zeros = 0;
        for (uint32_t i = 0; i < m; i++) zeros += regs[i] == 0;
        if (zeros != 0) estimate = m * std::log(static_cast<double>(m) / zeros);
    } else if (estimate > (1.0 / 30.0) * 4294967296.0) {
        estimate = -4294967296.0 * std::log(1.0 - (estimate / 4294967296.0));
    }
    return estimate;
}

}  // namespace hgah
