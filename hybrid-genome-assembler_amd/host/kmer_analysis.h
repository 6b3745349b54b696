// kmer_analysis.h — automatic k selection of jf_occurrences (src/occurrences/KmerAnalysis.cpp:26-56),
// with the HyperLogLog registers filled on the GPU (hga_hll_registers) and the estimate computed
// on the host exactly as hll::HyperLogLog::estimate (src/lib/HyperLogLog.hpp:113-132).
#pragma once

#include <cstdint>
#include <ostream>
#include <utility>

#include "hga.h"

namespace hgah {

// hll::HyperLogLog::estimate over 2^b registers (HyperLogLog.hpp:66-87 alpha, :113-132).
double hll_estimate(const uint8_t* regs, int b);

// get_approximate_kmer_count (KmerAnalysis.cpp:26-38): HyperLogLog(10) over every KmerIterator
// window of the reads set on ctx; the double estimate converted to uint64_t like the reference's
// return statement.  Throws std::runtime_error with hga_last_error() on failure.
uint64_t approximate_kmer_count(hga_ctx* ctx, int k);

// get_unique_k_length (KmerAnalysis.cpp:41-56): k = 11, 13, ... until two consecutive
// estimates differ by < 10 % of their mean; prints "k=<k> : ~<count> kmers" per estimate.
// Returns {k, count} of the smaller k of the converged pair.
std::pair<int, uint64_t> unique_k_length(hga_ctx* ctx, std::ostream& out);

}  // namespace hgah
