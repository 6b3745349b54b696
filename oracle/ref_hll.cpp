// ref_hll.cpp — TEST INFRASTRUCTURE ONLY (oracle/_ref; imported by tests/ and nothing else).
//
// A thin C-ABI driver around the reference's OWN HyperLogLog and MurmurHash3 code, compiled
// unmodified from where it lies in the reference tree (recipe: oracle/Makefile, target `ref`):
//   src/lib/HyperLogLog.hpp   hll::HyperLogLog — add :96-107, estimate :113-132, dump :192-198
//   src/lib/MurmurHash3.cpp   MurmurHash3_x86_32 :94-140
// Fed canonical k-mer codes the way approximate_kmer_count_thread does
// (src/occurrences/KmerAnalysis.cpp:15-23: hyper.add((void*)&it.current_kmer, sizeof(Kmer))),
// so the HyperLogLog auto-k row is pinned against the reference itself,
// not only against a restatement.  The k-mer codes come from the oracle's KmerIterator
// restatement (KmerIterator.cpp cannot be built here: it needs Boost, which is absent).
// Registers are read through the public dump() API (one byte b, then the m registers).
#include <cstdint>
#include <cstring>
#include <mutex>     // HyperLogLog.hpp uses std::mutex without including <mutex> itself
#include <sstream>
#include <string>

#include "HyperLogLog.hpp"
#include "MurmurHash3.h"

extern "C" {

// Registers (2^b bytes into regs) and estimate() of HyperLogLog(b) after add() of every code.
int ref_hll_registers(const uint64_t* codes, uint64_t n, int b, uint8_t* regs, double* estimate) {
    try {
        hll::HyperLogLog h((uint8_t)b);
        for (uint64_t i = 0; i < n; ++i) h.add((const void*)&codes[i], sizeof(uint64_t));
        std::ostringstream os;
        h.dump(os);
        const std::string s = os.str();
        if (s.size() != 1 + ((size_t)1 << b)) return -2;
        std::memcpy(regs, s.data() + 1, (size_t)1 << b);
        *estimate = h.estimate();
        return 0;
    } catch (...) {
        return -1;
    }
}

uint32_t ref_murmur3_x86_32(const void* key, int len, uint32_t seed) {
    uint32_t out = 0;
    MurmurHash3_x86_32(key, len, seed, &out);
    return out;
}

}  // extern "C"
