// Offline false-positive study of lk_scan's minimizer-blocked filter (lookup.hip), on the host with the
// kernel's own hash functions: the SDK keys build the filter, every valid ACGT window of the reads is
// queried, and the queries that pass but are not SDK keys are the false positives (each costs one
// table-bucket probe in lk_scan).  Schemes: 0 = the kernel's (one 32-bit word of the 16-B block picked by
// 2 hash bits, 3 bits in it); B = B bits anywhere in the 128-bit block (the lane loads the whole block
// anyway).  usage: sim <sdk.u64> <bases.txt> <offsets.u64> <k> <filter_words_log2> [schemes...]
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iterator>
#include <unordered_set>
#include <vector>

static std::vector<char> slurp(const char* p) {
    std::ifstream f(p, std::ios::binary);
    return std::vector<char>(std::istreambuf_iterator<char>(f), {});
}
static uint64_t revcomp(uint64_t x, int m) {   // reverse complement of an m-base code
    uint64_t y = 0;
    for (int i = 0; i < m; ++i) {
        y = (y << 2) | (3 - (x & 3));
        x >>= 2;
    }
    return y;
}
static uint32_t mmer_hash(uint64_t c) { return (uint32_t)((c * 0x9E3779B97F4A7C15ull) >> 32); }
static uint32_t end_mix(uint32_t e) { return (e ^ (e >> 16)) * 0x9E3779B1u; }
static int code(char c) { return c == 'A' ? 0 : c == 'C' ? 1 : c == 'G' ? 2 : c == 'T' ? 3 : -1; }

struct Q { uint32_t minh, x; };
static Q key_q(uint64_t key, int k, int km) {   // build side: lookup.hip key_minimizer + end_mix
    const int m = k - km;
    const uint64_t mm = (1ull << (2 * m)) - 1;
    uint32_t best = ~0u, e = 0;
    for (int i = 0; i <= km; ++i) {
        const uint64_t fm = (key >> (2 * (km - i))) & mm, rm = revcomp(fm, m);
        const uint32_t hh = mmer_hash(fm < rm ? fm : rm);
        best = std::min(best, hh);
        if (i == 0 || i == km) e ^= hh;
    }
    return {best, end_mix(e)};
}
// bit positions of scheme s for hash x (s = 0: the kernel's word + 3 bits)
static void bits_of(int s, uint32_t x, uint32_t b[4]) {
    b[0] = b[1] = b[2] = b[3] = 0;
    if (s == 0) {
        const uint32_t w = x >> 30;
        for (int i = 0; i < 3; ++i) b[w] |= 1u << ((x >> (25 - 5 * i)) & 31);
        return;
    }
    uint32_t y = x, z = x * 0x85EBCA6Bu ^ (x >> 13);
    if (s >= 100) {   // partitioned: (s - 100) bits in EVERY word (5-bit fields of x, then of z)
        const int per = s - 100;
        for (int w = 0; w < 4; ++w)
            for (int i = 0; i < per; ++i) {
                const int f = w * per + i;
                const uint32_t v = f < 6 ? (y >> (27 - 5 * f)) & 31 : (z >> (27 - 5 * (f - 6))) & 31;
                b[w] |= 1u << v;
            }
        return;
    }
    for (int i = 0; i < s; ++i) {
        const uint32_t v = i < 4 ? (y >> (25 - 7 * i)) & 127 : (z >> (25 - 7 * (i - 4))) & 127;
        b[v >> 5] |= 1u << (v & 31);
    }
}

int main(int argc, char** argv) {
    if (argc < 6) return 2;
    const auto sk = slurp(argv[1]), bases = slurp(argv[2]), ob = slurp(argv[3]);
    const uint64_t* keys = reinterpret_cast<const uint64_t*>(sk.data());
    const size_t nk = sk.size() / 8;
    const uint64_t* off = reinterpret_cast<const uint64_t*>(ob.data());
    const size_t nr = ob.size() / 8 - 1;
    const int k = atoi(argv[4]), fl2 = atoi(argv[5]);
    const int km = k >= 18 ? 7 : (k >= 15 ? k - 11 : 0);
    const uint64_t nblk = (1ull << fl2) / 4;
    std::vector<int> schemes;
    for (int i = 6; i < argc; ++i) schemes.push_back(atoi(argv[i]));
    if (schemes.empty()) schemes = {0, 4, 5, 6};
    std::unordered_set<uint64_t> set(keys, keys + nk);
    std::vector<uint32_t> load(nblk, 0);
    std::vector<std::vector<uint32_t>> filt(schemes.size(), std::vector<uint32_t>(nblk * 4, 0));
    for (size_t i = 0; i < nk; ++i) {
        const Q q = key_q(keys[i], k, km);
        const uint64_t bi = q.minh & (nblk - 1);
        ++load[bi];
        for (size_t s = 0; s < schemes.size(); ++s) {
            uint32_t b[4];
            bits_of(schemes[s], q.x, b);
            for (int w = 0; w < 4; ++w) filt[s][bi * 4 + w] |= b[w];
        }
    }
    std::vector<uint64_t> pass(schemes.size(), 0);
    uint64_t windows = 0, hits = 0, runs = 0;
    std::vector<uint64_t> qload_hist(64, 0);
    const int m = k - km;
    const uint64_t mm = (1ull << (2 * m)) - 1, kmask = (1ull << (2 * k)) - 1;
    for (size_t r = 0; r < nr; ++r) {
        const char* s = bases.data() + off[r];
        const size_t L = off[r + 1] - off[r];
        if (L < (size_t)k) continue;
        std::vector<uint32_t> mh(L, 0);   // canonical m-mer hash ending at base i (i >= m-1)
        uint64_t fw = 0, rc = 0;
        int valid = 0;
        std::vector<int> okm(L, 0);
        for (size_t i = 0; i < L; ++i) {
            const int c = code(s[i]);
            if (c < 0) { valid = 0; fw = rc = 0; continue; }
            fw = ((fw << 2) | (uint64_t)c) & kmask;
            ++valid;
            if (valid >= m) {
                const uint64_t f2 = fw & mm, r2 = revcomp(f2, m);
                mh[i] = mmer_hash(f2 < r2 ? f2 : r2);
                okm[i] = 1;
            }
            if (valid >= k) {
                uint32_t mn = ~0u;
                for (int t = 0; t <= km; ++t) mn = std::min(mn, mh[i - t]);
                const uint32_t x = end_mix(mh[i] ^ mh[i - km]);
                const uint64_t canon = std::min(fw, revcomp(fw, k));
                const uint64_t bi = mn & (nblk - 1);
                ++windows;
                const bool hit = set.count(canon) != 0;
                hits += hit;
                qload_hist[std::min<uint32_t>(load[bi], 63)]++;
                for (size_t sc = 0; sc < schemes.size(); ++sc) {
                    uint32_t b[4];
                    bits_of(schemes[sc], x, b);
                    bool p = true;
                    for (int w = 0; w < 4; ++w) p = p && (filt[sc][bi * 4 + w] & b[w]) == b[w];
                    if (p && !hit) ++pass[sc];
                }
            }
        }
    }
    std::printf("keys %zu reads %zu windows %llu hits %llu blocks %llu (%.2f keys/block)\n", nk, nr,
                (unsigned long long)windows, (unsigned long long)hits, (unsigned long long)nblk, (double)nk / nblk);
    for (size_t s = 0; s < schemes.size(); ++s)
        std::printf("scheme %d: false positives %llu (%.3f%% of non-hit windows, %.2f per hit)\n", schemes[s],
                    (unsigned long long)pass[s], 100.0 * pass[s] / (windows - hits), (double)pass[s] / hits);
    std::printf("queried block load (keys in the block of a window's minimizer):");
    for (int i = 0; i < 64; ++i)
        if (qload_hist[i]) std::printf(" %d:%.4f", i, (double)qload_hist[i] / windows);
    std::printf("\n");
    return 0;
}
