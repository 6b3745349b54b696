// gen.cpp — see gen.h.
#include "gen.h"

#include <algorithm>
#include <cmath>
#include <thread>

namespace hgah {

static inline uint64_t splitmix(uint64_t& x) {
    uint64_t z = (x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

Rng::Rng(uint64_t seed) {
    uint64_t x = seed;
    for (auto& v : s) v = splitmix(x);
}

uint64_t Rng::next() {
    auto rotl = [](uint64_t x, int k) { return (x << k) | (x >> (64 - k)); };
    const uint64_t r = rotl(s[1] * 5, 7) * 9;
    const uint64_t t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl(s[3], 45);
    return r;
}

uint64_t mix_seed(uint64_t a, uint64_t b) {
    uint64_t x = a ^ (b * 0xD1B54A32D192ED03ull);
    return splitmix(x);
}

static const char kB[4] = {'A', 'C', 'G', 'T'};

static inline char comp(char c) {
    switch (c) {
        case 'A': return 'T';
        case 'C': return 'G';
        case 'G': return 'C';
        case 'T': return 'A';
        default: return 'N';
    }
}

std::string gen_genome(uint64_t len, uint64_t seed) {
    Rng r(mix_seed(seed, 1));
    std::string g(len, 'A');
    uint64_t i = 0;
    while (i < len) {
        uint64_t w = r.next();
        for (int j = 0; j < 32 && i < len; ++j, ++i, w >>= 2) g[i] = kB[w & 3];
    }
    return g;
}

std::string gen_haplotype(const std::string& src, double d, uint64_t extra, uint64_t seed) {
    Rng r(mix_seed(seed, 2));
    std::string h = src;
    for (auto& c : h)
        if (r.uniform() < d) {
            const int cur = c == 'A' ? 0 : c == 'C' ? 1 : c == 'G' ? 2 : 3;
            c = kB[(cur + 1 + (int)r.below(3)) & 3];
        }
    uint64_t left = extra;
    while (left) {
        const uint64_t blk = std::min<uint64_t>(left, 10000);
        const uint64_t at = r.below(h.size() + 1);
        std::string ins(blk, 'A');
        for (auto& c : ins) c = kB[r.next() & 3];
        h.insert(at, ins);
        left -= blk;
    }
    return h;
}

namespace {

constexpr uint64_t CHUNK = 4096;   // reads per independently seeded chunk

template <class F>
void parallel_chunks(uint64_t n_chunks, F&& f) {
    unsigned nt = std::max(1u, std::min<unsigned>(std::thread::hardware_concurrency(), 16u));
    nt = (unsigned)std::min<uint64_t>(nt, std::max<uint64_t>(n_chunks, 1));
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            for (uint64_t c = t; c < n_chunks; c += nt) f(c);
        });
    for (auto& x : th) x.join();
}

struct Piece {
    std::string seq;
    std::vector<uint32_t> lens;
    std::vector<std::string> headers, quals;
};

ReadBatch assemble(std::vector<Piece>& pieces, bool with_text) {
    ReadBatch b;
    size_t total = 0, nr = 0;
    for (auto& p : pieces) { total += p.seq.size(); nr += p.lens.size(); }
    b.bases.reserve(total);
    b.offsets.reserve(nr + 1);
    b.offsets.push_back(0);
    b.seq.reserve(total + nr);
    for (auto& p : pieces) {
        size_t o = 0;
        for (size_t i = 0; i < p.lens.size(); ++i) {
            if (b.offsets.size() > 1) b.seq.push_back('\n');
            b.seq.append(p.seq, o, p.lens[i]);
            b.bases.insert(b.bases.end(), p.seq.begin() + o, p.seq.begin() + o + p.lens[i]);
            b.offsets.push_back(b.bases.size());
            o += p.lens[i];
        }
        if (with_text) {
            for (auto& h : p.headers) b.headers.push_back(std::move(h));
            for (auto& q : p.quals) b.quals.push_back(std::move(q));
        }
        Piece().seq.swap(p.seq);
    }
    return b;
}

}  // namespace

ReadBatch gen_art(const std::string& genome, const std::string& name, uint64_t n_reads, int read_len,
                  uint64_t seed, bool with_text) {
    const uint64_t G = genome.size();
    const uint64_t L = (uint64_t)read_len;
    const uint64_t n_chunks = (n_reads + CHUNK - 1) / CHUNK;
    std::vector<Piece> pieces(n_chunks);
    parallel_chunks(n_chunks, [&](uint64_t c) {
        Rng r(mix_seed(seed, 1000 + c));
        Piece& p = pieces[c];
        const uint64_t a = c * CHUNK, e = std::min(n_reads, a + CHUNK);
        p.seq.reserve((e - a) * L);
        std::string rd(L, 'A');
        for (uint64_t i = a; i < e; ++i) {
            const uint64_t len = std::min(L, G);
            const uint64_t st = r.below(G - len + 1);
            const bool rev = r.next() & 1;
            for (uint64_t j = 0; j < len; ++j) rd[j] = rev ? comp(genome[st + len - 1 - j]) : genome[st + j];
            std::string q(len, 'I');
            for (uint64_t j = 0; j < len; ++j) {
                const double pe = 0.001 + 0.002 * (double)j / (double)(len > 1 ? len - 1 : 1);
                if (r.uniform() < pe) {
                    const int cur = rd[j] == 'A' ? 0 : rd[j] == 'C' ? 1 : rd[j] == 'G' ? 2 : 3;
                    rd[j] = kB[(cur + 1 + (int)r.below(3)) & 3];
                    q[j] = '#';
                } else if (j + 30 > len) {
                    q[j] = 'A';
                }
            }
            p.seq.append(rd, 0, len);
            p.lens.push_back((uint32_t)len);
            if (with_text) {
                p.headers.push_back(name + "-" + std::to_string(i + 1));
                p.quals.push_back(std::move(q));
            }
        }
    });
    return assemble(pieces, with_text);
}

ReadBatch gen_nanosim(const std::string& genome, const std::string& name, uint64_t n_reads, uint64_t seed,
                      bool with_text) {
    const uint64_t G = genome.size();
    const uint64_t n_chunks = (n_reads + CHUNK - 1) / CHUNK;
    std::vector<Piece> pieces(n_chunks);
    const double sigma = 0.8, mu = std::log(7800.0) - sigma * sigma / 2.0;
    parallel_chunks(n_chunks, [&](uint64_t c) {
        Rng r(mix_seed(seed, 5000000 + c));
        Piece& p = pieces[c];
        const uint64_t a = c * CHUNK, e = std::min(n_reads, a + CHUNK);
        std::string src, out;
        for (uint64_t i = a; i < e; ++i) {
            // Box-Muller normal -> log-normal length
            const double u1 = std::max(r.uniform(), 1e-300), u2 = r.uniform();
            const double z = std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
            uint64_t len = (uint64_t)std::llround(std::exp(mu + sigma * z));
            len = std::min<uint64_t>(std::max<uint64_t>(len, 85), 59500);
            len = std::min<uint64_t>(len, G);
            const uint64_t st = r.below(G - len + 1);
            const bool rev = r.next() & 1;
            src.assign(len, 'A');
            for (uint64_t j = 0; j < len; ++j) src[j] = rev ? comp(genome[st + len - 1 - j]) : genome[st + j];
            out.clear();
            for (uint64_t j = 0; j < len; ++j) {
                const double u = r.uniform();
                if (u < 0.0333) {          // substitution
                    const int cur = src[j] == 'A' ? 0 : src[j] == 'C' ? 1 : src[j] == 'G' ? 2 : 3;
                    out.push_back(kB[(cur + 1 + (int)r.below(3)) & 3]);
                } else if (u < 0.0666) {   // insertion before the base
                    out.push_back(kB[r.next() & 3]);
                    out.push_back(src[j]);
                } else if (u < 0.1) {      // deletion
                } else {
                    out.push_back(src[j]);
                }
            }
            p.seq += out;
            p.lens.push_back((uint32_t)out.size());
            if (with_text)
                p.headers.push_back(name + "_" + std::to_string(st) + "_aligned_" + std::to_string(i) + "_" +
                                    (rev ? "R" : "F") + "_0_" + std::to_string(len) + "_0");
        }
    });
    return assemble(pieces, with_text);
}

}  // namespace hgah
