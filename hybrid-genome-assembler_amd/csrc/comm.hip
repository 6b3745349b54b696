// comm.hip — multi-GPU counting in the C ABI (SURVEY.md §8(b) hga_comm_init, §8(e)).
//
// One hga_ctx per rank: one process per GPU (torchrun, MPI, ...) or one thread per GPU in one
// process (bin/jf_occurrences --gpus N).  A rank's transport is RCCL over xGMI (hga_comm_init,
// ncclSend/ncclRecv of device buffers, enqueued on the ctx stream) or the caller's host-staged hook
// (hga_comm_init_host: gloo, MPI, sockets, threads).  The protocol is the same either way:
//   every rank: hga_count_run(ctx, 1) on its shard of every file (no per-file drop before the sum)
//   hga_count_exchange(ctx, min):
//     rows packed one u64 per row piece and ordered by hash bucket (owner o holds a range of the
//     counting mix's top bits; exchange.hip kx_xb_hist / kx_xb_scatter), piece counts all-gathered,
//     one all-to-all-v of the pieces and one of the per-bucket counts, owner merge of every sender's
//     runs + `--bc` drop (kx_xb_merge, run_jellyfish.sh:3-6).  Rows too wide to pack go as
//     (key, counts[F]) rows to code-range owners.
//   Afterwards the count queries of the ctx answer for the whole input, identically on every rank:
//     spec_hist  owners' (threshold, total, count) triples gathered and summed per bin
//                (JellyfishOccurrenceReader.cpp:88-108 over all k-mers);
//     select*    owners' sorted exports merged by key = ascending (:110-135);
//     select_device  keys stay on their owner, (n, n_discriminative) summed;
//     rows/dump  owners' sorted rows merged by key (:63-86; run_jellyfish.sh:5-6).
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <map>
#include <vector>

#include "exchange_protocol.hpp"
#include "hga_internal.hpp"

#define HGA_NCCL(call)                                                                               \
    do {                                                                                             \
        ncclResult_t r_ = (call);                                                                    \
        if (r_ != ncclSuccess) throw ::hga::Error(HGA_ERR_COMM, std::string(#call) + ": " + ncclGetErrorString(r_)); \
    } while (0)

static_assert(sizeof(ncclUniqueId) <= HGA_UNIQUE_ID_BYTES, "hga.h HGA_UNIQUE_ID_BYTES must hold an ncclUniqueId");

namespace hga {

namespace {

struct RcclComm : Comm {
    ncclComm_t comm = nullptr;
    bool on_device() const override { return true; }
    void alltoallv(hga_ctx* c, const void* const* send, const uint64_t* sb, void* const* recv,
                   const uint64_t* rb) override {
        // HGA_RCCL_SELF (test hook, read per call): the rank's own slice also goes through
        // ncclSend/ncclRecv, so a one-GPU box exercises the grouped point-to-point calls
        const bool self_p2p = std::getenv("HGA_RCCL_SELF") != nullptr;
        if (!self_p2p) {
            HGA_REQUIRE(rb[rank] == sb[rank], HGA_ERR_COMM, "alltoallv: self sizes disagree");
            if (sb[rank])
                HGA_HIP(hipMemcpyAsync(recv[rank], send[rank], sb[rank], hipMemcpyDeviceToDevice, c->stream));
        }
        HGA_NCCL(ncclGroupStart());
        for (int p = 0; p < nranks; ++p) {
            if (p == rank && !self_p2p) continue;
            if (sb[p]) HGA_NCCL(ncclSend(send[p], sb[p], ncclUint8, p, comm, c->stream));
            if (rb[p]) HGA_NCCL(ncclRecv(recv[p], rb[p], ncclUint8, p, comm, c->stream));
        }
        HGA_NCCL(ncclGroupEnd());
    }
    ~RcclComm() override {
        if (comm) (void)ncclCommDestroy(comm);
    }
};

struct HostComm : Comm {
    hga_transport t{};
    bool on_device() const override { return false; }
    void alltoallv(hga_ctx*, const void* const* send, const uint64_t* sb, void* const* recv,
                   const uint64_t* rb) override {
        const int r = t.alltoallv(t.user, send, sb, recv, rb);
        HGA_REQUIRE(r == 0, HGA_ERR_COMM, "host transport: alltoallv callback failed");
    }
};

Comm& need_comm(hga_ctx* c) {
    HGA_REQUIRE(c->comm, HGA_ERR_STATE, "no communicator: hga_comm_init / hga_comm_init_host first");
    return *c->comm;
}

}  // namespace

// Equal-size all-gather of host bytes: all[p * bytes ...] = rank p's `mine`.
void comm_allgather(hga_ctx* c, const void* mine, uint64_t bytes, void* all) {
    Comm& m = need_comm(c);
    const int P = m.nranks;
    std::vector<uint64_t> sz(P, bytes);
    std::vector<const void*> sp(P);
    std::vector<void*> rp(P);
    if (!m.on_device()) {
        for (int p = 0; p < P; ++p) {
            sp[p] = mine;
            rp[p] = static_cast<char*>(all) + (uint64_t)p * bytes;
        }
        m.alltoallv(c, sp.data(), sz.data(), rp.data(), sz.data());
        return;
    }
    // staged through pinned host memory both ways (true asynchronous copies, no pageable staging)
    char* ds = static_cast<char*>(m.stage.ensure(bytes * (P + 1) + 16));
    char* hs = static_cast<char*>(m.hstage.ensure(bytes * (P + 1) + 16));
    std::memcpy(hs, mine, bytes);
    HGA_HIP(hipMemcpyAsync(ds, hs, bytes, hipMemcpyHostToDevice, c->stream));
    for (int p = 0; p < P; ++p) {
        sp[p] = ds;
        rp[p] = ds + bytes * (p + 1);
    }
    m.alltoallv(c, sp.data(), sz.data(), rp.data(), sz.data());
    HGA_HIP(hipMemcpyAsync(hs + bytes, ds + bytes, bytes * P, hipMemcpyDeviceToHost, c->stream));
    c->sync();
    std::memcpy(all, hs + bytes, bytes * P);
}

// Variable-size all-gather of host bytes, in rank order.
std::vector<std::vector<char>> comm_allgatherv(hga_ctx* c, const void* mine, uint64_t bytes) {
    Comm& m = need_comm(c);
    const int P = m.nranks;
    std::vector<uint64_t> sz(P);
    comm_allgather(c, &bytes, 8, sz.data());
    std::vector<std::vector<char>> out(P);
    for (int p = 0; p < P; ++p) out[p].resize(sz[p]);
    std::vector<uint64_t> sb(P, bytes);
    std::vector<const void*> sp(P);
    std::vector<void*> rp(P);
    if (!m.on_device()) {
        for (int p = 0; p < P; ++p) {
            sp[p] = mine;
            rp[p] = out[p].data();
        }
        m.alltoallv(c, sp.data(), sb.data(), rp.data(), sz.data());
        return out;
    }
    uint64_t tot = 0;
    for (auto v : sz) tot += v;
    char* ds = static_cast<char*>(m.stage.ensure(bytes + tot + 16));
    if (bytes) HGA_HIP(hipMemcpyAsync(ds, mine, bytes, hipMemcpyHostToDevice, c->stream));
    uint64_t o = bytes;
    for (int p = 0; p < P; ++p) {
        sp[p] = ds;
        rp[p] = ds + o;
        o += sz[p];
    }
    m.alltoallv(c, sp.data(), sb.data(), rp.data(), sz.data());
    o = bytes;
    for (int p = 0; p < P; ++p) {
        if (sz[p]) HGA_HIP(hipMemcpyAsync(out[p].data(), ds + o, sz[p], hipMemcpyDeviceToHost, c->stream));
        o += sz[p];
    }
    c->sync();
    return out;
}

// Variable-size gather of host bytes to `root`, in rank order (empty on the other ranks): the sizes
// all-gathered (8 B each), then one all-to-all in which every rank sends only to the root.
std::vector<std::vector<char>> comm_gatherv_root(hga_ctx* c, const void* mine, uint64_t bytes, int root) {
    Comm& m = need_comm(c);
    const int P = m.nranks, me = m.rank;
    HGA_REQUIRE(root >= 0 && root < P, HGA_ERR_INVALID, "gather root out of range");
    std::vector<uint64_t> sz(P);
    comm_allgather(c, &bytes, 8, sz.data());
    std::vector<std::vector<char>> out(P);
    std::vector<uint64_t> sb(P, 0), rb(P, 0);
    sb[root] = bytes;
    if (me == root)
        for (int p = 0; p < P; ++p) rb[p] = sz[p];
    std::vector<const void*> sp(P);
    std::vector<void*> rp(P);
    if (!m.on_device()) {
        for (int p = 0; p < P; ++p) {
            if (me == root) out[p].resize(sz[p]);
            sp[p] = mine;
            rp[p] = me == root ? out[p].data() : nullptr;
        }
        m.alltoallv(c, sp.data(), sb.data(), rp.data(), rb.data());
        return out;
    }
    uint64_t tot = 0;
    for (int p = 0; p < P; ++p) tot += rb[p];
    char* ds = static_cast<char*>(m.stage.ensure(bytes + tot + 16));
    if (bytes) HGA_HIP(hipMemcpyAsync(ds, mine, bytes, hipMemcpyHostToDevice, c->stream));
    uint64_t o = bytes;
    for (int p = 0; p < P; ++p) {
        sp[p] = ds;
        rp[p] = ds + o;
        o += rb[p];
    }
    m.alltoallv(c, sp.data(), sb.data(), rp.data(), rb.data());
    if (me == root) {
        o = bytes;
        for (int p = 0; p < P; ++p) {
            out[p].resize(sz[p]);
            if (sz[p]) HGA_HIP(hipMemcpyAsync(out[p].data(), ds + o, sz[p], hipMemcpyDeviceToHost, c->stream));
            o += sz[p];
        }
    }
    c->sync();
    return out;
}

// All-to-all-v of DEVICE buffers whose per-peer slices are contiguous in rank order; keep_self
// false: the rank's own slice is not moved (rb[rank] must be 0).
void comm_alltoallv_dev(hga_ctx* c, const void* send, const uint64_t* sb_in, void* recv, const uint64_t* rb,
                        bool keep_self) {
    Comm& m = need_comm(c);
    const int P = m.nranks;
    std::vector<const void*> sp(P);
    std::vector<void*> rp(P);
    std::vector<uint64_t> sbv(sb_in, sb_in + P);
    uint64_t so = 0, ro = 0, st = 0, rt = 0;
    for (int p = 0; p < P; ++p) {
        sp[p] = static_cast<const char*>(send) + so;
        so += sbv[p];
    }
    if (!keep_self) {
        HGA_REQUIRE(rb[m.rank] == 0, HGA_ERR_COMM, "alltoallv: own slice kept in place but received");
        sbv[m.rank] = 0;
    }
    const uint64_t* sb = sbv.data();
    for (int p = 0; p < P; ++p) {
        st += sb[p];
        rt += rb[p];
    }
    if (m.on_device()) {
        for (int p = 0; p < P; ++p) {
            rp[p] = static_cast<char*>(recv) + ro;
            ro += rb[p];
        }
        m.alltoallv(c, sp.data(), sb, rp.data(), rb);
        return;
    }
    // host-staged: device -> host, the caller's transport, host -> device (the send buffer whole:
    // a kept-in-place own slice sits between the others)
    std::vector<char> hs(so), hr(rt);
    if (so) HGA_HIP(hipMemcpyAsync(hs.data(), send, so, hipMemcpyDeviceToHost, c->stream));
    c->sync();
    so = 0;
    for (int p = 0; p < P; ++p) {
        sp[p] = hs.data() + so;
        rp[p] = hr.data() + ro;
        so += sb_in[p];
        ro += rb[p];
    }
    (void)st;
    m.alltoallv(c, sp.data(), sb, rp.data(), rb);
    if (rt) HGA_HIP(hipMemcpyAsync(recv, hr.data(), rt, hipMemcpyHostToDevice, c->stream));
    c->sync();
}

std::vector<uint64_t> owner_splitters(int k, int P) { return proto::owner_splitters(k, P); }

namespace {

// The protocol's view of a rank: the ctx's communicator ...
struct CtxXport : proto::Xport {
    hga_ctx* c;
    explicit CtxXport(hga_ctx* cc) : c(cc) {
        rank = cc->comm->rank;
        nranks = cc->comm->nranks;
    }
    void allgather(const void* mine, uint64_t bytes, void* all) override { comm_allgather(c, mine, bytes, all); }
    std::vector<std::vector<char>> allgatherv(const void* mine, uint64_t bytes) override {
        return comm_allgatherv(c, mine, bytes);
    }
    void alltoallv_eng(const void* send, const uint64_t* sb, void* recv, const uint64_t* rb, bool keep_self) override {
        comm_alltoallv_dev(c, send, sb, recv, rb, keep_self);
    }
    std::vector<std::vector<char>> gatherv_root(const void* mine, uint64_t bytes, int root) override {
        return comm_gatherv_root(c, mine, bytes, root);
    }
};

[[noreturn]] void throw_query_error(const proto::QueryError& e);

// ... and its rows on the device (exchange.hip kernels).
struct DevEngine {
    hga_ctx* c;
    // extra[0] of the exchange is the rank's instance count: with the count not settled yet, the fused
    // head gathers it from the device counters
    bool extra0_instances = false;
    int k() const { return c->count.k; }
    uint32_t n_files() const { return c->count.n_files; }
    uint64_t rows() const { return c->count.rows; }
    int pack_bits() { return count_pack_bits(c); }
    void* send_buf(uint64_t bytes) { return c->count.xsend.ensure(bytes + 64); }
    void* recv_buf(uint64_t bytes) { return c->count.xrecv.ensure(bytes + 64); }
    int xb_pack(uint32_t P, uint64_t* per) { return count_xb_pack(c, P, per); }
    // Head of the packed exchange over an on-device communicator: the per-owner totals, R, the extras
    // and this rank's count error bits are all-gathered from device memory as W + 1 words on EVERY
    // rank, whatever its local state (a rank deciding alone between this gather and a
    // W-word one would mismatch the collective).  A rank whose count kernels wrote the pieces (xb_on)
    // enqueues its totals on the device and has its unsettled count's counters read back in the same
    // host round trip; any other rank (a bucket left to the generic kernel, cached dump rows, a count
    // already settled by a local query) settles first — without throwing: its error bits join the
    // gather — and bins its rows (count_xb_pack).  Errors are decided on the gathered bits, so every
    // rank raises the lowest failing rank's and none enters the piece all-to-all alone.
    bool xb_pack_gather(uint32_t P, std::vector<uint64_t>& per, std::vector<uint64_t>& all, int& R) {
        Comm& m = *c->comm;
        auto& s = c->count;
        if (!m.on_device()) return false;
        const size_t W = per.size(), Wg = W + 1;   // + the error word
        const uint64_t B = 8 * (uint64_t)Wg;
        char* ds = static_cast<char*>(m.stage.ensure(B * (P + 1) + 16));
        char* hs = static_cast<char*>(m.hstage.ensure(B * (P + 1) + 64 + 16));
        auto* hp = reinterpret_cast<unsigned long long*>(hs + B * (P + 1));   // the count's counters
        const bool emitted = s.xb_on && s.xb_P == P;
        const bool pend = emitted && s.pending;
        uint64_t ebits = 0;   // a non-emitting rank's settle bits
        if (emitted) {
            HGA_REQUIRE(count_xb_pack_begin(c, P, reinterpret_cast<uint64_t*>(ds)), HGA_ERR_STATE,
                        "the count did not emit exchange pieces");
            R = s.xb_R;
        } else {
            if (s.pending) {
                HGA_HIP(hipMemcpyAsync(hp, s.cursor.p, 64, hipMemcpyDeviceToHost, c->stream));
                c->sync();
                ebits = hp[2] & 7ull;
                if (ebits) {   // consumed as failed, as count_settle would (it would throw here)
                    s.pending = false;
                    s.last_err = ebits;
                    s.ran = false;
                } else {
                    count_settle(c, hp);
                }
            }
            if (ebits) {   // nothing to send: the gathered bits stop every rank before the all-to-all
                R = proto::xb_base_bits(s.k);
                std::fill(per.begin(), per.begin() + P, 0ull);
            } else {
                R = count_xb_pack(c, P, per.data());
            }
            if (extra0_instances && W > (size_t)P + 1) per[P + 1] = s.instances;
        }
        per[P] = (uint64_t)R;
        const size_t h0 = emitted ? P : 0;   // an emitting rank's totals are on the device already
        std::memcpy(hs + 8 * h0, per.data() + h0, 8 * (W - h0));
        HGA_HIP(hipMemcpyAsync(ds + 8 * h0, hs + 8 * h0, 8 * (W - h0), hipMemcpyHostToDevice, c->stream));
        if (pend) {   // settle bits (gstat[2]) and, if asked, instances (gstat[4]) from the device
            HGA_HIP(hipMemcpyAsync(ds + 8 * W, static_cast<char*>(s.cursor.p) + 16, 8, hipMemcpyDeviceToDevice,
                                   c->stream));
            if (extra0_instances && W > (size_t)P + 1)
                HGA_HIP(hipMemcpyAsync(ds + 8 * (P + 1), static_cast<char*>(s.cursor.p) + 32, 8,
                                       hipMemcpyDeviceToDevice, c->stream));
            HGA_HIP(hipMemcpyAsync(hp, s.cursor.p, 64, hipMemcpyDeviceToHost, c->stream));
        } else {
            reinterpret_cast<uint64_t*>(hs)[W] = ebits;
            HGA_HIP(hipMemcpyAsync(ds + 8 * W, hs + 8 * W, 8, hipMemcpyHostToDevice, c->stream));
        }
        std::vector<uint64_t> sz(P, B);
        std::vector<const void*> sp(P, ds);
        std::vector<void*> rp(P);
        for (uint32_t p = 0; p < P; ++p) rp[p] = ds + B * (p + 1);
        m.alltoallv(c, sp.data(), sz.data(), rp.data(), sz.data());
        HGA_HIP(hipMemcpyAsync(hs + B, ds + B, B * P, hipMemcpyDeviceToHost, c->stream));
        c->sync();
        const uint64_t* g = reinterpret_cast<const uint64_t*>(hs + B);
        std::vector<uint64_t> bits(P);
        for (uint32_t p = 0; p < P; ++p) bits[p] = g[(size_t)p * Wg + W] & 7ull;
        const proto::QueryError qe = proto::first_error(bits.data(), (int)P, 1);
        if (qe.rank >= 0) {
            if (pend) {   // this rank's run is consumed as failed (as count_settle would)
                s.pending = false;
                s.last_err = hp[2] & 7ull;
                if (s.last_err) s.ran = false;
            }
            throw_query_error(qe);
        }
        if (pend) count_settle(c, hp);
        all.assign((size_t)P * W, 0);
        for (uint32_t p = 0; p < P; ++p)
            for (size_t i = 0; i < W; ++i) all[(size_t)p * W + i] = g[(size_t)p * Wg + i];
        if (emitted) {
            for (uint32_t o = 0; o < P; ++o) per[o] = all[(size_t)m.rank * W + o];
            count_xb_pack_finish(c, P, per.data());
        }
        return true;
    }
    const void* xb_pieces() const { return c->count.xsend.p; }
    const void* xb_dir() const { return c->count.xdir.p; }
    void xb_merge(const uint64_t* in, const uint64_t* self, const uint64_t* n_from, const uint64_t* dir_in,
                  const int* r_from, uint32_t P, uint32_t me, uint32_t min) {
        count_xb_merge(c, in, self, n_from, dir_in, r_from, P, me, min);
    }
    void partition(const uint64_t* spl, uint32_t P, uint64_t* keys, uint32_t* counts, uint64_t* per) {
        count_partition(c, spl, P, keys, counts, per);
    }
    void merge(const uint64_t* keys, const uint32_t* counts, uint64_t n, uint32_t min) {
        count_merge(c, keys, counts, n, min);
    }
    void sync() { c->sync(); }
};

}  // namespace

void count_exchange(hga_ctx* c, uint32_t min_per_file) {
    auto& s = c->count;
    Comm& m = need_comm(c);
    // over an on-device communicator the packed exchange's head (DevEngine::xb_pack_gather) settles an
    // unsettled count itself, on every rank the same way, so that a failed count reaches the others
    // through the gathered error words instead of leaving this rank alone
    const bool dev_head = m.on_device() && count_pack_bits(c) > 0;
    if (!dev_head) count_settle(c);
    HGA_REQUIRE(s.ran, HGA_ERR_STATE, "hga_count_run(ctx, 1) first");
    HGA_REQUIRE(s.min_per_file == 1, HGA_ERR_STATE, "the local count must keep singletons: hga_count_run(ctx, 1)");
    HGA_REQUIRE(min_per_file >= 1, HGA_ERR_INVALID, "min_per_file must be >= 1");
    CtxXport x(c);
    // instances / bytes this rank counted, summed for the global stats (in the piece-count gather)
    std::vector<uint64_t> mine{s.instances, 0}, g;
    for (auto l : s.seq_len) mine[1] += l;
    DevEngine e{c};
    e.extra0_instances = dev_head;
    proto::count_exchange(e, x, min_per_file, mine, &g);
    s.g_instances = g[0];
    s.g_bytes = g[1];
    // the global row count once, here, so hga_count_get_stats stays local (not a collective); over
    // RCCL it is only enqueued (pinned staging both ways) and summed when get_stats asks for it
    const int P = x.nranks;
    if (m.on_device()) {
        uint64_t* hs = static_cast<uint64_t*>(s.g_rows_h.ensure(8 * ((uint64_t)P + 1)));
        char* ds = static_cast<char*>(m.stage.ensure(8 * ((uint64_t)P + 1) + 16));
        hs[0] = s.rows;
        std::vector<uint64_t> sz(P, 8);
        std::vector<const void*> sp(P, ds);
        std::vector<void*> rp(P);
        for (int p = 0; p < P; ++p) rp[p] = ds + 8 * (p + 1);
        HGA_HIP(hipMemcpyAsync(ds, hs, 8, hipMemcpyHostToDevice, c->stream));
        m.alltoallv(c, sp.data(), sz.data(), rp.data(), sz.data());
        HGA_HIP(hipMemcpyAsync(hs + 1, ds + 8, 8 * (uint64_t)P, hipMemcpyDeviceToHost, c->stream));
        s.g_rows_pending = true;
        s.g_rows_P = P;
    } else {
        std::vector<uint64_t> gr(P);
        uint64_t r = s.rows;
        comm_allgather(c, &r, 8, gr.data());
        s.g_rows = 0;
        for (auto v : gr) s.g_rows += v;
        s.g_rows_pending = false;
    }
    s.dist = true;
}

// The global row count of the last exchange (its all-gather was enqueued by count_exchange).
uint64_t count_global_rows(hga_ctx* c) {
    auto& s = c->count;
    if (s.g_rows_pending) {
        c->sync();
        const uint64_t* hs = static_cast<const uint64_t*>(s.g_rows_h.p);
        s.g_rows = 0;
        for (int p = 0; p < s.g_rows_P; ++p) s.g_rows += hs[1 + p];
        s.g_rows_pending = false;
    }
    return s.g_rows;
}

// ---- global answers of the count queries after hga_count_exchange ----------------------------

namespace {
using proto::HS_CAP;
using proto::HS_HDR;
using proto::HS_WORDS;

// A rank's histogram slot for the one-shot gather (proto::merge_hist_slots): [error bits, overflow
// rows, pairs, the first HS_CAP pairs]; gstat: the counters of an unconsumed count run (its settle
// bits), or null.
__global__ void kx_hist_slot(const unsigned long long* __restrict__ ctrl, const unsigned long long* __restrict__ pairs,
                             const unsigned long long* __restrict__ gstat, uint64_t ncap,
                             unsigned long long* __restrict__ slot) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t == 0) {
        slot[0] = (gstat ? (gstat[2] & 7ull) : 0ull) | ((ctrl[1] & 1ull) ? proto::QE_SPEC_THR : 0ull) |
                  ((ctrl[1] & 2ull) ? proto::QE_OVER : 0ull) | (ctrl[2] > ncap ? proto::QE_COMPACT : 0ull);
        slot[1] = ctrl[0];
        slot[2] = ctrl[2];
    }
    const uint64_t n = ctrl[2] < HS_CAP ? ctrl[2] : HS_CAP;
    for (uint64_t i = t; i < 2 * n; i += (uint64_t)gridDim.x * blockDim.x) slot[HS_HDR + i] = pairs[i];
}

// The same error on every rank (the lowest failing one's, as its own checks name it).
[[noreturn]] void throw_query_error(const proto::QueryError& e) {
    static const struct {
        uint64_t bit;
        hga_status code;
        const char* msg;
    } order[] = {{proto::QE_POOL, HGA_ERR_OOM, "level-1 block pool exhausted"},
                 {proto::QE_UNSPLIT, HGA_ERR_INVALID, "a bucket could not be split to fit the LDS table"},
                 {proto::QE_ROWCAP, HGA_ERR_OOM, "row capacity exceeded"},
                 {proto::QE_SPEC_THR, HGA_ERR_INVALID, "a row's specificity is above the last threshold"},
                 {proto::QE_OVER, HGA_ERR_OOM, "histogram overflow list full"},
                 {proto::QE_COMPACT, HGA_ERR_OOM, "histogram compaction buffer full"},
                 {proto::QE_LOCAL, HGA_ERR_STATE, "count query failed before its gather"}};
    for (const auto& o : order)
        if (e.bits & o.bit) throw Error(o.code, "rank " + std::to_string(e.rank) + ": " + o.msg);
    throw Error(HGA_ERR_INVALID, "rank " + std::to_string(e.rank) + ": count query failed");
}

// Runs a local query that may fail on this rank with an error the others must learn about: returns
// its error bits (CountState::last_err) instead of throwing them; other errors propagate.
template <class Fn>
uint64_t run_reporting(hga_ctx* c, Fn&& fn) {
    c->count.last_err = 0;
    try {
        fn();
    } catch (const Error&) {
        if (!c->count.last_err) throw;
    }
    return c->count.last_err;
}

// ---- code-range re-partition of device lists (proto::repartition) ----
// pos[o] = entries of the ascending list (codes = key & cmask) below spl[o], o < P - 1.
__global__ void kx_split_sorted(const uint64_t* __restrict__ keys, uint64_t n, uint64_t cmask,
                                const uint64_t* __restrict__ spl, uint32_t m, uint64_t* __restrict__ pos) {
    const uint32_t o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= m) return;
    const uint64_t v = spl[o];
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = lo + (hi - lo) / 2;
        if ((keys[mid] & cmask) < v) lo = mid + 1;
        else hi = mid;
    }
    pos[o] = lo;
}
// dst[i] = src[idx[i]] for entries of w u32 words
__global__ void kx_gather_words(const uint32_t* __restrict__ idx, const uint32_t* __restrict__ src, uint64_t n,
                                uint32_t w, uint32_t* __restrict__ dst) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t j = idx[i];
    for (uint32_t q = 0; q < w; ++q) dst[i * w + q] = src[j * w + q];
}
__global__ void kx_iota(uint32_t* v, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = (uint32_t)i;
}

// An ascending device list (keys[n] + n payloads of vb bytes, vb a multiple of 4) for proto::repartition;
// the rank's code range ends up in `out` (keys, then payloads), ascending.
struct DevList {
    hga_ctx* c;
    int bits;
    uint64_t n;
    const uint64_t* k;
    const void* v;
    uint32_t vb;
    DevBuf& out;
    DevBuf tmp;
    uint64_t n_out = 0;
    uint32_t vbytes() const { return vb; }
    const void* keys() const { return k; }
    const void* vals() const { return v; }
    void split(const uint64_t* spl, uint32_t P, uint64_t* per) {
        std::vector<uint64_t> pos(P + 1, 0);
        pos[P] = n;
        if (P > 1) {
            auto* d = static_cast<uint64_t*>(tmp.ensure(16 * (uint64_t)P + 64));
            HGA_HIP(hipMemcpyAsync(d, spl, 8ull * (P - 1), hipMemcpyHostToDevice, c->stream));
            const uint64_t cmask = bits >= 64 ? ~0ull : (1ull << bits) - 1;
            hipLaunchKernelGGL(kx_split_sorted, dim3((P + 254) / 255), dim3(256), 0, c->stream, k, n, cmask, d, P - 1,
                               d + P);
            c->check_launch("kx_split_sorted");
            HGA_HIP(hipMemcpyAsync(pos.data() + 1, d + P, 8ull * (P - 1), hipMemcpyDeviceToHost, c->stream));
            c->sync();
        }
        for (uint32_t o = 0; o < P; ++o) per[o] = pos[o + 1] - pos[o];
    }
    void* recv(uint64_t m) { return out.ensure(std::max<uint64_t>(m, 1) * (8 + vb) + 64); }
    void finish(const uint64_t*, uint32_t, uint64_t m) {
        n_out = m;
        if (m < 2) return;
        uint64_t* rk = out.as<uint64_t>();
        auto* rv = reinterpret_cast<uint32_t*>(rk + m);
        if (vb == 0) {
            radix_sort_u64(c, rk, nullptr, m, bits, c->count.scratch);
        } else if (vb == 4) {
            radix_sort_u64(c, rk, rv, m, bits, c->count.scratch);
        } else {   // wider payloads: sort (key, index), then gather the payloads
            const uint32_t w = vb / 4;
            char* t = static_cast<char*>(tmp.ensure(m * (4 + (uint64_t)vb) + 64));
            auto* idx = reinterpret_cast<uint32_t*>(t);
            auto* pv = reinterpret_cast<uint32_t*>(t + m * 4);
            hipLaunchKernelGGL(kx_iota, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, c->stream, idx, m);
            radix_sort_u64(c, rk, idx, m, bits, c->count.scratch);
            hipLaunchKernelGGL(kx_gather_words, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, c->stream, idx, rv, m, w, pv);
            c->check_launch("kx_gather_words");
            HGA_HIP(hipMemcpyAsync(rv, pv, m * (uint64_t)vb, hipMemcpyDeviceToDevice, c->stream));
        }
    }
};
}  // namespace

void count_spec_hist_global(hga_ctx* c, const double* thr, uint32_t n_thr, std::vector<int64_t>& out) {
    Comm& m = need_comm(c);
    std::vector<int64_t> local;
    CtxXport x(c);
    proto::QueryError qe;
    if (!m.on_device()) {
        uint64_t err;
        try {   // any local failure joins the gather as an error word (the others do not wait alone)
            err = run_reporting(c, [&] { count_spec_hist(c, thr, n_thr, local); });
        } catch (const Error&) {
            err = c->count.last_err ? c->count.last_err : proto::QE_LOCAL;
            local.clear();
        }
        out = proto::spec_hist_global(x, local, err, &qe);
        if (qe.rank >= 0) throw_query_error(qe);
        return;
    }
    // RCCL: every rank's device pairs and error bits gathered inside the local call's one
    // synchronisation; a rank with an overflow list or more than HS_CAP pairs sends everyone to the
    // general gather, a rank with an error makes every rank raise it (proto::merge_hist_slots)
    const int P = m.nranks;
    const uint64_t sb = HS_WORDS * 8;
    char* ds = static_cast<char*>(m.stage.ensure(sb * (P + 1) + 16));
    auto* hs = static_cast<unsigned long long*>(m.hstage.ensure(sb * P + 16));
    const unsigned long long* gst = c->count.pending ? static_cast<const unsigned long long*>(c->count.cursor.p) : nullptr;
    bool gathered = false;
    const SpecHook hook = [&](const unsigned long long* ctrl, const unsigned long long* pairs) {
        hipLaunchKernelGGL(kx_hist_slot, dim3(8), dim3(256), 0, c->stream, ctrl, pairs, gst, (uint64_t)1 << 20,
                           reinterpret_cast<unsigned long long*>(ds));
        c->check_launch("kx_hist_slot");
        std::vector<uint64_t> sz(P, sb);
        std::vector<const void*> sp(P, ds);
        std::vector<void*> rp(P);
        for (int p = 0; p < P; ++p) rp[p] = ds + sb * (p + 1);
        m.alltoallv(c, sp.data(), sz.data(), rp.data(), sz.data());
        HGA_HIP(hipMemcpyAsync(hs, ds + sb, sb * P, hipMemcpyDeviceToHost, c->stream));
        gathered = true;
    };
    // a local failure before the hook (no run, an allocation, a state check) still takes part in the
    // slot gather, with its error word only, so the other ranks do not wait in it alone
    uint64_t err = 0;
    std::exception_ptr fail;
    try {
        err = run_reporting(c, [&] { count_spec_hist(c, thr, n_thr, local, &hook); });
    } catch (...) {
        fail = std::current_exception();
    }
    if (!gathered) {
        unsigned long long hdr[HS_HDR] = {};
        hdr[0] = c->count.last_err ? c->count.last_err : proto::QE_LOCAL;
        HGA_HIP(hipMemcpyAsync(ds, hdr, sizeof(hdr), hipMemcpyHostToDevice, c->stream));
        std::vector<uint64_t> sz(P, sb);
        std::vector<const void*> sp(P, ds);
        std::vector<void*> rp(P);
        for (int p = 0; p < P; ++p) rp[p] = ds + sb * (p + 1);
        m.alltoallv(c, sp.data(), sz.data(), rp.data(), sz.data());
        HGA_HIP(hipMemcpyAsync(hs, ds + sb, sb * P, hipMemcpyDeviceToHost, c->stream));
        c->sync();
    } else if (fail) {
        std::rethrow_exception(fail);   // after its gather: a device failure, this rank's own
    }
    (void)err;   // this rank's bits are in its own slot
    const proto::SlotMerge r = proto::merge_hist_slots(reinterpret_cast<const uint64_t*>(hs), P, out, &qe);
    if (r == proto::SlotMerge::error) throw_query_error(qe);
    if (r == proto::SlotMerge::fallback) {   // the same decision on every rank (the same gathered words)
        out = proto::spec_hist_global(x, local, 0, &qe);
        if (qe.rank >= 0) throw_query_error(qe);
    }
}

void count_select_global(hga_ctx* c, int64_t lower, int64_t upper, uint64_t* n, uint64_t* nd) {
    Comm& m = need_comm(c);
    c->count.sel_rep_n = ~0ull;   // a new selection: not re-partitioned yet
    // an unconsumed count run is settled first, so a failed run is reported in the gathered words
    const uint64_t serr = run_reporting(c, [&] { count_settle(c); });
    const int P = m.nranks;
    uint64_t mine[3] = {0, 0, serr};
    std::vector<uint64_t> all(3 * (size_t)P);
    if (!m.on_device()) {
        if (!serr) count_select(c, lower, upper, &mine[0], &mine[1]);
        CtxXport x(c);
        x.allgather(mine, 24, all.data());
    } else {
        // RCCL: the counters' gather rides in the local call's one synchronisation
        char* ds = static_cast<char*>(m.stage.ensure(24 * ((uint64_t)P + 1) + 16));
        auto* hs = static_cast<uint64_t*>(m.hstage.ensure(24 * (uint64_t)P + 16));
        auto gather = [&] {
            std::vector<uint64_t> sz(P, 24);
            std::vector<const void*> sp(P, ds);
            std::vector<void*> rp(P);
            for (int p = 0; p < P; ++p) rp[p] = ds + 24 * (p + 1);
            m.alltoallv(c, sp.data(), sz.data(), rp.data(), sz.data());
            HGA_HIP(hipMemcpyAsync(hs, ds + 24, 24 * (uint64_t)P, hipMemcpyDeviceToHost, c->stream));
        };
        if (serr) {   // take part in the gather with the error word only
            HGA_HIP(hipMemcpyAsync(ds, mine, 24, hipMemcpyHostToDevice, c->stream));
            gather();
            c->sync();
        } else {
            const SelHook hook = [&](const unsigned long long* stat) {
                HGA_HIP(hipMemcpyAsync(ds, stat, 16, hipMemcpyDeviceToDevice, c->stream));
                HGA_HIP(hipMemsetAsync(ds + 16, 0, 8, c->stream));
                gather();
            };
            count_select(c, lower, upper, &mine[0], &mine[1], &hook);
        }
        std::memcpy(all.data(), hs, 24 * (size_t)P);
    }
    const proto::QueryError qe = proto::first_error(all.data() + 2, P, 3);
    if (qe.rank >= 0) throw_query_error(qe);
    *n = *nd = 0;
    for (int p = 0; p < P; ++p) {
        *n += all[3 * (size_t)p];
        *nd += all[3 * (size_t)p + 1];
    }
}

// This rank's code range of the global export (proto::repartition of the owners' sorted selections,
// one all-to-all of the selected keys), kept on the device in count.sel_rep; returns its size.
uint64_t count_export_repartition(hga_ctx* c) {
    auto& s = c->count;
    need_comm(c);
    count_settle(c);
    if (s.sel_rep_n != ~0ull) return s.sel_rep_n;
    CtxXport x(c);
    const bool flag_bit = s.k <= 31;
    const uint64_t cap = std::max<uint64_t>(s.rows, 1);
    const char* sb = static_cast<const char*>(s.sel_keys.p);
    DevList l{c, 2 * s.k, s.n_sel, reinterpret_cast<const uint64_t*>(sb), flag_bit ? nullptr : sb + cap * 8,
              flag_bit ? 0u : 4u, s.sel_rep, {}};
    s.sel_rep_n = proto::repartition(l, x, s.k);
    return s.sel_rep_n;
}

// The whole export (after count_select): the ranks' code ranges concatenated in rank order —
// ascending, no merge — on every rank, or on the gather root only (hga_comm_set_root: one writer,
// JellyfishOccurrenceReader.cpp:110-135; the other ranks get an empty list).
void count_fetch_selected_global(hga_ctx* c, std::vector<uint64_t>& keys, std::vector<uint8_t>& flags) {
    auto& s = c->count;
    const int root = need_comm(c).root;
    const uint64_t n = count_export_repartition(c);
    const bool flag_bit = s.k <= 31;
    std::vector<uint64_t> k(n);
    std::vector<uint8_t> f(n);
    if (n) {
        HGA_HIP(hipMemcpyAsync(k.data(), s.sel_rep.p, n * 8, hipMemcpyDeviceToHost, c->stream));
        std::vector<uint32_t> f32;
        if (!flag_bit) {
            f32.resize(n);
            HGA_HIP(hipMemcpyAsync(f32.data(), s.sel_rep.as<uint64_t>() + n, n * 4, hipMemcpyDeviceToHost, c->stream));
        }
        c->sync();
        for (uint64_t i = 0; i < n; ++i) {
            f[i] = flag_bit ? (uint8_t)(k[i] >> 63) : (uint8_t)f32[i];
            if (flag_bit) k[i] &= ~(1ull << 63);
        }
    }
    CtxXport x(c);
    keys = proto::concat_root(x, k, root);
    flags = proto::concat_root(x, f, root);
}

// The global rows (file < 0) or one file's dump rows: the owners' sorted rows re-partitioned by code
// range on the device (one all-to-all of the rows), each rank's range fetched, concatenated on every
// rank or on the gather root only (hga_comm_set_root).
void count_rows_global(hga_ctx* c, int file, std::vector<uint64_t>& keys, std::vector<uint32_t>& counts) {
    auto& s = c->count;
    const int root = need_comm(c).root;
    count_settle(c);
    HGA_REQUIRE(s.ran, HGA_ERR_STATE, "hga_count_run not called");
    count_dense(c);
    HGA_REQUIRE(file < (int)s.n_files, HGA_ERR_INVALID, "file index out of range");
    const uint32_t F = s.n_files;
    DevBuf dk, dc, out;
    count_rows_device(c, dk, dc);
    CtxXport x(c);
    DevList l{c, 2 * s.k, s.rows, dk.as<uint64_t>(), dc.p, 4u * F, out, {}};
    const uint64_t n = proto::repartition(l, x, s.k);
    std::vector<uint64_t> k(n);
    std::vector<uint32_t> v((size_t)n * F);
    if (n) {
        HGA_HIP(hipMemcpyAsync(k.data(), out.p, n * 8, hipMemcpyDeviceToHost, c->stream));
        HGA_HIP(hipMemcpyAsync(v.data(), out.as<uint64_t>() + n, n * 4ull * F, hipMemcpyDeviceToHost, c->stream));
    }
    c->sync();
    std::vector<uint64_t> mk;
    std::vector<uint32_t> mv;
    if (file < 0) {
        mk.swap(k);
        mv.swap(v);
    } else {
        for (uint64_t i = 0; i < n; ++i)
            if (v[i * F + (uint32_t)file]) {
                mk.push_back(k[i]);
                mv.push_back(v[i * F + (uint32_t)file]);
            }
    }
    keys = proto::concat_root(x, mk, root);
    counts = proto::concat_root(x, mv, root);
}

void comm_set_root(hga_ctx* c, int root) {
    Comm& m = need_comm(c);
    HGA_REQUIRE(root >= -1 && root < m.nranks, HGA_ERR_INVALID, "root must be -1 or a rank");
    m.root = root;
}

bool comm_is_gather_leaf(hga_ctx* c) {   // a rank that gets no copy of the gathered lists
    return c->comm && c->comm->root >= 0 && c->comm->root != c->comm->rank;
}

// ---- sharded categorization ------------------------------------------------------------------

void lookup_gather(hga_ctx* c) {
    auto& L = c->lookup;
    need_comm(c);
    HGA_REQUIRE(L.ran, HGA_ERR_STATE, "hga_lookup_run not called");
    HGA_REQUIRE(!L.gathered, HGA_ERR_STATE, "index already gathered: hga_lookup_run first");
    proto::CsrIndex in;
    in.n = L.n_reads;
    in.windows = L.windows;
    in.reads_hit = L.reads_hit;
    in.first_read_id = L.first_read_id;
    in.n_sdk = L.n_sdk;
    const uint64_t n = L.n_reads, H = L.hits, U = L.firsts, K = L.n_sdk;
    in.hit_ptr.resize(n + 1);
    in.first_ptr.resize(n + 1);
    in.kci_ptr.resize(K + 1);
    in.hit_kid.resize(H);
    in.hit_pos.resize(H);
    in.sorted_kid.resize(H);
    in.first_kid.resize(U);
    in.first_pos.resize(U);
    in.kci_read.resize(H);
    auto d2h = [&](void* dst, const DevBuf& src, size_t bytes) {
        if (bytes) HGA_HIP(hipMemcpyAsync(dst, src.p, bytes, hipMemcpyDeviceToHost, c->stream));
    };
    d2h(in.hit_ptr.data(), L.hit_ptr, (n + 1) * 8);
    d2h(in.hit_kid.data(), L.hit_kid, H * 4);
    d2h(in.hit_pos.data(), L.hit_pos, H * 4);
    d2h(in.sorted_kid.data(), L.s_val2, H * 4);
    d2h(in.first_ptr.data(), L.first_ptr, (n + 1) * 8);
    d2h(in.first_kid.data(), L.first_kid, U * 4);
    d2h(in.first_pos.data(), L.first_pos, U * 4);
    d2h(in.kci_ptr.data(), L.kci_ptr, (K + 1) * 8);
    d2h(in.kci_read.data(), L.kci_val, H * 4);
    c->sync();
    CtxXport x(c);
    proto::CsrIndex g;
    HGA_REQUIRE(proto::gather_index(x, in, g), HGA_ERR_INVALID,
                "lookup shards must load the same SDK set and cover contiguous ReadID ranges in rank order");
    HGA_REQUIRE(g.n < (1ull << 32), HGA_ERR_INVALID, "too many reads");
    auto h2d = [&](DevBuf& dst, const void* src, size_t bytes) {
        void* d = dst.ensure(bytes + 16);
        if (bytes) HGA_HIP(hipMemcpyAsync(d, src, bytes, hipMemcpyHostToDevice, c->stream));
    };
    const uint64_t Hg = g.hit_kid.size(), Ug = g.first_kid.size();
    h2d(L.hit_ptr, g.hit_ptr.data(), (g.n + 1) * 8);
    h2d(L.hit_kid, g.hit_kid.data(), Hg * 4);
    h2d(L.hit_pos, g.hit_pos.data(), Hg * 4);
    h2d(L.s_val2, g.sorted_kid.data(), Hg * 4);
    h2d(L.first_ptr, g.first_ptr.data(), (g.n + 1) * 8);
    h2d(L.first_kid, g.first_kid.data(), Ug * 4);
    h2d(L.first_pos, g.first_pos.data(), Ug * 4);
    h2d(L.kci_ptr, g.kci_ptr.data(), (K + 1) * 8);
    h2d(L.kci_val, g.kci_read.data(), Hg * 4);
    ++L.kci_epoch;
    c->sync();
    L.loc_n_reads = L.n_reads;
    L.loc_first_read_id = L.first_read_id;
    L.n_reads = g.n;
    L.first_read_id = g.first_read_id;
    L.hits = Hg;
    L.firsts = Ug;
    L.windows = g.windows;
    L.reads_hit = g.reads_hit;
    L.gathered = true;
    c->conn.ready = false;
}

void connections_gather(hga_ctx* c, uint64_t* n_out) {
    auto& S = c->conn;
    need_comm(c);
    HGA_REQUIRE(S.ready, HGA_ERR_STATE, "hga_connections_run not called");
    proto::ConnList in;
    in.x.resize(S.n);
    in.y.resize(S.n);
    in.s.resize(S.n);
    in.g.resize(S.n);
    connections_fetch(c, in.x.data(), in.y.data(), in.s.data(), in.g.data());
    CtxXport x(c);
    const proto::ConnList g = proto::merge_connections(x, in);
    const uint64_t N = g.x.size();
    auto h2d = [&](DevBuf& dst, const void* src, size_t bytes) {
        void* d = dst.ensure(bytes + 16);
        if (bytes) HGA_HIP(hipMemcpyAsync(d, src, bytes, hipMemcpyHostToDevice, c->stream));
    };
    h2d(S.ox, g.x.data(), N * 4);
    h2d(S.oy, g.y.data(), N * 4);
    h2d(S.os, g.s.data(), N * 8);
    h2d(S.og, g.g.data(), N);
    c->sync();
    S.n = N;
    *n_out = N;
}

void comm_init_rccl(hga_ctx* c, const void* id, int rank, int nranks) {
    HGA_REQUIRE(id, HGA_ERR_INVALID, "null unique id");
    HGA_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, HGA_ERR_INVALID, "rank out of range");
    auto cm = std::make_unique<RcclComm>();
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    HGA_NCCL(ncclCommInitRank(&cm->comm, nranks, uid, rank));
    cm->rank = rank;
    cm->nranks = nranks;
    c->comm = std::move(cm);
    c->count.dist = false;
}

void comm_init_host(hga_ctx* c, int rank, int nranks, const hga_transport* t) {
    HGA_REQUIRE(t && t->alltoallv, HGA_ERR_INVALID, "transport with an alltoallv callback required");
    HGA_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, HGA_ERR_INVALID, "rank out of range");
    auto cm = std::make_unique<HostComm>();
    cm->t = *t;
    cm->rank = rank;
    cm->nranks = nranks;
    c->comm = std::move(cm);
    c->count.dist = false;
}

}  // namespace hga

extern "C" hga_status hga_comm_unique_id(void* id) {
    if (!id) return HGA_ERR_INVALID;
    ncclUniqueId uid;
    const ncclResult_t r = ncclGetUniqueId(&uid);
    if (r != ncclSuccess) return HGA_ERR_COMM;
    std::memcpy(id, &uid, sizeof(uid));
    return HGA_OK;
}
