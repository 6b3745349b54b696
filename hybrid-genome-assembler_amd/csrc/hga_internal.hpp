// Internal host-side state of libhga: the context, device buffers, error plumbing and
// the per-kernel event profiler.  Not part of the ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <algorithm>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <functional>
#include <vector>

#include "../../include/hga.h"

namespace hga {

// Exceptions never cross the ABI: api.hip catches them and maps them to a status.
struct Error : std::runtime_error {
    hga_status code;
    Error(hga_status c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define HGA_HIP(call)                                                                      \
    do {                                                                                   \
        hipError_t e_ = (call);                                                            \
        if (e_ != hipSuccess)                                                              \
            throw ::hga::Error(e_ == hipErrorOutOfMemory ? HGA_ERR_OOM : HGA_ERR_HIP,     \
                               std::string(#call) + ": " + hipGetErrorString(e_));        \
    } while (0)

#define HGA_REQUIRE(cond, code, msg)                           \
    do {                                                       \
        if (!(cond)) throw ::hga::Error((code), (msg));        \
    } while (0)

// Grow-only device buffer.
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    void* ensure(size_t bytes) {
        if (bytes <= cap && p) return p;
        release();
        size_t b = bytes ? bytes : 16;
        HGA_HIP(hipMalloc(&p, b));
        cap = b;
        return p;
    }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
};

// Grow-only pinned host buffer for small async transfers (one per ctx).
struct PinnedBuf {
    void* p = nullptr;
    size_t cap = 0;
    PinnedBuf() = default;
    PinnedBuf(const PinnedBuf&) = delete;
    PinnedBuf& operator=(const PinnedBuf&) = delete;
    ~PinnedBuf() {
        if (p) (void)hipHostFree(p);
    }
    void* ensure(size_t bytes) {
        if (bytes <= cap && p) return p;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        // mapped + coherent: small results are also written straight into it by kernels (device
        // address from dev()), read by the host after the stream is synchronised
        HGA_HIP(hipHostMalloc(&p, bytes ? bytes : 16, hipHostMallocMapped | hipHostMallocCoherent));
        cap = bytes ? bytes : 16;
        HGA_HIP(hipHostGetDevicePointer(&dp, p, 0));
        return p;
    }
    void* dp = nullptr;   // device address of p
    // device address of host address h inside the buffer
    template <class T>
    T* dev(T* h) const {
        return reinterpret_cast<T*>(static_cast<char*>(dp) + (reinterpret_cast<char*>(h) - static_cast<char*>(p)));
    }
};

// Per-kernel event timing on the ctx stream (hga_profile_*).
struct Profiler {
    bool on = false;
    std::vector<std::string> only;   // if non-empty: time only these launch names
    struct Rec { std::string name; hipEvent_t a, b; };
    std::vector<Rec> pending;
    std::vector<hipEvent_t> pool;
    std::map<std::string, std::pair<double, uint64_t>> acc;

    hipEvent_t get() {
        if (!pool.empty()) { hipEvent_t e = pool.back(); pool.pop_back(); return e; }
        hipEvent_t e;
        HGA_HIP(hipEventCreate(&e));
        return e;
    }
    void drain() {
        for (auto& r : pending) {
            float ms = 0.f;
            HGA_HIP(hipEventSynchronize(r.b));
            HGA_HIP(hipEventElapsedTime(&ms, r.a, r.b));
            auto& s = acc[r.name];
            s.first += ms;
            s.second += 1;
            pool.push_back(r.a);
            pool.push_back(r.b);
        }
        pending.clear();
    }
    ~Profiler() {
        for (auto& r : pending) { (void)hipEventDestroy(r.a); (void)hipEventDestroy(r.b); }
        for (auto e : pool) (void)hipEventDestroy(e);
    }
};

struct CountState {
    bool begun = false, ran = false;
    int k = 0;
    uint32_t n_files = 0;
    uint32_t min_per_file = 2;
    // per-file resident sequence bytes
    std::vector<DevBuf*> seq;
    std::vector<uint64_t> seq_len;
    // pipeline scratch
    DevBuf file_start, cursor2, fine_hist, regions, binned1, binned, rows_key, rows_cnt, cursor, scratch,
        sel_keys, sel_tmp, sel_wtmp, hist_dense, hist_comp, xch, xch2, nblk, bin_files, blist,
        binned3, file_start3, xsend, xrecv, xdir, xsrc, xslab, xemit, xrbase, xdir_b;
    char xemit_host[64] = {};   // the XbEmit last uploaded to xemit (count.hip)
    // error bits of the last failed settle / histogram (proto::QE_*), so the global queries can report
    // them in their gathered words (comm.hip)
    uint64_t last_err = 0;
    // the export's code range of this rank after count_export_repartition (comm.hip): keys then
    // flags (u32, k = 32); sel_rep_n = ~0 until the current selection is re-partitioned
    DevBuf sel_rep;
    uint64_t sel_rep_n = ~0ull;
    PinnedBuf xsrc_h;           // the owner merge's run table, staged for upload (exchange.hip)
    PinnedBuf xpack_h;          // count counters + per-owner piece totals of count_xb_pack
    std::vector<uint64_t> l1_exact;   // exact level-1 region sizes after an overflowing attempt
    uint64_t instances = 0, rows = 0, rows_cap = 0, n_sel = 0;
    uint32_t sel_grid = 0;   // kc_select workgroups: as many as are resident at once (count.hip)
    uint64_t g_instances = 0, g_bytes = 0, g_rows = 0;   // over all ranks (set by count_exchange)
    bool g_rows_pending = false;   // g_rows' all-gather enqueued, not summed yet (count_global_rows)
    int g_rows_P = 0;
    PinnedBuf g_rows_h;
    std::vector<char> tab_host;
    std::vector<double> thr_dev;   // thresholds last uploaded next to the histogram (count_spec_hist)   // last uploaded per-file tables
    // pre-counted dump rows per file (hga_count_add_rows), merged verbatim at the end of count_run
    std::vector<std::vector<uint64_t>> dump_keys;
    std::vector<std::vector<uint32_t>> dump_cnt;
    uint32_t buckets = 0, fb = 0, max_split = 1;
    uint64_t listed = 0;   // buckets kc_count_s left to the generic kernel (per-file run >= 65536)
    // exchange emission of the last count_run (kc_count_s XbEmit): pieces in xslab by count bucket,
    // counts per (bucket, sub-bin) in xdir at resolution xb_R = fb + xb_x, for xb_P ranks
    bool xb_on = false;
    uint32_t xb_P = 0, xb_x = 0, xb_nbc = 0;
    int xb_R = 0;
    const uint64_t* xb_fs = nullptr;
    const void* xb_dev = nullptr;    // the XbEmit in device memory
    uint64_t xb_cap = 0;             // rows_key / rows_cnt capacity of that run
    bool dense_pending = false;      // rows_key / rows_cnt not written yet (count_dense)
    bool pending = false;   // count_run's counters not read back yet (count_settle)
    bool dist = false;      // rows are this rank's owner range after hga_count_exchange
    ~CountState() {
        for (auto* b : seq) delete b;
    }
};

struct LookupState {
    bool loaded = false, have_reads = false, ran = false;
    uint64_t kci_epoch = 0;   // bumped whenever kci_ptr / kci_val change (connect.hip's list slots follow it)
    bool packed_ok = false;   // packed / valid / starts / word_read hold the current reads (lookup_pack)
    int k = 0, km = 0;
    uint32_t n_sdk = 0;
    uint64_t slots = 0, fwords = 0, pk_words = 0;   // slots = table buckets
    uint32_t idb = 0;   // packed table entries: KmerID bits (0: 64-B buckets)
    DevBuf tab_key, tab_id, filter, packed, valid, starts, word_read, win_kid;
    uint64_t n_reads = 0, n_bases = 0;
    uint32_t first_read_id = 1;
    DevBuf bases, offsets;
    // results
    DevBuf tile_cnt, hit_read, hit_kid, hit_pos, hit_ptr, s_key, s_val, s_key2, s_val2,
        first_flag, first_kid, first_pos, first_read, first_ptr, kci_key, kci_val, kci_ptr, kci_tmp, scratch,
        scratch2, scratch3, big_list, hll_part;
    std::vector<uint64_t> h_offsets;
    uint64_t windows = 0, hits = 0, firsts = 0, reads_hit = 0;
    // hga_lookup_gather: the results hold the whole input's index; this rank's own read set is kept
    bool gathered = false;
    uint64_t loc_n_reads = 0;
    uint32_t loc_first_read_id = 1;
};

struct ConnState {
    bool ready = false;
    uint64_t n = 0, cap_hint = 0;
    // cn_wave's per-KmerID list slots (connect.hip cn_slots), built for the index of kci_epoch
    DevBuf slots;
    uint64_t slots_epoch = ~0ull;
    DevBuf piv, cat, ctr, rpre, ovf, ovf2, big, x, y, s, gk, gv, key, idx, skey, pos, ox, oy, os, og, pst, pcnt, sk2, sv2,
        lst;
};

// Multi-GPU transport of one rank (comm.hip): RCCL over xGMI, or a caller's host-staged hook.
struct Comm {
    int rank = 0, nranks = 1;
    int root = -1;   // hga_comm_set_root: gathered lists on this rank only (-1: every rank)
    DevBuf stage;   // device staging of host-memory collectives over RCCL (grow-only: no hipMalloc per call)
    PinnedBuf hstage;   // their host side
    virtual ~Comm() = default;
    // true: alltoallv moves device memory (RCCL); false: host memory (the caller stages)
    virtual bool on_device() const = 0;
    // Collective: send_bytes[p] bytes at send[p] go to rank p; recv_bytes[p] bytes from rank p land at
    // recv[p].  Every rank calls it in the same order.
    virtual void alltoallv(hga_ctx* c, const void* const* send, const uint64_t* send_bytes, void* const* recv,
                           const uint64_t* recv_bytes) = 0;
};

}  // namespace hga

struct hga_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    // a second stream for work that overlaps the main stream's (lookup.hip: kmer_component_index beside
    // the per-read sorts), forked and joined with these two events; created on first use
    hipStream_t side = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    hipStream_t side_stream() {
        if (!side) {
            HGA_HIP(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
            HGA_HIP(hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming));
            HGA_HIP(hipEventCreateWithFlags(&ev_join, hipEventDisableTiming));
        }
        return side;
    }
    int num_cu = 256;
    hga::Profiler prof;
    hga::CountState count;
    hga::LookupState lookup;
    hga::ConnState conn;
    hga::PinnedBuf pinned;   // small host<->device staging (see count_spec_hist)
    hga::PinnedBuf pinned_sel;   // count_select counters + top-digit histogram
    std::unique_ptr<hga::Comm> comm;   // hga_comm_init*: the count results become global
    // single-pass scans (sort.hip sc_onepass): per-tile status words tagged with the scan's epoch,
    // and a tile counter that only ever grows (its value at a launch is passed as the tile base)
    hga::DevBuf scan_state;
    uint64_t scan_tiles = 0;
    uint32_t scan_epoch = 0;

    // Launch helper: records events around the launch when profiling is on.
    template <class F>
    void launch(const char* name, F&& f) {
        if (!prof.on || (!prof.only.empty() &&
                         std::find(prof.only.begin(), prof.only.end(), name) == prof.only.end())) {
            f();
            return;
        }
        hipEvent_t a = prof.get(), b = prof.get();
        HGA_HIP(hipEventRecord(a, stream));
        f();
        HGA_HIP(hipEventRecord(b, stream));
        prof.pending.push_back({name, a, b});
        if (prof.pending.size() > 4096) prof.drain();
    }
    // the same on another stream (events recorded on that stream)
    template <class F>
    void launch_on(const char* name, hipStream_t s, F&& f) {
        if (!prof.on || (!prof.only.empty() &&
                         std::find(prof.only.begin(), prof.only.end(), name) == prof.only.end())) {
            f();
            return;
        }
        hipEvent_t a = prof.get(), b = prof.get();
        HGA_HIP(hipEventRecord(a, s));
        f();
        HGA_HIP(hipEventRecord(b, s));
        prof.pending.push_back({name, a, b});
        if (prof.pending.size() > 4096) prof.drain();
    }
    void check_launch(const char* name) {
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) throw hga::Error(HGA_ERR_HIP, std::string(name) + ": " + hipGetErrorString(e));
    }
    void sync() { HGA_HIP(hipStreamSynchronize(stream)); }
};

// Entry points implemented in count.hip / lookup.hip (called from api.hip).
namespace hga {
void count_begin(hga_ctx* c, int k, uint32_t n_files);
void count_add(hga_ctx* c, uint32_t file, const char* seq, uint64_t n);
void count_run(hga_ctx* c, uint32_t min_per_file);
// before_publish (optional): called once the histogram's (threshold << 56 | total, count) pairs are
// compacted on the device (ctrl[0] overflow rows, ctrl[2] pairs), before the call's one
// synchronisation — the multi-GPU gather enqueues its collective there
using SpecHook = std::function<void(const unsigned long long* d_ctrl, const unsigned long long* d_pairs)>;
void count_spec_hist(hga_ctx* c, const double* thr, uint32_t n_thr, std::vector<int64_t>& out,
                     const SpecHook* before_publish = nullptr);
// before_sync (optional): called with the device counters [n, n_discriminative] once kc_select has
// been enqueued, before the call's one synchronisation (the multi-GPU sum enqueues its collective)
using SelHook = std::function<void(const unsigned long long* d_stat)>;
void count_select(hga_ctx* c, int64_t lower, int64_t upper, uint64_t* n, uint64_t* n_discr,
                  const SelHook* before_sync = nullptr);
void count_fetch_selected(hga_ctx* c, uint64_t* dst, uint8_t* flags);
void count_rows(hga_ctx* c, int file, std::vector<uint64_t>& keys, std::vector<uint32_t>& counts);
void count_partition(hga_ctx* c, const uint64_t* splitters, uint32_t n_own, uint64_t* keys_out,
                     uint32_t* counts_out, uint64_t* rows_per_owner);
void count_merge(hga_ctx* c, const uint64_t* keys, const uint32_t* counts, uint64_t n, uint32_t min_c);
void connections_run(hga_ctx* c, const uint32_t* pivots, uint64_t n_piv, uint32_t min_kmers, uint64_t min_score,
                     const int32_t* categories, uint64_t* n_out);
void connections_fetch(hga_ctx* c, uint32_t* x, uint32_t* y, uint64_t* score, uint8_t* is_good, uint64_t first = 0,
                       uint64_t count = ~0ull);
void count_add_rows(hga_ctx* c, uint32_t file, const uint64_t* keys, const uint32_t* counts, uint64_t n);
int count_pack_bits(hga_ctx* c);
uint64_t count_partition_packed(hga_ctx* c, const uint64_t* splitters, uint32_t n_own, uint64_t* out,
                                uint64_t cap_out, uint64_t* pieces_per_owner, bool sync_out = true);
void count_merge_packed(hga_ctx* c, const uint64_t* pieces, uint64_t n, uint32_t min_c);
// hash-bucket exchange (exchange.hip; protocol in exchange_protocol.hpp): the sender's pieces in
// bucket order in `xsend` and its per-bucket counts in `xdir` (returns the resolution R), and the
// owner's merge of every sender's runs of its buckets
int count_xb_pack(hga_ctx* c, uint32_t P, uint64_t* per_owner);
// its fast path in two halves (count kernels that wrote the pieces): begin enqueues the per-owner
// totals into d_per (false: not applicable, nothing enqueued); finish gathers the pieces once the
// count is settled and the totals are on the host
bool count_xb_pack_begin(hga_ctx* c, uint32_t P, uint64_t* d_per);
int count_xb_pack_finish(hga_ctx* c, uint32_t P, const uint64_t* per_owner);
void count_xb_merge(hga_ctx* c, const uint64_t* in, const uint64_t* self, const uint64_t* n_from, const uint64_t* dir_in,
                    const int* r_from, uint32_t P, uint32_t me, uint32_t min_c);

// comm.hip: multi-GPU counting (hga_comm_*, hga_count_exchange) and the global query answers
void comm_init_rccl(hga_ctx* c, const void* id, int rank, int nranks);
void comm_init_host(hga_ctx* c, int rank, int nranks, const hga_transport* t);
void comm_allgather(hga_ctx* c, const void* mine, uint64_t bytes, void* all);
std::vector<std::vector<char>> comm_allgatherv(hga_ctx* c, const void* mine, uint64_t bytes);
std::vector<std::vector<char>> comm_gatherv_root(hga_ctx* c, const void* mine, uint64_t bytes, int root);
void comm_set_root(hga_ctx* c, int root);
bool comm_is_gather_leaf(hga_ctx* c);
void comm_alltoallv_dev(hga_ctx* c, const void* send, const uint64_t* sb, void* recv, const uint64_t* rb,
                        bool keep_self = true);
std::vector<uint64_t> owner_splitters(int k, int P);
void count_exchange(hga_ctx* c, uint32_t min_per_file);
uint64_t count_global_rows(hga_ctx* c);
void count_spec_hist_global(hga_ctx* c, const double* thr, uint32_t n_thr, std::vector<int64_t>& out);
void count_select_global(hga_ctx* c, int64_t lower, int64_t upper, uint64_t* n, uint64_t* nd);
void count_fetch_selected_global(hga_ctx* c, std::vector<uint64_t>& keys, std::vector<uint8_t>& flags);
// this rank's code range of the global export on the device (count.sel_rep), its size (comm.hip)
uint64_t count_export_repartition(hga_ctx* c);
// all merged rows ascending into malloc'ed buffers (hga_count_rows, count.hip)
void count_rows_to(hga_ctx* c, uint64_t** keys, uint32_t** counts, uint64_t* n_rows);
// the merged rows ascending on the device (count.hip): keys[rows], counts row-major [rows][F]
void count_rows_device(hga_ctx* c, DevBuf& keys, DevBuf& counts);
void count_rows_global(hga_ctx* c, int file, std::vector<uint64_t>& keys, std::vector<uint32_t>& counts);
void lookup_gather(hga_ctx* c);
void connections_gather(hga_ctx* c, uint64_t* n);

void lookup_load(hga_ctx* c, int k, const uint64_t* keys, uint32_t n);
void lookup_set_reads(hga_ctx* c, const char* bases, const uint64_t* offsets, uint64_t n,
                      uint32_t first_id);
void lookup_run(hga_ctx* c);
void lookup_pack(hga_ctx* c, bool skip_codes = false);   // per-base encode of the resident reads (lookup_run, hll_registers)
void lookup_sizes(hga_ctx* c, hga_lookup_sizes* out);
void lookup_fetch(hga_ctx* c, const hga_lookup_result* out);
void hll_registers(hga_ctx* c, int k, int b, uint8_t* regs);

// radix sort (sort.hip): stable LSD sort of `n` keys by their low `bits` bits, with an
// optional u32 payload.  Result ends in keys/vals (scratch used as ping-pong).
void radix_sort_u64(hga_ctx* c, uint64_t* keys, uint32_t* vals, uint64_t n, int bits,
                    DevBuf& scratch);
// keys <- src_k sorted by the low `bits` bits (src_k is left intact)
void radix_sort_u64_from(hga_ctx* c, const uint64_t* src_k, uint64_t* keys, uint64_t n, int bits, DevBuf& scratch);
void radix_sort_u32(hga_ctx* c, uint32_t* keys, uint32_t* vals, uint64_t n, int bits,
                    DevBuf& scratch);
// the same with the input read from src_k / src_v (left intact), the result in keys / vals
void radix_sort_u32_from(hga_ctx* c, const uint32_t* src_k, const uint32_t* src_v, uint32_t* keys, uint32_t* vals,
                         uint64_t n, int bits, DevBuf& scratch);
// exclusive scan of u64 in place (sort.hip)
void exclusive_scan_u64(hga_ctx* c, uint64_t* data, uint64_t n, DevBuf& scratch);
// status words + tile-id counter for one chained scan of nt tiles (kmer_dev.hpp chained_lookback)
struct ScanTicket {
    unsigned long long* status;
    unsigned long long* ctr;
    uint64_t tbase;
    uint32_t epoch;
};
ScanTicket scan_ticket(hga_ctx* c, uint64_t nt);
void count_settle(hga_ctx* c, const unsigned long long* h = nullptr);
void count_dense(hga_ctx* c);
// stable per-segment sort by the low kbits of sk (lookup.hip); false when a segment passes 16384
bool segment_sort(hga_ctx* c, const uint64_t* hptr, uint64_t nseg, uint64_t maxlen, int kbits, uint64_t* sk,
                  uint32_t* sv, DevBuf& list_buf, unsigned long long* ctr2, const char* label,
                  uint32_t* lists = nullptr, const unsigned long long* lists_n = nullptr);
void sort_export_u64(hga_ctx* c, uint64_t* keys, uint64_t n, int shift, uint32_t dbase, const uint32_t* d_hist,
                     const uint32_t* h_hist, DevBuf& scratch);
}  // namespace hga
