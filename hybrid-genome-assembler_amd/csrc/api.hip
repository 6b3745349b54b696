// api.hip — the extern "C" surface declared in include/hga.h.  Catches every
// exception and maps it to an hga_status + thread-local message.
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "hga_internal.hpp"

namespace {
thread_local std::string g_err;

template <class F>
hga_status guard(F&& f) {
    // a body that returns a value on one path would fall off its end on the others (undefined)
    static_assert(std::is_void<decltype(f())>::value, "guarded bodies return nothing");
    try {
        g_err.clear();
        f();
        return HGA_OK;
    } catch (const hga::Error& e) {
        g_err = e.what();
        return e.code;
    } catch (const std::bad_alloc&) {
        g_err = "host allocation failed";
        return HGA_ERR_OOM;
    } catch (const std::exception& e) {
        g_err = e.what();
        return HGA_ERR_INVALID;
    }
}

hga_status need_ctx(hga_ctx* c) {
    if (!c) {
        g_err = "null context";
        return HGA_ERR_INVALID;
    }
    return HGA_OK;
}

template <class T>
T* host_dup(const T* src, size_t n) {
    T* p = static_cast<T*>(std::malloc(n ? n * sizeof(T) : 1));
    if (!p) throw std::bad_alloc();
    if (n) std::memcpy(p, src, n * sizeof(T));
    return p;
}
}  // namespace

#define HGA_CTX_GUARD(c, ...)                               \
    do {                                                    \
        if (need_ctx(c) != HGA_OK) return HGA_ERR_INVALID;  \
        return guard([&] {                                  \
            HGA_HIP(hipSetDevice((c)->device));             \
            __VA_ARGS__;                                    \
        });                                                 \
    } while (0)

extern "C" {

const char* hga_last_error(void) { return g_err.c_str(); }
void hga_free(void* p) { std::free(p); }
const char* hga_version(void) { return "hga-mi355x 0.1 (gfx950)"; }

hga_status hga_device_count(int* n) {
    return guard([&] {
        HGA_REQUIRE(n, HGA_ERR_INVALID, "null out pointer");
        int d = 0;
        HGA_HIP(hipGetDeviceCount(&d));
        *n = d;
    });
}

hga_status hga_ctx_create(hga_ctx** out, int device) {
    return guard([&] {
        HGA_REQUIRE(out, HGA_ERR_INVALID, "null out pointer");
        int nd = 0;
        HGA_HIP(hipGetDeviceCount(&nd));
        HGA_REQUIRE(device >= 0 && device < nd, HGA_ERR_INVALID, "no such HIP device");
        HGA_HIP(hipSetDevice(device));
        auto* c = new hga_ctx();
        c->device = device;
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
            c->num_cu = prop.multiProcessorCount;
        hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
        if (e != hipSuccess) {
            delete c;
            throw hga::Error(HGA_ERR_HIP, std::string("hipStreamCreate: ") + hipGetErrorString(e));
        }
        *out = c;
    });
}

hga_status hga_ctx_destroy(hga_ctx* c) {
    if (!c) return HGA_OK;
    return guard([&] {
        (void)hipSetDevice(c->device);
        (void)hipStreamSynchronize(c->stream);
        if (c->side) (void)hipStreamSynchronize(c->side);
        hipStream_t s = c->stream, s2 = c->side;
        hipEvent_t e1 = c->ev_fork, e2 = c->ev_join;
        delete c;
        (void)hipStreamDestroy(s);
        if (s2) {
            (void)hipEventDestroy(e1);
            (void)hipEventDestroy(e2);
            (void)hipStreamDestroy(s2);
        }
    });
}

hga_status hga_count_begin(hga_ctx* c, int k, uint32_t n_files) {
    HGA_CTX_GUARD(c, hga::count_begin(c, k, n_files));
}

hga_status hga_count_add(hga_ctx* c, uint32_t file, const char* seq, uint64_t n_bytes) {
    HGA_CTX_GUARD(c, {
        HGA_REQUIRE(seq || n_bytes == 0, HGA_ERR_INVALID, "null sequence pointer");
        hga::count_add(c, file, seq, n_bytes);
    });
}

hga_status hga_connections_run(hga_ctx* c, const uint32_t* pivots, uint64_t n_pivots, uint32_t min_kmers,
                               uint64_t min_score, const int32_t* categories, uint64_t* n) {
    HGA_CTX_GUARD(c, {
        HGA_REQUIRE(n, HGA_ERR_INVALID, "null out pointer");
        HGA_REQUIRE(pivots || n_pivots == 0, HGA_ERR_INVALID, "null pivots with n_pivots > 0");
        hga::connections_run(c, pivots, n_pivots, min_kmers, min_score, categories, n);
    });
}

hga_status hga_connections_fetch(hga_ctx* c, uint32_t* x, uint32_t* y, uint64_t* score, uint8_t* is_good) {
    HGA_CTX_GUARD(c, hga::connections_fetch(c, x, y, score, is_good));
}

hga_status hga_connections_fetch_range(hga_ctx* c, uint64_t first, uint64_t count, uint32_t* x, uint32_t* y,
                                       uint64_t* score, uint8_t* is_good) {
    HGA_CTX_GUARD(c, hga::connections_fetch(c, x, y, score, is_good, first, count));
}

hga_status hga_count_add_rows(hga_ctx* c, uint32_t file, const uint64_t* keys, const uint32_t* counts,
                              uint64_t n) {
    HGA_CTX_GUARD(c, hga::count_add_rows(c, file, keys, counts, n));
}

hga_status hga_count_run(hga_ctx* c, uint32_t min_per_file) {
    HGA_CTX_GUARD(c, hga::count_run(c, min_per_file));
}

hga_status hga_count_get_stats(hga_ctx* c, hga_count_stats* out) {
    HGA_CTX_GUARD(c, {
        HGA_REQUIRE(out, HGA_ERR_INVALID, "null out pointer");
        auto& s = c->count;
        hga::count_settle(c);
        HGA_REQUIRE(s.ran, HGA_ERR_STATE, "hga_count_run not called");
        out->instances = s.instances;
        out->distinct_rows = s.rows;
        uint64_t b = 0;
        for (auto l : s.seq_len) b += l;
        out->bytes = b;
        if (s.dist) {   // after hga_count_exchange: the whole input over all ranks (no collective)
            out->distinct_rows = hga::count_global_rows(c);
            out->instances = s.g_instances;
            out->bytes = s.g_bytes;
        }
        out->buckets = s.buckets;
        out->max_split = s.max_split;
    });
}

hga_status hga_count_spec_hist(hga_ctx* c, const double* thr, uint32_t n_thr, int64_t** triples,
                               uint64_t* n) {
    HGA_CTX_GUARD(c, {
        HGA_REQUIRE(thr && triples && n, HGA_ERR_INVALID, "null pointer");
        std::vector<int64_t> v;
        if (c->count.dist) hga::count_spec_hist_global(c, thr, n_thr, v);
        else hga::count_spec_hist(c, thr, n_thr, v);
        *triples = host_dup(v.data(), v.size());
        *n = v.size() / 3;
    });
}

hga_status hga_count_select(hga_ctx* c, int64_t lower, int64_t upper, uint64_t** keys, uint64_t* n,
                            uint64_t* n_discriminative) {
    HGA_CTX_GUARD(c, {
        HGA_REQUIRE(keys && n && n_discriminative, HGA_ERR_INVALID, "null pointer");
        uint64_t m = 0, d = 0;
        if (c->count.dist) {
            hga::count_select_global(c, lower, upper, &m, &d);
            std::vector<uint64_t> k;
            std::vector<uint8_t> f;
            hga::count_fetch_selected_global(c, k, f);
            *keys = host_dup(k.data(), k.size());
            const bool leaf = hga::comm_is_gather_leaf(c);   // (hga_comm_set_root: an empty list here)
            *n = leaf ? 0 : m;
            *n_discriminative = leaf ? 0 : d;
            return;
        }
        hga::count_select(c, lower, upper, &m, &d);
        uint64_t* out = static_cast<uint64_t*>(std::malloc(m ? m * 8 : 8));
        if (!out) throw std::bad_alloc();
        hga::count_fetch_selected(c, out, nullptr);
        *keys = out;
        *n = m;
        *n_discriminative = d;
    });
}

hga_status hga_count_select_ex(hga_ctx* c, int64_t lower, int64_t upper, uint64_t** keys, uint8_t** disc,
                               uint64_t* n, uint64_t* n_discriminative) {
    HGA_CTX_GUARD(c, {
        HGA_REQUIRE(keys && disc && n && n_discriminative, HGA_ERR_INVALID, "null pointer");
        uint64_t m = 0, d = 0;
        if (c->count.dist) {
            hga::count_select_global(c, lower, upper, &m, &d);
            std::vector<uint64_t> k;
            std::vector<uint8_t> f;
            hga::count_fetch_selected_global(c, k, f);
            *keys = host_dup(k.data(), k.size());
            *disc = host_dup(f.data(), f.size());
            const bool leaf = hga::comm_is_gather_leaf(c);   // (hga_comm_set_root: an empty list here)
            *n = leaf ? 0 : m;
            *n_discriminative = leaf ? 0 : d;
            return;
        }
        hga::count_select(c, lower, upper, &m, &d);
        uint64_t* out = static_cast<uint64_t*>(std::malloc(m ? m * 8 : 8));
        uint8_t* fl = static_cast<uint8_t*>(std::malloc(m ? m : 1));
        if (!out || !fl) { std::free(out); std::free(fl); throw std::bad_alloc(); }
        hga::count_fetch_selected(c, out, fl);
        *keys = out;
        *disc = fl;
        *n = m;
        *n_discriminative = d;
    });
}

hga_status hga_count_select_device(hga_ctx* c, int64_t lower, int64_t upper, uint64_t* n,
                                   uint64_t* n_discriminative) {
    HGA_CTX_GUARD(c, {
        HGA_REQUIRE(n && n_discriminative, HGA_ERR_INVALID, "null pointer");
        if (c->count.dist) hga::count_select_global(c, lower, upper, n, n_discriminative);
        else hga::count_select(c, lower, upper, n, n_discriminative);
    });
}

hga_status hga_count_partition(hga_ctx* c, const uint64_t* splitters, uint32_t n_owners, uint64_t* keys_out,
                               uint32_t* counts_out, uint64_t* rows_per_owner) {
    HGA_CTX_GUARD(c, {
        HGA_REQUIRE(rows_per_owner && (n_owners <= 1 || splitters), HGA_ERR_INVALID, "null pointer");
        hga::count_partition(c, splitters, n_owners, keys_out, counts_out, rows_per_owner);
    });
}

hga_status hga_count_merge(hga_ctx* c, const uint64_t* keys, const uint32_t* counts, uint64_t n,
                           uint32_t min_per_file) {
    HGA_CTX_GUARD(c, { hga::count_merge(c, keys, counts, n, min_per_file); });
}

hga_status hga_count_pack_bits(hga_ctx* c, int* bits) {
    HGA_CTX_GUARD(c, {
        HGA_REQUIRE(bits, HGA_ERR_INVALID, "null pointer");
        HGA_REQUIRE(c->count.begun, HGA_ERR_STATE, "hga_count_begin not called");
        hga::count_settle(c);   // (a failed count reports here)
        *bits = hga::count_pack_bits(c);
    });
}

hga_status hga_count_partition_packed(hga_ctx* c, const uint64_t* splitters, uint32_t n_owners, uint64_t* out,
                                      uint64_t capacity, uint64_t* pieces_per_owner, uint64_t* total) {
    HGA_CTX_GUARD(c, {
        HGA_REQUIRE(pieces_per_owner && total && (n_owners <= 1 || splitters), HGA_ERR_INVALID, "null pointer");
        *total = hga::count_partition_packed(c, splitters, n_owners, out, capacity, pieces_per_owner);
        HGA_REQUIRE(*total <= capacity, HGA_ERR_OOM, "output capacity too small (see *total)");
    });
}

hga_status hga_count_merge_packed(hga_ctx* c, const uint64_t* pieces, uint64_t n, uint32_t min_per_file) {
    HGA_CTX_GUARD(c, { hga::count_merge_packed(c, pieces, n, min_per_file); });
}

hga_status hga_count_rows(hga_ctx* c, uint64_t** keys, uint32_t** counts, uint64_t* rows) {
    HGA_CTX_GUARD(c, {
        HGA_REQUIRE(keys && counts && rows, HGA_ERR_INVALID, "null pointer");
        // (no early return: the guarded lambda returns void on every path)
        if (!c->count.dist) {   // sorted on the device, copied straight into the returned buffers
            hga::count_rows_to(c, keys, counts, rows);
        } else {
            std::vector<uint64_t> k;
            std::vector<uint32_t> v;
            hga::count_rows_global(c, -1, k, v);
            *keys = host_dup(k.data(), k.size());
            *counts = host_dup(v.data(), v.size());
            *rows = k.size();
        }
    });
}

hga_status hga_count_dump(hga_ctx* c, uint32_t file, uint64_t** keys, uint32_t** counts, uint64_t* rows) {
    HGA_CTX_GUARD(c, {
        HGA_REQUIRE(keys && counts && rows, HGA_ERR_INVALID, "null pointer");
        HGA_REQUIRE(file < c->count.n_files, HGA_ERR_INVALID, "file index out of range");
        std::vector<uint64_t> k;
        std::vector<uint32_t> v;
        if (c->count.dist) hga::count_rows_global(c, (int)file, k, v);
        else hga::count_rows(c, (int)file, k, v);
        *keys = host_dup(k.data(), k.size());
        *counts = host_dup(v.data(), v.size());
        *rows = k.size();
    });
}

hga_status hga_lookup_load(hga_ctx* c, int k, const uint64_t* keys, uint32_t n) {
    HGA_CTX_GUARD(c, {
        HGA_REQUIRE(keys || n == 0, HGA_ERR_INVALID, "null keys");
        hga::lookup_load(c, k, keys, n);
    });
}

hga_status hga_lookup_set_reads(hga_ctx* c, const char* bases, const uint64_t* offsets, uint64_t n_reads,
                                uint32_t first_read_id) {
    HGA_CTX_GUARD(c, {
        HGA_REQUIRE(offsets, HGA_ERR_INVALID, "null offsets");
        HGA_REQUIRE(bases || offsets[n_reads] == 0, HGA_ERR_INVALID, "null bases");
        hga::lookup_set_reads(c, bases, offsets, n_reads, first_read_id);
    });
}

hga_status hga_lookup_run(hga_ctx* c) { HGA_CTX_GUARD(c, hga::lookup_run(c)); }

hga_status hga_lookup_get_sizes(hga_ctx* c, hga_lookup_sizes* out) {
    HGA_CTX_GUARD(c, {
        HGA_REQUIRE(out, HGA_ERR_INVALID, "null out pointer");
        hga::lookup_sizes(c, out);
    });
}

hga_status hga_lookup_fetch(hga_ctx* c, const hga_lookup_result* out) {
    HGA_CTX_GUARD(c, {
        HGA_REQUIRE(out, HGA_ERR_INVALID, "null out pointer");
        hga::lookup_fetch(c, out);
    });
}

hga_status hga_hll_registers(hga_ctx* c, int k, uint32_t b, uint8_t* registers) {
    HGA_CTX_GUARD(c, {
        HGA_REQUIRE(registers, HGA_ERR_INVALID, "null registers");
        hga::hll_registers(c, k, (int)b, registers);
    });
}

hga_status hga_profile_enable(hga_ctx* c, int on) {
    HGA_CTX_GUARD(c, {
        c->prof.drain();
        c->prof.on = on != 0;
    });
}

hga_status hga_profile_select(hga_ctx* c, const char* names) {
    HGA_CTX_GUARD(c, {
        c->prof.drain();
        c->prof.only.clear();
        std::string cur;
        for (const char* p = names ? names : ""; ; ++p) {
            if (*p == ',' || *p == 0) {
                if (!cur.empty()) c->prof.only.push_back(cur);
                cur.clear();
                if (*p == 0) break;
            } else {
                cur += *p;
            }
        }
    });
}

hga_status hga_profile_reset(hga_ctx* c) {
    HGA_CTX_GUARD(c, {
        c->prof.drain();
        c->prof.acc.clear();
    });
}

hga_status hga_profile_get(hga_ctx* c, const char* name, double* ms, uint64_t* launches) {
    HGA_CTX_GUARD(c, {
        HGA_REQUIRE(name && ms && launches, HGA_ERR_INVALID, "null pointer");
        c->prof.drain();
        auto it = c->prof.acc.find(name);
        *ms = it == c->prof.acc.end() ? 0.0 : it->second.first;
        *launches = it == c->prof.acc.end() ? 0 : it->second.second;
    });
}

hga_status hga_sync(hga_ctx* c) { HGA_CTX_GUARD(c, c->sync()); }

hga_status hga_comm_init(hga_ctx* c, const void* unique_id, int rank, int nranks) {
    HGA_CTX_GUARD(c, hga::comm_init_rccl(c, unique_id, rank, nranks));
}

hga_status hga_comm_init_host(hga_ctx* c, int rank, int nranks, const hga_transport* t) {
    HGA_CTX_GUARD(c, hga::comm_init_host(c, rank, nranks, t));
}

hga_status hga_comm_info(hga_ctx* c, int* rank, int* nranks) {
    HGA_CTX_GUARD(c, {
        HGA_REQUIRE(rank && nranks, HGA_ERR_INVALID, "null pointer");
        *rank = c->comm ? c->comm->rank : 0;
        *nranks = c->comm ? c->comm->nranks : 1;
    });
}

hga_status hga_comm_set_root(hga_ctx* c, int root) {
    HGA_CTX_GUARD(c, { hga::comm_set_root(c, root); });
}

hga_status hga_comm_destroy(hga_ctx* c) {
    HGA_CTX_GUARD(c, {
        c->sync();
        c->comm.reset();
        c->count.dist = false;
    });
}

hga_status hga_count_exchange(hga_ctx* c, uint32_t min_per_file) {
    HGA_CTX_GUARD(c, hga::count_exchange(c, min_per_file));
}

hga_status hga_lookup_gather(hga_ctx* c) { HGA_CTX_GUARD(c, hga::lookup_gather(c)); }

hga_status hga_connections_gather(hga_ctx* c, uint64_t* n) {
    HGA_CTX_GUARD(c, {
        HGA_REQUIRE(n, HGA_ERR_INVALID, "null out pointer");
        hga::connections_gather(c, n);
    });
}

}  // extern "C"
