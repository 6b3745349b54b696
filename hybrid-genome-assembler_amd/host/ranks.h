// ranks.h — one hga_ctx per GPU inside one process, for the CLIs' `--gpus N` mode.
//
// Rank r runs on device (dev0 + r) mod #devices with its own HIP stream.  By default the ranks exchange
// through an in-process host transport (hga_comm_init_host): the threads meet at a barrier and copy
// each other's slices (verified on hardware: tests/test_cli_gpu.py, --gpus 2/3 equal one GPU).  With
// HGA_COMM=rccl and every rank on its own device they share an RCCL communicator over xGMI
// (hga_comm_unique_id + hga_comm_init, one thread per rank) — opt-in until a multi-GPU run of the CLIs
// has recorded parity (bench.py --gpus N checks the RCCL exchange against the oracle on every N > 1
// run).  Collective library calls are issued by Ranks::each, one thread per rank.
#pragma once

#include <barrier>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "hga.h"

namespace hgah {

// All-to-all-v between the rank threads of one process (host memory).
class LocalTransport {
   public:
    explicit LocalTransport(int n) : slots_(n), bar_(n), eps_(n) {
        for (int r = 0; r < n; ++r) eps_[r] = {this, r};
    }
    hga_transport transport(int rank) { return hga_transport{&eps_[rank], &LocalTransport::alltoallv}; }

   private:
    struct Slot {
        const void* const* send = nullptr;
        const uint64_t* bytes = nullptr;
    };
    struct Ep {
        LocalTransport* t;
        int rank;
    };
    static int alltoallv(void* user, const void* const* send, const uint64_t* sb, void* const* recv,
                         const uint64_t* rb) {
        Ep* e = static_cast<Ep*>(user);
        LocalTransport* t = e->t;
        t->slots_[e->rank] = {send, sb};
        t->bar_.arrive_and_wait();   // every rank's send list is published
        int bad = 0;
        for (size_t p = 0; p < t->slots_.size(); ++p) {
            const Slot& s = t->slots_[p];
            if (s.bytes[e->rank] != rb[p]) bad = 1;
            else if (rb[p]) std::memcpy(recv[p], s.send[e->rank], rb[p]);
        }
        t->bar_.arrive_and_wait();   // every copy out of the send buffers is done
        return bad;
    }
    std::vector<Slot> slots_;
    std::barrier<> bar_;
    std::vector<Ep> eps_;
};

class Ranks {
   public:
    std::vector<hga_ctx*> ctx;

    Ranks(int n, int dev0) {
        if (n < 1) throw std::invalid_argument("--gpus must be >= 1");
        int nd = 0;
        check(hga_device_count(&nd), "hga_device_count");
        if (nd < 1) throw std::runtime_error("no HIP device");
        const char* cm = std::getenv("HGA_COMM");
        const bool host = n > nd || !(cm && std::string(cm) == "rccl");
        ctx.assign(n, nullptr);
        for (int r = 0; r < n; ++r) check(hga_ctx_create(&ctx[r], (dev0 + r) % nd), "hga_ctx_create");
        if (n == 1) return;
        if (host) {
            local_ = std::make_unique<LocalTransport>(n);
            for (int r = 0; r < n; ++r) {
                tr_.push_back(local_->transport(r));
            }
            for (int r = 0; r < n; ++r) check(hga_comm_init_host(ctx[r], r, n, &tr_[r]), "hga_comm_init_host");
        } else {
            std::vector<char> uid(HGA_UNIQUE_ID_BYTES);
            check(hga_comm_unique_id(uid.data()), "hga_comm_unique_id");
            each([&](int r, hga_ctx* c) { check(hga_comm_init(c, uid.data(), r, n), "hga_comm_init"); });
        }
    }
    ~Ranks() {
        for (auto* c : ctx) hga_ctx_destroy(c);
    }
    int size() const { return (int)ctx.size(); }

    // fn(rank, ctx) on every rank at once (collective calls); a failure ends the process, since the
    // other ranks may be waiting inside a collective for the one that failed.
    void each(const std::function<void(int, hga_ctx*)>& fn) {
        if (ctx.size() == 1) {
            fn(0, ctx[0]);
            return;
        }
        std::vector<std::thread> th;
        for (int r = 0; r < size(); ++r)
            th.emplace_back([&, r] {
                try {
                    fn(r, ctx[r]);
                } catch (const std::exception& e) {
                    std::fprintf(stderr, "rank %d: %s\n", r, e.what());
                    std::fflush(stderr);
                    std::_Exit(EXIT_FAILURE);
                }
            });
        for (auto& t : th) t.join();
    }

    static void check(hga_status s, const char* what) {
        if (s != HGA_OK) throw std::runtime_error(std::string(what) + ": " + hga_last_error());
    }

   private:
    std::unique_ptr<LocalTransport> local_;
    std::vector<hga_transport> tr_;
};

// [begin, end) of rank r's contiguous share of a '\n'-separated read stream (cut after separators
// so no read is split).
inline std::pair<uint64_t, uint64_t> shard_of(const char* s, uint64_t n, int r, int P) {
    auto cut = [&](int i) -> uint64_t {
        if (i <= 0) return 0;
        if (i >= P) return n;
        uint64_t c = n * (uint64_t)i / (uint64_t)P;
        while (c < n && s[c] != '\n') ++c;
        return c < n ? c + 1 : n;
    };
    return {cut(r), cut(r + 1)};
}

}  // namespace hgah
