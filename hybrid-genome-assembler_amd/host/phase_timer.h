// phase_timer.h — HGA_TIMING=1 phase marks of the drop-in CLIs: "hga-timing <phase> <ms>" lines on
// stderr (bench.py reads them into `phases_ms`); stdout stays the reference's.
#pragma once

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>

namespace hgah {

struct PhaseTimer {
    bool on = false;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now(), last = t0;
    PhaseTimer() {
        if (const char* te = std::getenv("HGA_TIMING")) on = std::string(te) == "1";
    }
    void mark(const char* phase) {
        if (!on) return;
        const auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "hga-timing %s %.2f\n", phase, std::chrono::duration<double, std::milli>(now - last).count());
        last = now;
    }
    void total() {
        if (on)
            std::fprintf(stderr, "hga-timing total %.2f\n",
                         std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
};

}  // namespace hgah
