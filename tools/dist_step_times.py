#!/usr/bin/env python3
"""Wall time of each call of one distributed count step (bench.py dist_count_step) at one rank with
the library's RCCL communicator (no torch process group needed: a one-rank unique id):
count_run(1) | count_exchange(2) | spec_hist | select_device, each followed by a device sync.

    python tools/dist_step_times.py [--self-p2p]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hybrid-genome-assembler_amd")]
import bench  # noqa: E402
import hga  # noqa: E402

if "--self-p2p" in sys.argv:
    os.environ["HGA_RCCL_SELF"] = "1"
ga, gb, ra, rb = bench.make_c2(0)
ctx = hga.Ctx(0)
ctx.comm_init(hga.comm_unique_id(), 0, 1)
ctx.count_begin(19, 2)
ctx.count_add(0, ra.seq)
ctx.count_add(1, rb.seq)
calls = [("count_run(1)", lambda: ctx.count_run(1)), ("count_exchange(2)", lambda: ctx.count_exchange(2)),
         ("spec_hist", lambda: ctx.spec_hist(bench.THRESHOLDS)), ("select_device", lambda: ctx.select_device(10, 25))]
acc = {n: [] for n, _ in calls}
whole = []
for it in range(14):
    ctx.sync()
    t00 = time.perf_counter()
    for n, f in calls:
        t0 = time.perf_counter()
        f()
        ctx.sync()
        acc[n].append(time.perf_counter() - t0)
    whole.append(time.perf_counter() - t00)
print({n: round(float(np.median(v[4:])) * 1e3, 3) for n, v in acc.items()},
      "step ms", round(float(np.median(whole[4:])) * 1e3, 3), flush=True)
# per-kernel device time of the exchange (event-timed launches, 5 steps)
names = ["kc_count", "kx_xb_hist", "kx_xb_pack", "kx_xb_scatter", "kx_xb_gather", "kx_xb_units", "kx_xb_merge",
         "kx_mb_compact", "scan"]
ctx.profile(True)
ctx.profile_reset()
for it in range(5):
    for n, f in calls:
        f()
ctx.sync()
print({n: round(ctx.profile_get(n)[0] / 5, 4) for n in names},
      "(ms per step)", flush=True)
ctx.close()
