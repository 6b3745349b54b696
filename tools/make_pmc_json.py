#!/usr/bin/env python3
"""Turn a pmc_summary JSON (FETCH_SIZE/WRITE_SIZE passes) into one profiles-style file per kernel:
pmc_<kernel>.json = {"hbm_bytes_per_launch", "read_bytes", "write_bytes", "ms_median", ...}.
bench.py reads profiles/pmc_<kernel>.json for roofline.traffic.

    python tools/make_pmc_json.py gpurun_out/hbm_r01.json out_dir
"""
import json
import os
import re
import sys


def main(src, out_dir):
    d = json.load(open(src))
    os.makedirs(out_dir, exist_ok=True)
    for k, row in d.items():
        base = re.sub(r"<.*", "", k)
        rd, wr = row["read_bytes_corr"], row["write_bytes"]
        rec = {"kernel": k, "hbm_bytes_per_launch": int(rd + wr), "read_bytes": int(rd), "write_bytes": int(wr),
               "ms_median": row["ms_median"], "dispatches": row["dispatches"],
               "note": "FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, KB->B, mean over dispatches; "
                       "separate --pmc passes over tools/kprof.py (MI355X_MICROARCH.md HBM section)"}
        name = f"pmc_{base}.json"
        p = os.path.join(out_dir, name)
        # keep the heaviest instantiation when a template kernel has several
        if os.path.exists(p) and json.load(open(p))["hbm_bytes_per_launch"] > rec["hbm_bytes_per_launch"]:
            continue
        json.dump(rec, open(p, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
