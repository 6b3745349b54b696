#!/usr/bin/env python3
"""Every counter of a set of rocprofv3 --pmc pass directories, per kernel (mean over dispatches),
for kernels matching the given substrings:  python tools/pmc_raw.py 'gpurun_out/pmc_x_*' kc_bin1 kc_count_s"""
import collections
import csv
import glob
import sys

pat, keys = sys.argv[1], sys.argv[2:]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(pat + "/*counter_collection.csv") + glob.glob(pat + "/*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        for k in keys:
            if k in r["Kernel_Name"]:
                agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in keys:
    print(k)
    for c, v in sorted(agg[k].items()):
        print(f"   {c:28s} {sum(v) / len(v):16.4g}")
