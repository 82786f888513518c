#!/usr/bin/env python3
"""Average rocprofv3 --pmc counters per fecgpu kernel: pmc_summary.py gpurun_out/<dir> ..."""
import collections
import csv
import sys

for d in sys.argv[1:]:
    rows = list(csv.DictReader(open(f"{d}/run_counter_collection.csv")))
    agg = collections.defaultdict(list)
    for r in rows:
        n = r["Kernel_Name"]
        if "fecgpu" in n and ("encode" in n or "decode" in n):
            agg[(n.split("(")[0].replace("void fecgpu::", ""), r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(agg.items()):
        print(f"{d.split('/')[-1]:8s} {k:32s} {c:22s} n={len(v):2d} avg={sum(v)/len(v):.4g}")
