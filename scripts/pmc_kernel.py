"""Average each PMC counter per kernel (name substring) over dispatches from
rocprofv3 --pmc csv outputs: python scripts/pmc_kernel.py <substr> run_counter_collection.csv..."""
import csv
import sys
from collections import defaultdict


def main():
    sub = sys.argv[1]
    agg = defaultdict(list)
    meta = {}
    for path in sys.argv[2:]:
        with open(path) as f:
            for r in csv.DictReader(f):
                if sub not in r["Kernel_Name"]:
                    continue
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
                meta = {k: r[k] for k in ("Grid_Size", "Workgroup_Size", "LDS_Block_Size", "VGPR_Count",
                                           "SGPR_Count", "Scratch_Size")}
    print(meta)
    for k, v in sorted(agg.items()):
        print(f"{k:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")


if __name__ == "__main__":
    main()
