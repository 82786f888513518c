#!/usr/bin/env python3
"""HBM traffic per launch of the fecgpu kernels from two rocprofv3 --pmc passes.

  python scripts/pmc_traffic.py --config 2 --fetch gpurun_out/pmc2r --write gpurun_out/pmc2w \
         --out profiles/r01_cfg2_traffic.json

MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) reports exactly half the bytes of a
wide coalesced streaming read on gfx950, so read bytes = 2 x FETCH_SIZE x 1024;
WRITE_SIZE (KB) is exact for 16-B-per-lane streaming stores.  FETCH_SIZE and
WRITE_SIZE are collected in separate passes (they do not fit one TCC pass).
"""
import argparse
import collections
import csv
import json
import statistics


def kind(name, config):
    """encode / decode / None for a kernel name (config 7, sliding window: the
    encode is sw_stream_kernel; every combine launch belongs to the decode —
    syndromes comb_kernel<1>, solves comb_kernel<4>)."""
    if "fecgpu" not in name:
        return None
    if config == 7:  # the streaming encode (the default); the decode's chain, its combine passes included
        if "sw_stream_kernel" in name:
            return "encode"
        return "decode" if ("sw_dec_" in name or "comb_kernel<" in name) else None
    return "encode" if "encode" in name else "decode" if "decode" in name else None


def per_kernel(path, counter, config):
    out = collections.defaultdict(list)
    calls = 0  # config 7: decode calls (one plan kernel each, or header kernel unfused); the chain summed per call
    for r in csv.DictReader(open(f"{path}/run_counter_collection.csv")):
        if r["Counter_Name"] != counter:
            continue
        if config == 7 and ("sw_dec_plan_kernel" in r["Kernel_Name"] or "sw_dec_hdr_kernel" in r["Kernel_Name"]):
            calls += 1
        kd = kind(r["Kernel_Name"], config)
        if kd:
            out[kd].append(float(r["Counter_Value"]))
    res = {k: statistics.median(v) for k, v in out.items()}
    if config == 7 and calls and "decode" in out:
        res["decode"] = sum(out["decode"]) / calls
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    f = per_kernel(a.fetch, "FETCH_SIZE", a.config)
    w = per_kernel(a.write, "WRITE_SIZE", a.config)
    res = {"config": a.config, "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes; "
           "read = 2 x FETCH_SIZE x 1024 (gfx950 correction), write = WRITE_SIZE x 1024",
           "kernels": {}}
    for k in sorted(set(f) | set(w)):
        rd = 2 * f.get(k, 0) * 1024
        wr = w.get(k, 0) * 1024
        res["kernels"][k] = {"read_bytes": int(rd), "write_bytes": int(wr), "traffic_bytes": int(rd + wr)}
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
