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


def per_call_wide(path, counter):
    """Wide codes (k + r > 64, `--k`): bytes per encode / decode CALL.  In
    dispatch order a decode is wide_dec_plan_kernel, the stage-1 bit-sliced
    pass (gf_encode_rbs_kernel right after the plan) and the stage-2 combine
    pass; an encode is a gf_encode_rbs_kernel on its own."""
    rows = [r for r in csv.DictReader(open(f"{path}/run_counter_collection.csv")) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    enc, dec = [], []
    cur = None  # the decode call being summed
    for r in rows:
        n, v = r["Kernel_Name"], float(r["Counter_Value"])
        if "fecgpu" not in n:
            continue
        if "wide_dec_plan_kernel" in n or "gf_decode_bs_plan_kernel" in n:
            cur = [v, False]
            dec.append(cur)
        elif "gf_encode_rbs_kernel" in n and cur is not None and not cur[1]:
            cur[0] += v
            cur[1] = True  # stage 1 of the current decode
        elif ("comb_kernel" in n or "gf_decode_bs_kernel" in n) and cur is not None:
            cur[0] += v
            cur = None
        elif "gf_encode_rbs_kernel" in n:
            enc.append(v)
    out = {}
    if enc:
        out["encode"] = statistics.median(enc)
    if dec:
        out["decode"] = statistics.median([d[0] for d in dec])
    return out


def per_kernel(path, counter, config):
    if config == "wide":
        return per_call_wide(path, counter)
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
    ap.add_argument("--config", required=True, help="config id, or 'wide' (bench.py --k K --r R)")
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    if a.config != "wide":
        a.config = int(a.config)
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
