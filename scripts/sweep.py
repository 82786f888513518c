#!/usr/bin/env python3
"""In-process launch-knob sweep: for each workgroups-per-CU setting, time
encode and decode of a BASELINE config (interleaved rounds, one process, so the
comparison is not cross-process noise).  Tuning aid, not part of the product.

  python scripts/sweep.py --config 2 --bpc 0,2,3,4,6,8 --rounds 3
(bpc 0 = the library's automatic choice)
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quic-fec-eps_amd"))

import torch  # noqa: E402

import fecgpu  # noqa: E402
from fecgpu import workloads  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--bpc", default="0,2,3,4,6,8")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    cfg = workloads.CONFIGS[args.config]
    ctx = fecgpu.Context()
    b = workloads.Batch.allocate(cfg, cfg.nwin_per_gpu, torch.device("cuda"))
    b.synthesize(ctx, 0)
    b.make_erasures(ctx, 0)
    alg = b.algorithmic_bytes()
    src = b.source_bytes()
    bpcs = [int(x) for x in args.bpc.split(",")]
    res = {v: {"encode": [], "decode": []} for v in bpcs}

    def timed(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.steps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / args.steps

    for _ in range(args.rounds):
        for v in bpcs:
            ctx.set_tuning("blocks_per_cu", v)
            b.encode(ctx)
            b.decode(ctx)
            res[v]["encode"].append(timed(lambda: b.encode(ctx)))
            res[v]["decode"].append(timed(lambda: b.decode(ctx)))
    lib = os.path.basename(fecgpu.LIB_PATH)
    for v in bpcs:
        e = statistics.median(res[v]["encode"])
        d = statistics.median(res[v]["decode"])
        print(json.dumps({"lib": lib, "config": args.config, "bpc": v,
                          "enc_ms": round(e, 4), "dec_ms": round(d, 4),
                          "enc_TBps": round(alg["encode"] / e / 1e9, 3),
                          "dec_TBps": round(alg["decode"] / d / 1e9, 3),
                          "src_GBps": round(src / (e + d) / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
