#!/usr/bin/env python3
"""Encode / decode throughput across code shapes on one MI355X (device-resident,
S = 1200 B FIXED, exactly r sources erased per window, ~1.2 GB of windows per
shape), with the kernel the library picks for each: XOR, GF table multiply,
compiled bit-sliced masks, runtime-mask bit-slicing.  HIP events around 10
encodes / 10 decodes after 3 warm-ups; TB/s of algorithmic bytes ((k + r) * S
per window for encode; (k + e) * S for decode, e = r).  Verifies every window.
One JSON line per (scheme, matrix, k, r)."""
import dataclasses
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quic-fec-eps_amd"))

import torch  # noqa: E402

import fecgpu  # noqa: E402
from fecgpu import workloads  # noqa: E402

SHAPES = [("xor", "cauchy", 4, 1), ("xor", "cauchy", 8, 2), ("xor", "cauchy", 16, 4),
          ("gf256", "cauchy", 4, 2), ("gf256", "cauchy", 8, 2), ("gf256", "cauchy", 10, 4),
          ("gf256", "cauchy", 16, 4), ("gf256", "cauchy", 20, 5), ("gf256", "cauchy", 24, 6),
          ("gf256", "cauchy", 12, 8), ("gf256", "cauchy", 16, 8), ("gf256", "cauchy", 32, 8),
          ("gf256", "cauchy", 48, 8), ("gf256", "rlc", 16, 4), ("gf256", "rlc", 32, 8),
          ("gf256", "vandermonde", 32, 8)]


def kernel_name(ctx_bs: bool, scheme, matrix, k, r):
    if scheme == "xor":
        return "xor"
    if (k, r) in ((16, 8), (24, 8), (32, 8)) and matrix in ("cauchy", "vandermonde"):
        return "bit-sliced (compiled masks)"
    return "bit-sliced (runtime masks)" if r >= 5 else "table multiply"


def main():
    only = sys.argv[1] if len(sys.argv) > 1 else ""  # "rbs": the runtime-mask shapes only
    ctx = fecgpu.Context()
    dev = torch.device("cuda")
    base = workloads.CONFIGS[3]
    for scheme, matrix, k, r in SHAPES:
        if only == "rbs" and kernel_name(True, scheme, matrix, k, r) != "bit-sliced (runtime masks)":
            continue
        if only == "r8" and (scheme != "gf256" or r != 8):  # the e = r = 8 decode rows
            continue
        if only.startswith("shape=") and only[6:] != f"{scheme}-{matrix}-{k}-{r}":  # e.g. shape=gf256-cauchy-32-8
            continue
        stride = 1216
        nwin = int(1.2e9 // ((k + r) * stride))
        cfg = dataclasses.replace(base, name=f"{scheme}-{matrix}-k{k}r{r}", scheme=scheme, k=k, r=r,
                                  nwin_per_gpu=nwin, matrix=matrix, erasure=workloads.ERASURE_EXACT)
        b = workloads.Batch.allocate(cfg, nwin, dev)
        b.synthesize(ctx, 0)
        b.make_erasures(ctx, 0)
        for _ in range(3):
            b.encode(ctx)
            b.decode(ctx)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        ev[0].record()
        for _ in range(10):
            b.encode(ctx)
        ev[1].record()
        for _ in range(10):
            b.decode(ctx)
        ev[2].record()
        torch.cuda.synchronize()
        enc = ev[0].elapsed_time(ev[1]) / 10
        dec = ev[1].elapsed_time(ev[2]) / 10
        alg = b.algorithmic_bytes()
        v = b.verify(ctx, 0)
        print(json.dumps({"scheme": scheme, "matrix": matrix, "k": k, "r": r, "windows": nwin,
                          "encode_kernel": kernel_name(True, scheme, matrix, k, r),
                          "encode_ms": round(enc, 4), "decode_ms": round(dec, 4),
                          "encode_TBps": round(alg["encode"] / enc / 1e9, 3),
                          "decode_TBps": round(alg["decode"] / dec / 1e9, 3),
                          "src_GBps_enc_dec": round(nwin * k * cfg.L / (enc + dec) / 1e6, 1),
                          "verify_ok": v["ok"], "unrecoverable": v["unrecoverable"]}), flush=True)
        del b
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
