#!/usr/bin/env python3
"""Bit-sliced vs table-multiply GF encode, per compiled code (tuning aid).

  python scripts/bs_probe.py [--libs lib/libfecgpu.so,lib/libfecgpu_x.so] [--S 1200]
Device-resident uniform windows of ~1.5 GB; median of 5 rounds x 5 launches.
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
sys.path.insert(0, os.path.join(ROOT, "quic-fec-eps_amd"))
import torch  # noqa: E402

from ab import load_variant  # noqa: E402

CODES = [(16, 8), (24, 8), (32, 8)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="quic-fec-eps_amd/lib/libfecgpu.so")
    ap.add_argument("--S", type=int, default=1200)
    ap.add_argument("--codes", default="")
    ap.add_argument("--mixed", action="store_true", help="per-window S: alternate 1202 / S")
    ap.add_argument("--gb", type=float, default=1.5, help="window bytes on the device")
    args = ap.parse_args()
    codes = CODES if not args.codes else [tuple(map(int, c.split("x"))) for c in args.codes.split(",")]
    stride = (args.S + 15) // 16 * 16
    for li, lib in enumerate(args.libs.split(",")):
        m = load_variant(os.path.join(ROOT, lib), f"p{li}")
        ctx = m.Context()
        for k, r in codes:
            nwin = int(args.gb * 1e9 // ((k + r) * stride))
            d = torch.randint(0, 256, (nwin, k + r, stride), dtype=torch.uint8, device="cuda")
            code = m.Code("gf256", k, r)
            kw = dict(sym_len_all=args.S)
            if args.mixed:
                sl = torch.full((nwin,), args.S, dtype=torch.int32, device="cuda")
                sl[::2] = 1202
                kw = dict(sym_len=sl)
            res = {}
            for bs in (1, 0):
                ctx.set_tuning("bitslice", bs)
                ctx.encode_batch(code, d, nwin=nwin, stride=stride, **kw)
                torch.cuda.synchronize()
                ts = []
                for _ in range(5):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(5):
                        ctx.encode_batch(code, d, nwin=nwin, stride=stride, **kw)
                    e1.record()
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1) / 5)
                res[bs] = statistics.median(ts)
            alg = nwin * (k + r) * (args.S if not args.mixed else (args.S + 1202) / 2)
            print(json.dumps({"lib": os.path.basename(lib), "k": k, "r": r, "S": args.S, "nwin": nwin,
                              "bs_ms": round(res[1], 4), "tab_ms": round(res[0], 4),
                              "bs_TBps": round(alg / res[1] / 1e9, 3), "tab_TBps": round(alg / res[0] / 1e9, 3),
                              "speedup": round(res[0] / res[1], 3)}), flush=True)
            del d
        ctx.close()


if __name__ == "__main__":
    main()
