#!/usr/bin/env python3
"""Sliding-window RLC (fecgpu_sw_*) throughput on one GPU — a DESIGN.md measurement,
not the driver's bench line.

Stream: nsrc sources of L bytes (device-resident), a repair after every k sources
over the last W (RFC 8681, dt 15).  Encode: GB/s of source bytes, and the
algorithmic HBM rate (sources read once + repairs written once; the W/k-fold
re-reads of each source are served by L2).  Decode: i.i.d. loss of sources and
repairs; the call's wall time (host split into linked systems + device kernels,
synchronous) per lost source and per source byte.
  python scripts/sw_bench.py [--nsrc 524288] [--k 8] [--W 32] [--loss 0.02]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quic-fec-eps_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import fecgpu  # noqa: E402


def schedule(nsrc, k, W, key0=0, dt=15):
    a = np.zeros(nsrc // k, fecgpu.SW_REPAIR_DTYPE)
    end = (np.arange(nsrc // k, dtype=np.int64) + 1) * k
    fss = np.maximum(0, end - W)
    a["fss"], a["nss"], a["key"], a["dt"] = fss, end - fss, (key0 + np.arange(len(a))) & 0xFFFF, dt
    return a


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nsrc", type=int, default=524288)
    ap.add_argument("--L", type=int, default=1200)
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--W", type=int, default=32)
    ap.add_argument("--loss", type=float, default=0.02)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--sw-group", type=int, default=0, help="tuning: repairs per encode job (0 = library default)")
    args = ap.parse_args()
    nsrc, L, k, W = args.nsrc, args.L, args.k, args.W
    stride = (L + 15) // 16 * 16
    ctx = fecgpu.Context()
    if args.sw_group:
        ctx.set_tuning("sw_group", args.sw_group)
    g = torch.Generator(device="cuda").manual_seed(1)
    src = torch.randint(0, 256, (nsrc, stride), dtype=torch.uint8, device="cuda", generator=g)
    hdr = schedule(nsrc, k, W)
    nrep = len(hdr)
    d_hdr = torch.from_numpy(hdr.view(np.uint8).copy()).cuda()
    rep = torch.empty((nrep, stride), dtype=torch.uint8, device="cuda")

    def enc():
        ctx.sw_encode(src, rep, d_hdr, nsrc=nsrc, nrep=nrep, sym_len=L, stride=stride, max_window=W)

    for _ in range(3):
        enc()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        enc()
    e1.record()
    torch.cuda.synchronize()
    enc_ms = e0.elapsed_time(e1) / args.iters

    rng = np.random.default_rng(2)
    sp = (rng.random(nsrc) >= args.loss).astype(np.uint8)
    rp = (rng.random(nrep) >= args.loss).astype(np.uint8)
    orig = src.clone()
    lost_t = torch.from_numpy(sp == 0).cuda()
    st = np.zeros(nsrc, np.uint8)
    times = []
    for i in range(5):
        src.copy_(orig)
        src[lost_t] = 0
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = ctx.sw_decode(src, sp, rep, rp, hdr, st, nsrc=nsrc, nrep=nrep, sym_len=L, stride=stride)
        times.append(time.perf_counter() - t0)
    ok = torch.from_numpy(st == 0).cuda()
    verified = bool(torch.equal(src[ok], orig[ok]))
    dec_ms = sorted(times)[len(times) // 2] * 1e3
    nlost = int((sp == 0).sum())
    alg = (nsrc + nrep) * L
    print(json.dumps({
        "what": "sliding-window RLC (RFC 8681), device-resident symbols",
        "nsrc": nsrc, "L": L, "k": k, "W": W, "nrep": nrep, "sw_group": args.sw_group or 4,
        "encode_ms": round(enc_ms, 4), "encode_src_GBps": round(nsrc * L / enc_ms / 1e6, 1),
        "encode_alg_TBps": round(alg / enc_ms / 1e9, 3),
        "loss": args.loss, "lost": nlost, "recovered": n, "verify_ok": verified,
        "decode_wall_ms": round(dec_ms, 3), "decode_us_per_lost": round(dec_ms * 1e3 / max(1, nlost), 3),
        "decode_src_GBps": round(nsrc * L / dec_ms / 1e6, 1),
    }))


if __name__ == "__main__":
    main()
