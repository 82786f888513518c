#!/usr/bin/env python3
"""cfg4 encode spread probe: per-call encode / decode times
of config 4's 44 GiB batch under different allocation histories, in one process.

  A  cfg4 allocated first in a fresh process
  B  after cfg3's batch (6.3 GB) was allocated, used and freed (the bench order)
  C  the same cfg4 batch re-used after B, data re-synthesised
  D  cfg3 allocated in the memory cfg4's batch freed
  E  cfg3 first in a fresh process
Prints one JSON line per phase: per-call HIP-event ms (min / median / max) and
the batch's base address (2 MiB / 1 GiB alignment)."""
from __future__ import annotations

import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quic-fec-eps_amd"))

import torch  # noqa: E402

import fecgpu  # noqa: E402
from fecgpu import workloads  # noqa: E402


def timed(fn, n):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in evs:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return [a.elapsed_time(b) for a, b in evs]


def summary(xs):
    return {"n": len(xs), "min": round(min(xs), 4), "med": round(statistics.median(xs), 4),
            "max": round(max(xs), 4), "first5": [round(x, 3) for x in xs[:5]]}


def phase(name, ctx, b, n=20, warm=3):
    for _ in range(warm):
        b.encode(ctx)
        b.decode(ctx)
    torch.cuda.synchronize()
    enc = timed(lambda: b.encode(ctx), n)
    dec = timed(lambda: b.decode(ctx), n)
    alt = []
    for _ in range(n // 2):  # bench's alternation: encode right after decode
        a = timed(lambda: b.encode(ctx), 1)
        b.decode(ctx)
        alt += a
    ptr = b.win.data_ptr()
    print(json.dumps({"phase": name, "encode": summary(enc), "decode": summary(dec),
                      "encode_alternating": summary(alt), "base": hex(ptr),
                      "base_mod_2M": ptr % (2 << 20), "base_mod_1G": ptr % (1 << 30),
                      "t": time.strftime("%H:%M:%S")}), flush=True)


def make(cid, ctx, dev):
    c = workloads.CONFIGS[cid]
    b = workloads.Batch.allocate(c, c.nwin_per_gpu, dev)
    b.synthesize(ctx, 0)
    b.make_erasures(ctx, 0)
    return b


def main():
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    ctx = fecgpu.Context()
    order = sys.argv[1] if len(sys.argv) > 1 else "ABC"
    b4 = None
    for ph in order:
        if ph == "A":
            b4 = make(4, ctx, dev)
            phase("A-cfg4-first", ctx, b4)
        elif ph == "B":
            del b4
            b4 = None
            torch.cuda.empty_cache()
            b3 = make(3, ctx, dev)
            phase("B0-cfg3", ctx, b3, n=10)
            del b3
            torch.cuda.empty_cache()
            b4 = make(4, ctx, dev)
            phase("B-cfg4-after-cfg3", ctx, b4)
        elif ph == "C":
            b4.synthesize(ctx, 0)
            phase("C-cfg4-again", ctx, b4)
        elif ph == "D":  # cfg3 in the memory cfg4 freed
            del b4
            b4 = None
            torch.cuda.empty_cache()
            b3 = make(3, ctx, dev)
            phase("D-cfg3-after-cfg4", ctx, b3, n=10)
            del b3
            torch.cuda.empty_cache()
        elif ph == "E":  # cfg3 first in a fresh process
            b3 = make(3, ctx, dev)
            phase("E-cfg3-first", ctx, b3, n=10)
            del b3
            torch.cuda.empty_cache()
    ctx.close()


if __name__ == "__main__":
    main()
