#!/usr/bin/env python3
"""Measured HBM stream rates on this MI355X (denominators beside the 8 TB/s spec).

copy: torch's device copy of a 4 GiB buffer (read + write bytes / time);
read: a 4 GiB int64 sum (read bytes / time).  Median of 10 after warmup.
"""
import json
import sys

import torch


def timed(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e-3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    n = 4 << 30
    src = torch.randint(0, 255, (n,), dtype=torch.uint8, device="cuda")
    dst = torch.empty_like(src)
    t = timed(lambda: dst.copy_(src))
    copy = 2 * n / t / 1e9
    v = src.view(torch.int64)
    t = timed(lambda: v.sum())
    read = n / t / 1e9
    print(json.dumps({"copy_GBps": round(copy, 1), "read_GBps": round(read, 1),
                      "bytes": n, "device": torch.cuda.get_device_name(0)}))


if __name__ == "__main__":
    sys.exit(main())
