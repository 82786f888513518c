#!/usr/bin/env python3
"""In-process A/B of libfecgpu builds: every variant library is loaded side by
side (separate ctypes handles, one HIP runtime), all run on the same device
batch, interleaved round by round — cross-process clock/DVFS variance drops out.

  python scripts/ab.py --config 2 --libs quic-fec-eps_amd/lib/libfecgpu.so,quic-fec-eps_amd/lib/libfecgpu_x.so
Tuning aid, not part of the product.
"""
import argparse
import importlib.util
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "quic-fec-eps_amd")
sys.path.insert(0, PKG)

import torch  # noqa: E402

import fecgpu  # noqa: E402  (default library; provides Batch / configs)
from fecgpu import workloads  # noqa: E402


def load_variant(path: str, tag: str):
    """A second copy of the fecgpu package bound to another library file."""
    os.environ["FECGPU_LIB"] = path
    spec = importlib.util.spec_from_file_location(f"fecgpu_{tag}", os.path.join(PKG, "fecgpu", "__init__.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[spec.name] = mod  # dataclasses resolve annotations through sys.modules
    spec.loader.exec_module(mod)
    del os.environ["FECGPU_LIB"]
    return mod


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--libs", required=True)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--bpc", type=int, default=0)
    ap.add_argument("--alt", action="store_true",
                    help="also time alternating encode/decode pairs (the bench's step)")
    args = ap.parse_args()
    # entries: path[@bpc] or path@key=val:key=val (fecgpu_ctx_set_tuning keys);
    # the same library may appear several times with different knobs
    entries = args.libs.split(",")
    libs = [e.split("@")[0] for e in entries]
    mods = [load_variant(p, str(i)) for i, p in enumerate(libs)]
    ctxs = [m.Context() for m in mods]
    for c, e in zip(ctxs, entries):
        knobs = e.split("@")[1] if "@" in e else (str(args.bpc) if args.bpc else "")
        for kv in filter(None, knobs.split(":")):
            key, val = kv.split("=") if "=" in kv else ("blocks_per_cu", kv)
            c.set_tuning(key, int(val))
    cfg = workloads.CONFIGS[args.config]
    b = workloads.Batch.allocate(cfg, cfg.nwin_per_gpu, torch.device("cuda"))
    b.synthesize(ctxs[0], 0)
    b.make_erasures(ctxs[0], 0)
    alg = b.algorithmic_bytes()
    src = b.source_bytes()
    res = [{"encode": [], "decode": [], "pair": []} for _ in libs]

    def timed(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.steps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / args.steps

    for c in ctxs:  # warm every variant (tables, code objects)
        b.encode(c)
        b.decode(c)
    for _ in range(args.rounds):
        for i, c in enumerate(ctxs):
            res[i]["encode"].append(timed(lambda: b.encode(c)))
            res[i]["decode"].append(timed(lambda: b.decode(c)))
            if args.alt:
                res[i]["pair"].append(timed(lambda: (b.encode(c), b.decode(c))))
    # the buffer must still decode correctly with the last variant
    ver = b.verify(ctxs[-1], 0)
    for i, p in enumerate(entries):
        e = statistics.median(res[i]["encode"])
        d = statistics.median(res[i]["decode"])
        print(json.dumps({"lib": os.path.basename(p), "config": args.config,
                          "enc_ms": round(e, 4), "dec_ms": round(d, 4),
                          "enc_min": round(min(res[i]["encode"]), 4),
                          "dec_min": round(min(res[i]["decode"]), 4),
                          "enc_TBps": round(alg["encode"] / e / 1e9, 3),
                          "dec_TBps": round(alg["decode"] / d / 1e9, 3),
                          "src_GBps": round(src / (e + d) / 1e6, 1), "verify_ok": ver["ok"],
                          **({"pair_ms": round(statistics.median(res[i]["pair"]), 4)} if args.alt else {})}),
              flush=True)


if __name__ == "__main__":
    main()
