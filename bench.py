#!/usr/bin/env python3
"""bench.py — FEC encode+decode throughput on MI355X (BASELINE.json metric).

One step = one pass of the hot path over one batch: fecgpu_encode_batch over
every window (sender: repair generation) then fecgpu_decode_batch over every
window (receiver: recovery of the erased sources), inputs already resident in
HBM.  value = source-packet bytes (sum of packet lengths, no prefix or
padding) of all ranks x steps / max-over-ranks wall time.

Workloads (BASELINE.json configs):
  --config 2          : XOR k=8 r=2, 65,536 windows x 8 x 1200 B per GPU,
                        one source erased per XOR group (e = r = 2)
  --config 3 (default): GF(2^8) Cauchy k=16 r=4, 262,144 windows x 16 x 1200 B,
                        exactly r sources erased per window (the largest
                        device-resident BASELINE config that one GPU holds whole)
  --config 4          : GF(2^8) k=32 r=8, mixed MTU 1200/9000 LENPREFIX,
                        131,072 windows per GPU (1M over 8), i.i.d. 10% erasures
  --config 7          : sliding-window RLC (RFC 8681): 524,288 x 1200 B sources per
                        GPU, a repair after every 8 over the last 32, 2% i.i.d. loss
                        of sources and repairs (a widening row, not a BASELINE config)
The default run (one GPU, config 3) also times configs 2, 4, 5 and 7 in the
same process and reports them under "configs" in the same JSON line (each with
its own ms_per_step, roofline, cpu_baseline and verify); the headline fields
are config 3's.
Multi-GPU: one process per GPU, windows sharded by rank with no data-path
collective (weak scaling); RCCL only carries the barrier, the max-over-ranks
time reduction and the 8-byte digest all-gather.  `--gpus N` launched without
WORLD_SIZE (plain `python bench.py --gpus N`) starts the N ranks itself: a
torch.distributed.run child, spawned before this process touches the GPU.
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import os
import sys
import time

_ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(_ROOT, "quic-fec-eps_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import fecgpu  # noqa: E402
from fecgpu import shard, workloads  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
PCIE_DIR_PEAK_GBS = 63.0  # PCIe Gen5 x16, per direction (spec; MI355X_MICROARCH.md host link)
DEFAULT_CONFIG = 3
# config -> (steps, warmup) when --steps / --warmup are not given; cfg3 warms up
# longer (its first ~10 calls run slow while the clocks and TLBs settle)
DEFAULT_STEPS = {2: (200, 20), 3: (50, 10), 4: (5, 2), 5: (10, 2), 6: (10, 2), 7: (50, 10)}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 0 = the config's default (DEFAULT_STEPS): cfg3 50 steps of ~2.7 ms keep the
    # timed region (~0.14 s) well above barrier / launch jitter across ranks
    ap.add_argument("--steps", type=int, default=0)
    ap.add_argument("--warmup", type=int, default=-1)
    ap.add_argument("--config", type=int, default=DEFAULT_CONFIG, choices=sorted(workloads.CONFIGS))
    ap.add_argument("--nwin", type=int, default=0, help="windows per GPU (0 = config default)")
    ap.add_argument("--matrix", default="cauchy", choices=["cauchy", "vandermonde", "rlc"],
                    help="GF configs: parity rows (rlc: RFC 8681 random linear code, dense)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="target CPU work for the cpu_baseline sample (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--grid-mult", type=int, default=0, help="tuning: persistent grid multiplier")
    ap.add_argument("--bitslice", type=int, choices=[0, 1], default=None,
                    help="tuning: GF encode by the bit-sliced kernels (1, default) or the table multiply (0)")
    ap.add_argument("--bs-passes", type=int, default=0,
                    help="tuning: bit-sliced encode on per-window lengths, 256-unit passes per window group")
    ap.add_argument("--wpb", type=int, default=0, help="tuning: windows per workgroup")
    ap.add_argument("--gs", type=int, choices=[0, 1], default=None,
                    help="tuning: bit-sliced encode of short uniform rows with the repairs stored through LDS "
                         "(1, default) or the flat bit-sliced kernel (0)")
    ap.add_argument("--bpc", type=int, default=0, help="tuning: persistent workgroups per CU")
    ap.add_argument("--sw-long-min", type=int, default=0,
                    help="tuning (config 7): unknowns from which a linked system takes the banded long path")
    ap.add_argument("--sw-stream", type=int, default=-1, choices=[-1, 0, 1, 2, 3, 4, 5, 6],
                    help="sliding-window encode: 0 combine jobs, 1/2 streaming (dwords per lane); "
                         "-1 the library default")
    ap.add_argument("--sw-group", type=int, default=0, choices=[0, 1, 2, 4, 8],
                    help="tuning (config 7): sliding-window repairs per combine job (0 = library default)")
    ap.add_argument("--sw-loss", type=float, default=-1.0,
                    help="config 7: i.i.d. loss rate of sources and repairs (-1 = the config's 2 %%)")
    ap.add_argument("--sw-window", type=int, default=0,
                    help="config 7: repair window in sources (0 = the config's 32)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="N>1: nccl (= RCCL, one rank per GPU) or gloo (rehearsal: ranks may "
                         "share a GPU; the reductions run on the host)")
    ap.add_argument("--event-every", type=int, default=4,
                    help="bracket encode/decode with HIP events on every Nth timed step (0 = never): "
                         "each timestamped event costs ~3 us of GPU time, so sampling keeps the "
                         "wall-clock value unperturbed while kernels_ms stays measured live")
    ap.add_argument("--host-direct", type=int, default=-1,
                    help="tuning (config 5/6): kernels write outputs to mapped host memory, bit 0 encode, bit 1 decode")
    ap.add_argument("--host-chunk-mb", type=int, default=0, help="tuning (config 5/6): pipeline chunk size")
    ap.add_argument("--k", type=int, default=0,
                    help="GF codes wider than one mask (k + r > 64, fec_wide.hip): sources per window; with "
                         "--r, config 3's workload (1200-B packets, exactly r sources erased) on that code, "
                         "~5 GB of source bytes per GPU")
    ap.add_argument("--r", type=int, default=0, help="repairs per window for --k")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VAL",
                    help="tuning: fecgpu_ctx_set_tuning(KEY, VAL), repeatable")
    ap.add_argument("--extra-configs", type=int, choices=[0, 1], default=1,
                    help="default run (config 3): also time configs 2, 4, 5 and 7 in this process and "
                         "report them under \"configs\" (0 = config 3 only)")
    a = ap.parse_args()
    st, wu = DEFAULT_STEPS[a.config]
    a.steps = a.steps if a.steps > 0 else st
    a.warmup = a.warmup if a.warmup >= 0 else wu
    return a


def pmc_traffic(cfgid, kernel: str):
    """HBM bytes per launch of `kernel` (per call for the wide codes) from the
    newest committed rocprofv3 PMC summary for this config
    (profiles/rNN_cfgN_traffic.json, or rNN_cfgwideKrR_traffic.json for
    `--k K --r R`; written by scripts/pmc_traffic.py from separate FETCH_SIZE /
    WRITE_SIZE passes)."""
    import glob
    files = sorted(glob.glob(os.path.join(_ROOT, "profiles", f"r*_cfg{cfgid}_traffic.json")))
    if not files:
        return None, None
    try:
        d = json.load(open(files[-1]))
        return int(d["kernels"][kernel]["traffic_bytes"]), os.path.relpath(files[-1], _ROOT)
    except (KeyError, ValueError, OSError):
        return None, None


def log(msg: str) -> None:
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def host_share() -> int:
    """Host threads for the CPU baseline: every core this process may run on
    (sched_getaffinity), bounded by the CPU share the GPU pool grants one GPU's
    job (OMP_NUM_THREADS, 16 on the box: its nproc / cpu_count show the whole
    machine, whose other cores belong to other GPUs' jobs)."""
    n = len(os.sched_getaffinity(0))
    share = os.environ.get("OMP_NUM_THREADS", "")
    if share.isdigit() and int(share) > 0:
        n = min(n, int(share))
    return max(1, n)


def cpu_baseline(cfg, seconds: float, threads: int) -> dict:
    """Time the CPU codec (oracle/fec_cpu_simd.c: the oracle's contract with
    AVX2 nibble tables / GFNI affine products, ISA-L style; kind "port") on a
    bounded sample of the same workload: same packets, same erasure stream."""
    sys.path.insert(0, os.path.join(_ROOT, "oracle"))
    import oracle as O  # test/baseline infrastructure only

    O.lib()
    aff = len(os.sched_getaffinity(0))
    if threads <= 0:
        threads = host_share()
    scheme = (O.XOR if cfg.scheme == "xor" else O.RLC(cfg.rlc_key, cfg.rlc_dt) if cfg.matrix == "rlc"
              else O.GF256_VDM if cfg.matrix == "vandermonde" else O.GF256)
    win_bytes = (cfg.k + cfg.r) * cfg.stride
    max_nw = max(threads, (2 << 30) // win_bytes)  # sample buffer <= 2 GiB

    def make(nw: int):
        return O.make_batch(cfg.workload, workloads.SEED, 0, nw, scheme, cfg.erasure, cfg.k, cfg.r, cfg.L,
                            cfg.stride, threads)

    def run(batch):
        # encode then decode; a repeated pass does the same work on the same
        # windows (decode rebuilds the erased sources each time)
        wins, S, pres, _ = batch
        t0 = time.perf_counter()
        O.encode_batch_simd(scheme, cfg.k, cfg.r, S, wins, threads)
        O.decode_batch_simd(scheme, cfg.k, cfg.r, S, wins, pres, threads)
        return time.perf_counter() - t0

    nw = 4 * threads
    batch = make(nw)
    dt = run(batch)
    while dt < 0.25 and nw < max_nw:
        nw = min(max_nw, nw * 4)
        batch = make(nw)
        dt = run(batch)
    # scale to ~seconds of work; repeat the (built once) sample if it is still short
    per_win = dt / nw
    want = min(max_nw, max(nw, int(seconds / per_win)))
    if want != nw:
        nw, batch = want, make(want)
    reps = min(1000, max(1, int(seconds / (per_win * nw) + 0.5)))
    tot_dt, tot_src = 0.0, 0
    for _ in range(reps):
        tot_dt += run(batch)
        tot_src += batch[3]
        if tot_dt >= seconds:
            break
    dt, src = tot_dt, tot_src
    del batch
    return {"value": round(src / dt / 1e9, 4), "unit": "GB/s", "cores": threads, "kind": "port",
            "host_cores": {"affinity": aff, "cpu_count": os.cpu_count(), "used": threads,
                           "share_env": os.environ.get("OMP_NUM_THREADS")},
            "codec": f"oracle/fec_cpu_simd.c ({O.SIMD_NAMES[O.simd_level()]}; equal outputs to the "
                     f"scalar oracle: tests/test_oracle_simd.py)",
            "sample": f"{nw} windows of {cfg.name} (encode+decode, same packets and erasures; "
                      f"the sample repeated {reps}x at most), {dt:.1f} s on {threads} host threads"}


def cpu_baseline_wide(cfg, seconds: float, threads: int = 0) -> dict:
    """Codes with k + r > 64 (--k / --r): the CPU codec (oracle/fec_cpu_simd.c,
    multi-word present masks; outputs equal to the numpy restatement,
    tests/test_oracle_simd.py) on a bounded sample of the same shape: windows
    of k sources of L random bytes, exactly r sources erased per window."""
    import numpy as np
    sys.path.insert(0, os.path.join(_ROOT, "oracle"))
    import oracle as O  # test/baseline infrastructure only

    O.lib()
    if threads <= 0:
        threads = host_share()
    k, r, L, n = cfg.k, cfg.r, cfg.L, cfg.k + cfg.r
    stride = O.round_up(L, 16)
    nwin = max(threads, int((1 << 30) // (n * stride)))  # ~1 GiB sample
    rng = np.random.default_rng(workloads.SEED)
    wins = np.zeros((nwin, n, stride), np.uint8)
    wins[:, :k, :L] = rng.integers(0, 256, (nwin, k, L), dtype=np.uint8)
    S = np.full(nwin, L, np.uint32)
    nw = (n + 63) // 64
    pres = np.zeros((nwin, nw), np.uint64)
    for q in range(nw):
        lo, hi = 64 * q, min(n, 64 * q + 64)
        pres[:, q] = np.uint64((1 << (hi - lo)) - 1) if hi - lo < 64 else np.uint64(2**64 - 1)
    for w in range(nwin):
        for j in rng.choice(k, r, replace=False):
            pres[w, j // 64] &= ~np.uint64(1 << (j % 64))
    tot, reps = 0.0, 0
    while tot < seconds and reps < 1000:
        t0 = time.perf_counter()
        O.encode_batch_simd(O.GF256, k, r, S, wins, threads)
        O.decode_batch_simd(O.GF256, k, r, S, wins, pres, threads)
        tot += time.perf_counter() - t0
        reps += 1
    return {"value": round(reps * nwin * k * L / tot / 1e9, 4), "unit": "GB/s", "cores": threads, "kind": "port",
            "codec": f"oracle/fec_cpu_simd.c ({O.SIMD_NAMES[O.simd_level()]}; k + r up to 256, multi-word masks; "
                     f"equal outputs to np_oracle: tests/test_oracle_simd.py)",
            "sample": f"{reps} passes over {nwin} windows of k {k} r {r} x {L} B (exactly r sources erased), "
                      f"{tot:.1f} s on {threads} host threads"}


def cpu_baseline_sw(cfg, seconds: float, threads: int = 0, nsrc: int = 0) -> dict:
    """Config 7: the sliding-window CPU codec (oracle/fec_cpu_simd.c
    orc_sw_encode_simd / orc_sw_decode_simd: AVX2 / GFNI products, threads over
    repairs and over runs of whole linked systems; outputs equal to the oracle,
    tests/test_oracle_simd.py) on the config's own stream shape (nsrc sources,
    a repair every k over the last W, the same i.i.d. loss), repeated until
    ~seconds of CPU time; kind "port"."""
    import numpy as np
    sys.path.insert(0, os.path.join(_ROOT, "oracle"))
    import oracle as O  # test/baseline infrastructure only

    O.lib()
    if threads <= 0:
        threads = host_share()
    n = nsrc or cfg.nwin_per_gpu * cfg.k
    L, stride, k, W = cfg.L, cfg.stride, cfg.k, cfg.window
    nrep = n // k
    end = (np.arange(nrep, dtype=np.int64) + 1) * k
    hdr = np.zeros(nrep, O.SW_REPAIR_DTYPE)
    hdr["fss"] = np.maximum(0, end - W)
    hdr["nss"] = end - hdr["fss"]
    hdr["key"], hdr["dt"] = np.arange(nrep) & 0xFFFF, 15
    rng = np.random.default_rng(workloads.SEED)
    src = np.zeros((n, stride), np.uint8)
    src[:, :L] = rng.integers(0, 256, (n, L), dtype=np.uint8)
    sp = (rng.random(n) >= cfg.loss).astype(np.uint8)
    rp = (rng.random(nrep) >= cfg.loss).astype(np.uint8)
    tot, src_b, reps = 0.0, 0, 0
    while tot < seconds and reps < 1000:
        d = src.copy()
        d[sp == 0] = 0
        t0 = time.perf_counter()
        rep = O.sw_encode_simd(d, hdr, L, threads)
        O.sw_decode_simd(d, sp, rep, rp, hdr, L, threads)
        tot += time.perf_counter() - t0
        src_b += n * L
        reps += 1
    return {"value": round(src_b / tot / 1e9, 4), "unit": "GB/s", "cores": threads, "kind": "port",
            "codec": f"oracle/fec_cpu_simd.c orc_sw_encode_simd + orc_sw_decode_simd "
                     f"({O.SIMD_NAMES[O.simd_level()]}; banded decode of whole linked systems per thread; "
                     f"equal outputs to the scalar oracle: tests/test_oracle_simd.py)",
            "sample": f"{reps} passes over {n} sources x {L} B (W {W}, step {k}, loss {cfg.loss}), "
                      f"{tot:.1f} s on {threads} host threads"}


def launch_ranks(args) -> int:
    """`bench.py --gpus N` without a launcher: run N ranks (one per GPU) through a
    torch.distributed.run child and return its exit code.  Called before anything
    touches the GPU (device_count() does not initialise it on this image), and
    the child is a separate process, never an exec of this one."""
    import socket
    import subprocess
    if args.dist_backend == "nccl":
        ndev = torch.cuda.device_count()
        if ndev < args.gpus:
            log(f"--gpus {args.gpus} needs {args.gpus} GPUs (one rank per GPU over RCCL); "
                f"{ndev} visible (use --dist-backend gloo for a shared-GPU rehearsal)")
            return 2
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    log(f"launching {args.gpus} ranks: {' '.join(cmd[1:6])} ...")
    return subprocess.run(cmd).returncode


# extra configs timed by the default run (VERDICT r02 item 5, r03 items 6 and 8,
# r04 item 2): config -> (steps, warmup).  One GPU: configs 2, 4, 5 (host
# buffers, PCIe-inclusive: bound "pcie", never the headline) and 7.  N ranks:
# the device-resident configs, each rank on its own window shard (cfg4: 131,072
# windows per rank, the 1M windows of BASELINE config 4 at N = 8) with the
# digest gathered over RCCL.
EXTRA_CONFIGS = {2: (200, 20), 4: (5, 2), 5: (10, 2), 7: (50, 10)}
EXTRA_CONFIGS_MULTI = (2, 4, 7)


def make_ctx(args):
    ctx = fecgpu.Context()
    if args.grid_mult:
        ctx.set_tuning("grid_mult", args.grid_mult)
    if args.bitslice is not None:
        ctx.set_tuning("bitslice", args.bitslice)
    if args.bs_passes:
        ctx.set_tuning("bs_passes", args.bs_passes)
    if args.wpb:
        ctx.set_tuning("wpb", args.wpb)
    if args.gs is not None:
        ctx.set_tuning("gs", args.gs)
    if args.bpc:
        ctx.set_tuning("blocks_per_cu", args.bpc)
    if args.sw_group:
        ctx.set_tuning("sw_group", args.sw_group)
    if args.sw_stream >= 0:
        ctx.set_tuning("sw_stream", args.sw_stream)
    if args.sw_long_min:
        ctx.set_tuning("sw_long_min", args.sw_long_min)
    if args.host_direct >= 0:
        ctx.set_tuning("host_direct", args.host_direct)
    if args.host_chunk_mb:
        ctx.set_tuning("host_chunk_mb", args.host_chunk_mb)
    for kv in args.tune:
        key, val = kv.split("=", 1)
        ctx.set_tuning(key, int(val))
    return ctx


def run_config(cfgid: int, args, rank: int, world: int, dev, ctx, steps: int, warmup: int, nwin_arg: int):
    """Time `steps` steps of one config (after `warmup`), verify, digest; rank 0
    returns the JSON line's dict (others None).  Raises nothing on a failed
    verify: the line carries it."""
    cfg = workloads.CONFIGS[cfgid]
    if args.matrix != "cauchy" and cfg.scheme not in ("xor", "sw"):
        cfg = dataclasses.replace(cfg, matrix=args.matrix, name=f"{cfg.name}-{args.matrix}")
    if cfg.scheme == "sw" and (args.sw_loss >= 0 or args.sw_window > 0):
        loss = args.sw_loss if args.sw_loss >= 0 else cfg.loss
        win = args.sw_window or cfg.window
        cfg = dataclasses.replace(cfg, loss=loss, window=win, name=f"{cfg.name}-W{win}-loss{loss:g}",
                                  erasure_desc=f"i.i.d. p={loss:g} over sources and repairs")
    wide = args.k > 0 and cfg.scheme == "gf256" and cfg.workload == 0 and not cfg.host
    if wide:  # a code wider than one mask on config 3's workload
        cfg = dataclasses.replace(cfg, k=args.k, r=args.r, name=f"cfg3wide-gf256-k{args.k}r{args.r}-1200B",
                                  nwin_per_gpu=max(1, 5_033_164_800 // (args.k * cfg.L)),
                                  erasure_desc=f"exactly r={args.r} sources per window")
    nwin = nwin_arg or cfg.nwin_per_gpu
    w0, nwin = shard.weak_shard(rank, world, nwin)  # this rank's global window range
    if wide:
        batch = workloads.WideBatch.allocate(cfg, nwin, dev)
        log(f"rank {rank}: {cfg.name}, windows [{w0}, {w0 + nwin}), {batch.win.numel() / 2**30:.2f} GiB")
        batch.synthesize(ctx, w0)
        batch.make_erasures(ctx, w0)
    elif cfg.scheme == "sw":  # config 7: one sliding-window stream per rank
        batch = workloads.SwBatch.allocate(cfg, nwin, dev)
        log(f"rank {rank}: {cfg.name}, {batch.nsrc} sources, {batch.nrep} repairs, "
            f"{(batch.src.numel() + batch.rep.numel()) / 2**30:.2f} GiB")
        batch.synthesize(ctx, w0)
        batch.make_erasures(ctx, w0)
    elif cfg.host:  # config 5: host buffers, PCIe-inclusive (never the headline value)
        batch = workloads.HostBatch.allocate(cfg, nwin, dev)
        log(f"rank {rank}: {cfg.name}, windows [{w0}, {w0 + nwin}), "
            f"{batch.buf.nbytes / 2**30:.2f} GiB pinned host")
        batch.synthesize(ctx, w0, dev)
    else:
        batch = workloads.Batch.allocate(cfg, nwin, dev)
        log(f"rank {rank}: {cfg.name}, windows [{w0}, {w0 + nwin}), "
            f"{batch.win.numel() / 2**30:.2f} GiB")
        batch.synthesize(ctx, w0)
        batch.make_erasures(ctx, w0)
    src_bytes = batch.source_bytes()      # per rank, per step
    alg = batch.algorithmic_bytes()       # {'encode': B, 'decode': B} per launch
    batch_pcie = batch.pcie_bytes() if cfg.host else None

    log(f"{cfg.name}: warmup {warmup}")
    if cfg.scheme == "sw":
        # one synchronous decode first: it sizes the long-system log for this
        # stream (the asynchronous timed calls never retry), and any error it
        # cannot fix is raised here
        batch.encode(ctx)
        batch.decode(ctx, sync=True)
        ctx.sw_decode_errors()  # start the timed calls with clear flags
    for _ in range(warmup):
        batch.encode(ctx)
        batch.decode(ctx)
    torch.cuda.synchronize()

    every = args.event_every
    ev_steps = [i for i in range(steps) if every > 0 and i % every == 0]
    ev = {i: (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
              torch.cuda.Event(enable_timing=True)) for i in ev_steps}
    host_t = [0.0, 0.0]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        if cfg.host:  # synchronous calls on the library's own streams
            ta = time.perf_counter()
            batch.encode(ctx)
            tb = time.perf_counter()
            batch.decode(ctx)
            host_t[0] += tb - ta
            host_t[1] += time.perf_counter() - tb
            continue
        if i not in ev:
            batch.encode(ctx)
            batch.decode(ctx)
            continue
        e0, e1, e2 = ev[i]
        e0.record()
        batch.encode(ctx)
        e1.record()
        batch.decode(ctx)
        e2.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if cfg.host:
        enc_ms, dec_ms = host_t[0] * 1e3 / steps, host_t[1] * 1e3 / steps
    elif not ev:
        enc_ms = dec_ms = float("nan")
    else:
        enc_ms = sum(a.elapsed_time(b) for a, b, _ in ev.values()) / len(ev)
        dec_ms = sum(b.elapsed_time(c) for _, b, c in ev.values()) / len(ev)

    log(f"{cfg.name}: timed {steps} steps: {elapsed:.4f} s (encode {enc_ms:.3f} ms, decode {dec_ms:.3f} ms)")
    decode_only = None
    if cfg.scheme == "sw" and steps > 0:
        # the receiver alone (no encode launch to hide its plan under): `steps`
        # back-to-back decode calls, wall clock and HIP events on the launch stream
        torch.cuda.synchronize()
        d0, d1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ta = time.perf_counter()
        d0.record()
        for _ in range(steps):
            batch.decode(ctx)
        d1.record()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - ta) * 1e3 / steps
        decode_only = {"steps": steps, "ms_per_call": round(d0.elapsed_time(d1) / steps, 4),
                       "wall_ms_per_call": round(wall, 4),
                       "what": "fecgpu_sw_decode_device calls back to back, no encode in between"}
        log(f"{cfg.name}: decode only {decode_only['ms_per_call']:.4f} ms per call")
    # error flags of every asynchronous decode timed above (a long system left
    # undecoded by a full operation log would have done less work): any flag
    # fails the line
    async_errors = ctx.sw_decode_errors() if cfg.scheme == "sw" else None
    elapsed, tot = shard.reduce_run(elapsed, src_bytes, dev if args.dist_backend == "nccl" else None)
    # every rank's own HIP-event kernel times (north_star: the roofline fraction
    # at 1, 2, 4 and 8 GPUs per GPU, not rank 0's alone)
    rank_ms = shard.gather_floats([enc_ms, dec_ms], dev if args.dist_backend == "nccl" else None)
    total_src = float(tot) * steps
    value = total_src / elapsed / 1e9

    verify = None if args.no_verify else batch.verify(ctx, w0)
    if async_errors:
        log(f"{cfg.name}: asynchronous decodes raised error flags {async_errors:#x}")
        verify = dict(verify or {}, ok=False, async_error_flags=async_errors)
    log(f"{cfg.name}: verify: {verify}")
    # run digest of every rank's encoded windows, gathered over RCCL (8 B per
    # rank over xGMI: the path's only collective, outside the timed region)
    digest = None
    if verify is not None and not cfg.host:
        digest = shard.gather_digest(batch.digest(ctx, w0),
                                     dev if args.dist_backend == "nccl" else None)
    del batch
    torch.cuda.empty_cache()
    if rank != 0:
        return None
    dom = "decode" if dec_ms > enc_ms else "encode"
    dom_ms = enc_ms if dom == "encode" else dec_ms
    achieved = alg[dom] / (dom_ms * 1e-3) / 1e9
    pcie = None
    if cfg.host:  # PCIe is full duplex: each direction against its own 63 GB/s
        pb = batch_pcie
        pcie = {call: {d: {"bytes": pb[call][d], "GBs": round(pb[call][d] / (ms * 1e-3) / 1e9, 2),
                           "frac": round(pb[call][d] / (ms * 1e-3) / 1e9 / PCIE_DIR_PEAK_GBS, 4)}
                       for d in ("h2d", "d2h")}
                for call, ms in (("encode", enc_ms), ("decode", dec_ms))}
        bound_dir = max(("h2d", "d2h"), key=lambda d: pb[dom][d])
        achieved = pcie[dom][bound_dir]["GBs"]
    # traffic files: profiles/rNN_cfg<key>_traffic.json; a sliding-window run
    # with another loss / window has its own (key 7w<W>l<loss>)
    sw_variant = cfg.scheme == "sw" and cfg.name != workloads.CONFIGS[cfgid].name
    tkey = (f"wide{cfg.k}r{cfg.r}" if wide else f"{cfgid}w{cfg.window}l{cfg.loss:g}" if sw_variant else cfgid)
    traffic, traffic_src = (pmc_traffic(tkey, dom)
                            if nwin == cfg.nwin_per_gpu
                            and (wide or sw_variant or cfg.name == workloads.CONFIGS[cfgid].name)
                            and (cfg.matrix == "cauchy" or cfg.scheme == "sw")
                            else (None, None))
    cpu = None
    if args.cpu_seconds > 0 and world == 1 and not cfg.host:  # cfg5's codec and shape are cfg2's
        log(f"{cfg.name}: cpu baseline")
        cpu = (cpu_baseline_sw(cfg, args.cpu_seconds, args.cpu_threads) if cfg.scheme == "sw" else
               cpu_baseline_wide(cfg, args.cpu_seconds, args.cpu_threads) if wide else
               cpu_baseline(cfg, args.cpu_seconds, args.cpu_threads))
    peak, bound = (PCIE_DIR_PEAK_GBS, f"pcie-{bound_dir}") if cfg.host else (HBM_PEAK_GBS, "hbm")
    return {
        "metric": ("GB/s source-packet bytes FEC encode+decode, host buffers, PCIe-inclusive"
                   if cfg.host else
                   "GB/s source-packet bytes FEC encode+decode, device-resident, per MI355X"),
        "value": round(value, 3),
        "unit": "GB/s",
        "n_gpus": world,
        "ranks": world,
        "gpus_used": min(world, torch.cuda.device_count()),
        "rehearsal": (None if world <= torch.cuda.device_count() else
                      f"{world} ranks share {torch.cuda.device_count()} GPU(s) ({args.dist_backend}): "
                      f"exercises the N>1 path, not a multi-GPU measurement"),
        "value_per_gpu": round(value / world, 3),
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": round(elapsed / steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": ("synthetic (seeded torch bytes on the device, seeded host loss flags)" if cfg.scheme == "sw"
                 else "synthetic (on-device splitmix64 packets, seeded erasures)"),
        "config": ({
            "workload": cfg.name, "scheme": "sliding-window RLC (RFC 8681)",
            "sources_per_gpu": nwin * cfg.k, "repairs_per_gpu": nwin, "window": cfg.window,
            "step": cfg.k, "packet_bytes": cfg.L, "erasures": cfg.erasure_desc,
            "parallelism": f"stream per rank x{world}",
            "decode": "planned on the device (fecgpu_sw_decode_device: arrival flags, headers and "
                      "statuses in HBM; no host work per call)",
        } if cfg.scheme == "sw" else {
            "workload": cfg.name,
            "scheme": cfg.scheme, "k": cfg.k, "r": cfg.r,
            **({"matrix": cfg.matrix} if cfg.scheme != "xor" else {}),
            "windows_per_gpu": nwin, "packet_bytes": cfg.L if cfg.workload == 0 else "1200|9000 mixed",
            "erasures": cfg.erasure_desc,
            "parallelism": f"window-shard x{world}",
        }),
        "kernels_ms": {"encode": round(enc_ms, 4), "decode": round(dec_ms, 4)},
        "kernel_timing": ("host wall clock per synchronous call" if cfg.host else
                          f"HIP events on the launch stream around encode/decode, "
                          f"every {args.event_every}th timed step ({len(ev)} samples)"),
        "roofline": {
            "bound": bound,
            "kernel": dom,
            "achieved": round(achieved, 1),
            "peak": peak,
            "unit": "GB/s",
            "frac": round(achieved / peak, 4),
            "traffic": traffic,
            "traffic_source": traffic_src,
            "alg_bytes_per_launch": (batch_pcie[dom][bound_dir] if cfg.host else alg[dom]),
            **({} if cfg.host else {"per_rank": shard.per_rank_roofline(rank_ms, alg, peak)}),
            **({"pcie_directions": pcie,
                "note": "bytes of the bound direction of the slower call / its host wall time, "
                        "against 63 GB/s per direction"} if cfg.host else {}),
        },
        "roofline_other": {
            k2: round(alg[k2] / (ms * 1e-3) / 1e9, 1)
            for k2, ms in (("encode", enc_ms), ("decode", dec_ms))
        },
        "cpu_baseline": cpu,
        **({"decode_only": decode_only} if decode_only else {}),
        **({"async_error_flags": async_errors} if async_errors is not None else {}),
        "verify": verify,
        "digest": None if digest is None else f"{digest:016x}",
    }


def main():
    args = parse()
    if args.k:
        if args.k + args.r <= 64 or args.r < 1 or args.r > 8 or args.k + args.r > 256:
            log("--k/--r: a GF code with 64 < k + r <= 256 and 1 <= r <= 8")
            sys.exit(2)
        args.config = 3  # the wide code runs on config 3's workload
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"WORLD_SIZE={world} but --gpus {args.gpus}: refusing to report a mislabelled run")
        sys.exit(2)
    log(f"rank {rank}/{world} (local {local}) starting, backend "
        f"{args.dist_backend if world > 1 else 'none'}")
    ndev = torch.cuda.device_count()  # does not initialise the GPU on this image
    if world > 1:
        if args.dist_backend == "nccl":  # RCCL: one rank per GPU
            if ndev == 0:
                log(f"rank {rank}: no GPU visible; RCCL needs one per rank")
                sys.exit(2)
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:  # rehearsal of the N>1 path with ranks sharing the box's GPUs
            dist.init_process_group("gloo")  # host-only: every rank joins before any can leave
            if ndev == 0:
                log(f"rank {rank}: no GPU visible; nothing to time")
                dist.barrier()
                dist.destroy_process_group()
                sys.exit(2)
            torch.cuda.set_device(local % ndev)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    ctx = make_ctx(args)
    line = run_config(args.config, args, rank, world, dev, ctx, args.steps, args.warmup, args.nwin)
    ok = line is None or line["verify"] is None or line["verify"].get("ok", False)
    # the default run also times the other configs in this process (each on
    # its own batch, freed after), under "configs"; the headline line above is
    # config 3's
    if args.extra_configs and args.config == DEFAULT_CONFIG and not args.nwin and not args.k:
        extras = {}
        for cid, (st, wu) in EXTRA_CONFIGS.items():
            if world > 1 and cid not in EXTRA_CONFIGS_MULTI:
                continue
            try:
                sub = run_config(cid, args, rank, world, dev, ctx, st, wu, 0)
            except Exception as exc:  # keep the headline line; report the failure
                log(f"config {cid} failed: {exc!r}")
                extras[f"cfg{cid}"] = {"error": repr(exc)}
                ok = False
                continue
            if sub is None:  # ranks other than 0
                continue
            ok = ok and (sub["verify"] is None or sub["verify"].get("ok", False))
            extras[f"cfg{cid}"] = {k: sub[k] for k in ("metric", "value", "unit", "ms_per_step", "steps", "warmup",
                                                       "config", "kernels_ms", "roofline", "roofline_other",
                                                       "cpu_baseline", "verify", "digest", "decode_only",
                                                       "async_error_flags", "value_per_gpu")
                                 if k in sub}
        if line is not None:
            line["configs"] = extras
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if not ok:
        sys.exit(3)


if __name__ == "__main__":
    main()
