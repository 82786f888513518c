"""Window sharding across ranks: one process per GPU, contiguous
window ranges, no data-path collective.  torch.distributed (RCCL on the GPU box,
gloo in the CPU tests) carries only the barrier, the max-over-ranks time and
the optional digest gather."""
from __future__ import annotations

import torch
import torch.distributed as dist


def weak_shard(rank: int, world: int, nwin_per_rank: int) -> tuple[int, int]:
    """Fixed work per rank: rank g owns global windows [g*n, (g+1)*n)."""
    assert 0 <= rank < world
    return rank * nwin_per_rank, nwin_per_rank


def strong_shard(rank: int, world: int, nwin_total: int) -> tuple[int, int]:
    """Fixed total work: contiguous near-equal ranges [g*N/G, (g+1)*N/G)."""
    lo = nwin_total * rank // world
    hi = nwin_total * (rank + 1) // world
    return lo, hi - lo


def _active() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def reduce_run(elapsed_s: float, src_bytes: int, device=None) -> tuple[float, int]:
    """(max elapsed over ranks, sum of source bytes over ranks)."""
    if not _active():
        return float(elapsed_s), int(src_bytes)
    t = torch.tensor([elapsed_s], dtype=torch.float64, device=device)
    b = torch.tensor([src_bytes], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(b, op=dist.ReduceOp.SUM)
    return float(t.item()), int(b.item())


def gather_digest(digest: int, device=None) -> int:
    """XOR of every rank's run digest (order independent, shard invariant)."""
    if not _active():
        return digest & (2**64 - 1)
    v = digest & (2**64 - 1)
    t = torch.tensor([v - (1 << 64) if v >= 1 << 63 else v], dtype=torch.int64, device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    x = 0
    for o in out:
        x ^= int(o.item()) & (2**64 - 1)
    return x


def gather_floats(values, device=None) -> list[list[float]]:
    """Every rank's `values` (same length on every rank), in rank order: the
    per-rank kernel times bench.py turns into per-GPU roofline fractions, so an
    N-rank line shows the slowest GPU and not rank 0's alone."""
    vals = [float(v) for v in values]
    if not _active():
        return [vals]
    t = torch.tensor(vals, dtype=torch.float64, device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [[float(x) for x in o.cpu().tolist()] for o in out]


def per_rank_roofline(kernel_ms, alg_bytes: dict, peak_gbs: float) -> dict:
    """kernel_ms: [[encode_ms, decode_ms], ...] per rank; alg_bytes: algorithmic
    bytes per launch of each kernel (the same shard shape on every rank).
    Returns each rank's rate and fraction of `peak_gbs` for both kernels, and
    per kernel the min / max fraction over the ranks (None where a rank has no
    kernel time, e.g. HIP events switched off)."""
    ranks = []
    for r, (enc, dec) in enumerate(kernel_ms):
        row = {"rank": r}
        for name, ms in (("encode", enc), ("decode", dec)):
            ok = ms == ms and ms > 0  # not NaN, positive
            gbs = alg_bytes[name] / (ms * 1e-3) / 1e9 if ok else None
            row[f"{name}_ms"] = round(ms, 4) if ok else None
            row[f"{name}_GBs"] = round(gbs, 1) if ok else None
            row[f"{name}_frac"] = round(gbs / peak_gbs, 4) if ok else None
        ranks.append(row)
    out = {"ranks": ranks}
    for name in ("encode", "decode"):
        fr = [row[f"{name}_frac"] for row in ranks if row[f"{name}_frac"] is not None]
        out[f"{name}_frac_min"] = min(fr) if fr else None
        out[f"{name}_frac_max"] = max(fr) if fr else None
    return out
