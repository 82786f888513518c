"""N>1 path on CPU: world_size-2 gloo.  Each rank encodes its weak shard of windows
(CPU oracle stands in for the GPU, whose kernels do not see rank), and the XOR of
the ranks' digests equals the single-process digest of the whole window range;
the max-over-ranks time and byte sums reduce as bench.py reports them."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from fecgpu import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


K, R, L, NPER = 8, 2, 200, 6


def _digest(O, w0, nwin):
    S = np.full(nwin, L, np.uint32)
    wins = O.make_windows(0, 77, w0, nwin, K, R, L, 208)
    O.encode_batch(O.GF256, K, R, S, wins)
    return O.batch_digest(K, R, S, wins, w0)


def _worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(here, "..", "oracle"))
    import oracle as O
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    w0, n = shard.weak_shard(rank, world, NPER)
    d = shard.gather_digest(_digest(O, w0, n))
    t, b = shard.reduce_run(0.5 + rank, 1000 * (rank + 1))
    # per-rank kernel times as bench.py gathers them for the N-rank roofline
    ms = shard.gather_floats([1.0 + rank, 2.0 + rank])
    roof = shard.per_rank_roofline(ms, {"encode": 4e9, "decode": 6e9}, 8000.0)
    q.put((rank, d, t, b, ms, roof))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shards_match_single_process(oracle_lib):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    whole = _digest(oracle_lib, 0, NPER * world)
    for rank, d, t, b, ms, roof in res:
        assert d == whole
        assert t == 1.5
        assert b == 3000
        # every rank sees both ranks' kernel times, in rank order
        assert ms == [[1.0, 2.0], [2.0, 3.0]]
        assert [row["rank"] for row in roof["ranks"]] == [0, 1]
        assert roof["ranks"][1]["encode_GBs"] == 2000.0  # 4e9 B / 2 ms
        assert roof["encode_frac_max"] == 0.5 and roof["encode_frac_min"] == 0.25
        assert roof["decode_frac_max"] == 0.375 and roof["decode_frac_min"] == 0.25


def test_shard_ranges():
    assert [shard.weak_shard(g, 4, 10) for g in range(4)] == [(0, 10), (10, 10), (20, 10), (30, 10)]
    got = [shard.strong_shard(g, 8, 1 << 20) for g in range(8)]
    assert sum(n for _, n in got) == 1 << 20
    assert all(got[i][0] + got[i][1] == got[i + 1][0] for i in range(7))
    got = [shard.strong_shard(g, 3, 10) for g in range(3)]
    assert got == [(0, 3), (3, 3), (6, 4)]
    assert shard.reduce_run(1.25, 7) == (1.25, 7)
    assert shard.gather_floats([1.5, 2.5]) == [[1.5, 2.5]]
    roof = shard.per_rank_roofline([[float("nan"), 2.0]], {"encode": 1e9, "decode": 1e9}, 8000.0)
    assert roof["encode_frac_min"] is None and roof["ranks"][0]["encode_ms"] is None
    assert roof["decode_frac_min"] == roof["decode_frac_max"] == 0.0625
