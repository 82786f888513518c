"""Sliding-window RLC on the GPU (fecgpu_sw_encode / fecgpu_sw_decode through the
C ABI) against the CPU oracle (oracle/fec_oracle.c orc_sw_*, itself checked
against the numpy restatement in tests/test_sw_oracle.py and pinned to RFC
8682's TinyMT32 vectors in tests/test_rlc_spec.py).  Bit-exact on every byte
[0, S) of every repair and recovered source; statuses equal.
PARITY UNPINNED vs the fec branch (not mounted)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
import fecgpu  # noqa: E402
import oracle as O  # noqa: E402
import np_oracle as N  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    assert torch.cuda.is_available()
    O.build()
    c = fecgpu.Context()
    yield c
    c.close()


def hdr_array(h):
    a = np.zeros(len(h), O.SW_REPAIR_DTYPE)
    for t, (fss, nss, key, dt) in enumerate(h):
        a[t]["fss"], a[t]["nss"], a[t]["key"], a[t]["dt"] = fss, nss, key, dt
    return a


def stream(nsrc, L, stride, seed):
    rng = np.random.default_rng(seed)
    src = np.zeros((nsrc, stride), np.uint8)
    src[:, :L] = rng.integers(0, 256, (nsrc, L), dtype=np.uint8)
    return src


def gpu_encode(ctx, src, hdr, L, max_window=0):
    nsrc, stride = src.shape
    d_src = torch.from_numpy(src).cuda()
    d_rep = torch.full((len(hdr), stride), 0x77, dtype=torch.uint8, device="cuda")
    d_hdr = torch.from_numpy(hdr.view(np.uint8).copy()).cuda()
    ctx.sw_encode(d_src, d_rep, d_hdr, nsrc=nsrc, nrep=len(hdr), sym_len=L, stride=stride,
                  max_window=max_window)
    torch.cuda.synchronize()
    return d_rep.cpu().numpy()


def gpu_decode(ctx, src, sp, rep, rp, hdr, L, poison=0xAB):
    nsrc, stride = src.shape
    d = src.copy()
    d[sp == 0] = poison
    d_src = torch.from_numpy(d).cuda()
    d_rep = torch.from_numpy(np.where(rp[:, None] == 1, rep, poison).astype(np.uint8)).cuda()
    st = np.full(nsrc, 9, np.uint8)
    n = ctx.sw_decode(d_src, sp, d_rep, rp, hdr, st, nsrc=nsrc, nrep=len(hdr), sym_len=L, stride=stride)
    torch.cuda.synchronize()
    return d_src.cpu().numpy(), st, n


ENC = [  # nsrc, k, W, dt, L, max_window
    (256, 8, 32, 15, 1200, 32),
    (200, 4, 16, 15, 17, 0),
    (300, 1, 255, 15, 33, 255),     # the largest window
    (97, 3, 10, 5, 1, 10),
    (64, 8, 64, 0, 9000, 64),
    (500, 16, 48, 11, 100, 48),
]


@pytest.mark.parametrize("nsrc,k,W,dt,L,mw", ENC)
def test_sw_encode_vs_oracle(ctx, nsrc, k, W, dt, L, mw):
    stride = O.round_up(L, 16)
    src = stream(nsrc, L, stride, nsrc + W)
    hdr = hdr_array(N.sw_schedule(nsrc, k, W, key0=65530, dt=dt))   # keys wrap at 2^16
    g = gpu_encode(ctx, src, hdr, L, mw)
    o = O.sw_encode(src, hdr, L)
    assert np.array_equal(g[:, :L], o[:, :L])


def test_sw_encode_host_pointers(ctx):
    nsrc, L, stride = 120, 50, 64
    src = stream(nsrc, L, stride, 3)
    hdr = hdr_array(N.sw_schedule(nsrc, 5, 20, key0=9))
    rep = np.zeros((len(hdr), stride), np.uint8)
    assert ctx.sw_encode(src, rep, hdr, nsrc=nsrc, nrep=len(hdr), sym_len=L, stride=stride,
                         flags=fecgpu.F_HOST_PTRS) == len(hdr)
    assert np.array_equal(rep[:, :L], O.sw_encode(src, hdr, L)[:, :L])
    bad = hdr.copy()
    bad[3]["nss"] = 0
    with pytest.raises(fecgpu.FecError):
        ctx.sw_encode(src, rep, bad, nsrc=nsrc, nrep=len(hdr), sym_len=L, stride=stride,
                      flags=fecgpu.F_HOST_PTRS)
    bad = hdr.copy()
    bad[-1]["fss"] = nsrc - 2   # window past the end
    with pytest.raises(fecgpu.FecError):
        ctx.sw_encode(src, rep, bad, nsrc=nsrc, nrep=len(hdr), sym_len=L, stride=stride,
                      flags=fecgpu.F_HOST_PTRS)


def test_sw_encode_device_headers_are_clipped(ctx):
    """Device headers are not validated: a window past nsrc or past max_window is clipped."""
    nsrc, L, stride = 40, 32, 32
    src = stream(nsrc, L, stride, 5)
    hdr = hdr_array([(30, 20, 1, 15), (0, 12, 2, 15), (39, 1, 3, 15), (45, 4, 4, 15)])
    g = gpu_encode(ctx, src, hdr, L, max_window=10)
    clipped = hdr_array([(30, 10, 1, 15), (0, 10, 2, 15), (39, 1, 3, 15)])
    o = O.sw_encode(src, clipped, L)
    assert np.array_equal(g[:3, :L], o[:, :L])
    assert not g[3, :L].any()   # empty window: zero repair


@pytest.mark.parametrize("L", [300, 1200])   # < 64 / >= 64 columns: zero-skip off / on
@pytest.mark.parametrize("group", [1, 2, 4, 8])
@pytest.mark.parametrize("host", [False, True], ids=["dev_hdr", "host_hdr"])
def test_sw_encode_grouped_jobs(group, host, L):
    """Grouped encode jobs (ctx "sw_group"): consecutive repairs share one combine
    job over the union of their windows when it spans <= 2 * max_window sources,
    else fall back to one job per repair (the tail; skipped when the host sees
    the headers and every group fits).  A stream schedule with some repairs moved
    far away (mixed fitting / non-fitting groups), a ragged last group, and one
    with every group fitting: equal to the oracle."""
    c = fecgpu.Context()
    try:
        c.set_tuning("sw_group", group)
        nsrc, W = 700, 32
        stride = O.round_up(L, 16)
        src = stream(nsrc, L, stride, 11 + group)
        base = N.sw_schedule(nsrc, 8, W, key0=100)
        moved = list(base)
        for t in range(5, len(moved), 9):   # some windows far from their group neighbours
            fss, nss, key, dt = moved[t]
            moved[t] = ((fss + 333) % (nsrc - nss), nss, key, dt)
        for sched in (base, moved, base[:-3]):
            hdr = hdr_array(sched)
            o = O.sw_encode(src, hdr, L)
            if host:
                rep = np.zeros((len(hdr), stride), np.uint8)
                c.sw_encode(src, rep, hdr, nsrc=nsrc, nrep=len(hdr), sym_len=L, stride=stride,
                            max_window=W, flags=fecgpu.F_HOST_PTRS)
            else:
                rep = gpu_encode(c, src, hdr, L, W)
            assert np.array_equal(rep[:, :L], o[:, :L])
        with pytest.raises(fecgpu.FecError):
            c.set_tuning("sw_group", 3)
    finally:
        c.close()


LOSS = [("iid", 0.03), ("iid", 0.1), ("iid", 0.25), ("burst", 7), ("burst", 30), ("reps", 0.5)]


@pytest.mark.parametrize("loss", LOSS, ids=[f"{a}{b}" for a, b in LOSS])
@pytest.mark.parametrize("nsrc,k,W,dt,L", [(400, 8, 32, 15, 1200), (300, 4, 16, 15, 40),
                                           (300, 4, 12, 3, 24), (256, 2, 20, 15, 16)])
def test_sw_decode_vs_oracle(ctx, loss, nsrc, k, W, dt, L):
    stride = O.round_up(L, 16)
    src = stream(nsrc, L, stride, 11 * k + W)
    hdr = hdr_array(N.sw_schedule(nsrc, k, W, key0=1234, dt=dt))
    rep = O.sw_encode(src, hdr, L)
    rng = np.random.default_rng(k + W + int(loss[1] * 100))
    sp = np.ones(nsrc, np.uint8)
    rp = np.ones(len(hdr), np.uint8)
    if loss[0] == "iid":
        sp = (rng.random(nsrc) >= loss[1]).astype(np.uint8)
        rp = (rng.random(len(hdr)) >= loss[1]).astype(np.uint8)
    elif loss[0] == "burst":
        b = int(rng.integers(0, nsrc - loss[1]))
        sp[b:b + loss[1]] = 0
        sp[(b + 90) % nsrc] = 0
    else:  # half the repairs lost, a few sources
        rp = (rng.random(len(hdr)) >= loss[1]).astype(np.uint8)
        sp[rng.choice(nsrc, 12, replace=False)] = 0
    gd, gst, gn = gpu_decode(ctx, src, sp, rep, rp, hdr, L)
    od = src.copy()
    od[sp == 0] = 0xAB
    ost, on = O.sw_decode(od, sp, rep, rp, hdr, L)
    assert np.array_equal(gst, ost), np.argwhere(gst != ost)[:8].tolist()
    assert gn == on
    assert np.array_equal(gd[:, :L], od[:, :L])
    assert np.array_equal(gd[gst == 0, :L], src[gst == 0, :L])
    assert (sp == 0).sum() == 0 or gn > 0 or loss[1] >= 0.25


def test_sw_decode_unknown_cap(ctx):
    """A linked system of more than 64 lost sources stays lost (FECGPU_SW_MAX_UNKNOWNS);
    a separate system of 30 in the same stream is recovered."""
    nsrc, L, stride, k, W = 600, 32, 32, 2, 40
    src = stream(nsrc, L, stride, 17)
    hdr = hdr_array(N.sw_schedule(nsrc, k, W, key0=5))
    rep = O.sw_encode(src, hdr, L)
    sp = np.ones(nsrc, np.uint8)
    sp[100:170] = 0      # 70 lost, linked
    sp[400:430] = 0      # 30 lost
    rp = np.ones(len(hdr), np.uint8)
    gd, gst, gn = gpu_decode(ctx, src, sp, rep, rp, hdr, L)
    assert (gst[100:170] == 1).all()
    assert (gst[400:430] == 0).all() and gn == 30
    assert np.array_equal(gd[400:430, :L], src[400:430, :L])


def test_sw_decode_equation_cap(ctx):
    """More than 96 received repairs over one system: the first 96 are used (still full rank)."""
    nsrc, L, stride = 400, 16, 16
    src = stream(nsrc, L, stride, 23)
    hdr = hdr_array(N.sw_schedule(nsrc, 1, 200, key0=77))   # a repair after every source
    rep = O.sw_encode(src, hdr, L)
    sp = np.ones(nsrc, np.uint8)
    sp[150:160] = 0
    rp = np.ones(len(hdr), np.uint8)
    gd, gst, gn = gpu_decode(ctx, src, sp, rep, rp, hdr, L)
    assert gn == 10 and (gst == 0).all()
    assert np.array_equal(gd[:, :L], src[:, :L])


def test_sw_decode_host_pointers_and_args(ctx):
    nsrc, L, stride = 200, 40, 48
    src = stream(nsrc, L, stride, 29)
    hdr = hdr_array(N.sw_schedule(nsrc, 4, 16, key0=3))
    rep = O.sw_encode(src, hdr, L)
    sp = np.ones(nsrc, np.uint8)
    sp[[5, 50, 51, 52, 199]] = 0
    rp = np.ones(len(hdr), np.uint8)
    d = src.copy()
    d[sp == 0] = 0
    st = np.zeros(nsrc, np.uint8)
    n = ctx.sw_decode(d, sp, rep, rp, hdr, st, nsrc=nsrc, nrep=len(hdr), sym_len=L, stride=stride,
                      flags=fecgpu.F_HOST_PTRS)
    assert n == 5 and (st == 0).all() and np.array_equal(d[:, :L], src[:, :L])
    unsorted = hdr[::-1].copy()
    with pytest.raises(fecgpu.FecError):
        ctx.sw_decode(d, sp, rep, rp, unsorted, st, nsrc=nsrc, nrep=len(hdr), sym_len=L, stride=stride,
                      flags=fecgpu.F_HOST_PTRS)


def test_sw_full_size_roundtrip(ctx):
    """131,072 sources of 1200 B (157 MB), a repair after every 8 over the last 32, 2 %
    i.i.d. loss of sources and repairs: every source the decoder reports recovered
    equals the original, and the recovered count equals the oracle's on a prefix
    that ends where no received repair crosses."""
    nsrc, L, stride, k, W = 131072, 1200, 1200, 8, 32
    g = torch.Generator(device="cuda").manual_seed(7)
    d_src = torch.randint(0, 256, (nsrc, stride), dtype=torch.uint8, device="cuda", generator=g)
    h = N.sw_schedule(nsrc, k, W, key0=0)
    hdr = hdr_array(h)
    d_hdr = torch.from_numpy(hdr.view(np.uint8).copy()).cuda()
    d_rep = torch.empty((len(h), stride), dtype=torch.uint8, device="cuda")
    ctx.sw_encode(d_src, d_rep, d_hdr, nsrc=nsrc, nrep=len(h), sym_len=L, stride=stride, max_window=W)
    orig = d_src.clone()
    rng = np.random.default_rng(1)
    sp = (rng.random(nsrc) >= 0.02).astype(np.uint8)
    rp = (rng.random(len(h)) >= 0.02).astype(np.uint8)
    lost = torch.from_numpy(sp == 0).cuda()
    d_src[lost] = 0xCD
    st = np.zeros(nsrc, np.uint8)
    n = ctx.sw_decode(d_src, sp, d_rep, rp, hdr, st, nsrc=nsrc, nrep=len(h), sym_len=L, stride=stride)
    torch.cuda.synchronize()
    ok = torch.from_numpy(st == 0).cuda()
    assert torch.equal(d_src[ok], orig[ok])
    assert n == int(((sp == 0) & (st == 0)).sum()) and n > 0.9 * (sp == 0).sum()
    # the oracle on a prefix [0, c) whose last W sources all arrived: no linked system
    # crosses c (two linked lost sources lie < W apart) and every repair that holds a
    # lost source below c - W lies inside [0, c), so statuses there must be equal
    c = next(c for c in range(4096, 2 * W, -1) if sp[c - W:c].all())
    hp = [x for x in h if x[0] + x[1] <= c]
    sub = orig[:c].cpu().numpy()
    od = sub.copy()
    od[sp[:c] == 0] = 0
    ost, _ = O.sw_decode(od, sp[:c].copy(), d_rep[:len(hp)].cpu().numpy(), rp[:len(hp)].copy(),
                         hdr_array(hp), L)
    assert np.array_equal(st[:c], ost)
    assert np.array_equal(od[ost == 0], sub[ost == 0])


def test_bench_config7_batch(ctx):
    """bench.py --config 7's SwBatch: its repairs equal the oracle's over the
    stream's first sources, and its verify step (poison, decode, compare)
    recovers every determined lost source byte for byte."""
    from fecgpu import workloads
    cfg = workloads.CONFIGS[7]
    b = workloads.SwBatch.allocate(cfg, 2048, torch.device("cuda"))
    b.synthesize(ctx, 0)
    b.make_erasures(ctx, 0)
    b.encode(ctx)
    torch.cuda.synchronize()
    n = 512
    src = b.src[:n].cpu().numpy()
    hdr = b.hdr[: n // cfg.k]
    o = O.sw_encode(src, hdr, cfg.L)
    assert np.array_equal(b.rep[: n // cfg.k, :cfg.L].cpu().numpy(), o[:, :cfg.L])
    v = b.verify(ctx, 0)
    assert v["ok"] and v["lost"] > 0 and v["recovered"] > 0.9 * v["lost"], v
    alg = b.algorithmic_bytes()
    assert alg["encode"] == (b.nsrc + b.nrep) * cfg.L
