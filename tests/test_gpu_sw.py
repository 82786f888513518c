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


@pytest.mark.parametrize("stream_enc", [1, 0], ids=["streaming", "combine"])
def test_sw_coefficient_table_keys_and_mixed_dt(stream_enc):
    """The dense (dt 15) coefficients come from the ctx's 16 MiB table of every
    repair key's sequence, other dt values are drawn per coefficient: one stream
    mixing both, keys spread over all 2^16 (0 and 65535 included), windows up to
    255: encode and decode equal to the oracle."""
    c = fecgpu.Context()
    try:
        c.set_tuning("sw_stream", stream_enc)
        nsrc, L = 1500, 40
        stride = O.round_up(L, 16)
        src = stream(nsrc, L, stride, 77 + stream_enc)
        h = []
        for t, fss in enumerate(range(0, nsrc - 255, 3)):
            nss = 255 if t % 5 == 0 else 1 + (t * 37) % 64
            key = 65535 if t == 1 else (t * 2731) & 0xFFFF
            h.append((fss, nss, key, 15 if t % 4 else (t // 4) % 15))
        hdr = hdr_array(h)
        o = O.sw_encode(src, hdr, L)
        g = gpu_encode(c, src, hdr, L, 255)
        assert np.array_equal(g[:, :L], o[:, :L])
        rng = np.random.default_rng(5)
        sp = (rng.random(nsrc) >= 0.05).astype(np.uint8)
        rp = (rng.random(len(hdr)) >= 0.05).astype(np.uint8)
        gd, gst, gn = gpu_decode(c, src, sp, o, rp, hdr, L)
        od, ost, on = oracle_decode(src, sp, o, rp, hdr, L)
        assert np.array_equal(gst, ost) and gn == on and gn > 0
        assert np.array_equal(gd[:, :L], od[:, :L])
    finally:
        c.close()


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
        c.set_tuning("sw_stream", 0)   # the combine-job encode
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


def oracle_decode(src, sp, rep, rp, hdr, L):
    """Banded oracle (oracle/fec_sw_banded.c: equal to the dense Gauss-Jordan on
    every status and byte, tests/test_sw_oracle.py), poisoned like gpu_decode."""
    od = src.copy()
    od[sp == 0] = 0xAB
    ost, on = O.sw_decode_banded(od, sp, rep, rp, hdr, L)
    return od, ost, on


def check_vs_oracle(ctx, src, sp, rep, rp, hdr, L):
    gd, gst, gn = gpu_decode(ctx, src, sp, rep, rp, hdr, L)
    od, ost, on = oracle_decode(src, sp, rep, rp, hdr, L)
    assert np.array_equal(gst, ost), np.argwhere(gst != ost)[:8].tolist()
    assert gn == on
    assert np.array_equal(gd[:, :L], od[:, :L])
    assert np.array_equal(gd[gst == 0, :L], src[gst == 0, :L])
    return gn


def max_system(sp, rp, hdr):
    """Unknowns of the largest linked system (two lost sources are linked when a
    received repair's window holds both)."""
    lost = np.flatnonzero(sp == 0)
    if len(lost) == 0:
        return 0
    end = np.where(rp == 1, hdr["fss"].astype(np.int64) + hdr["nss"], 0)
    pe = np.maximum.accumulate(end)
    idx = np.searchsorted(hdr["fss"].astype(np.int64), lost, side="right") - 1
    reach = np.where(idx >= 0, pe[np.maximum(idx, 0)], 0)
    start = np.ones(len(lost), bool)
    start[1:] = reach[:-1] <= lost[1:]
    return int(np.bincount(np.cumsum(start) - 1).max())


# (W, step, loss): i.i.d. loss of sources and repairs at the rates VERDICT r02
# asks for; the long streams make linked systems of hundreds of unknowns
LONG = [(W, k, p) for W in (32, 64, 255) for k in (1, 4, 8) for p in (0.02, 0.05, 0.10, 0.15)]


@pytest.mark.parametrize("W,k,loss", LONG, ids=[f"W{w}-step{k}-{int(p * 100)}pct" for w, k, p in LONG])
def test_sw_decode_long_systems_vs_oracle(ctx, W, k, loss):
    """No cap on linked systems: statuses, count and every byte equal the
    oracle's global decode, for windows 32/64/255, steps 1/4/8 and 2-15 %
    loss.  Streams are sized so the heavier cases link hundreds of unknowns."""
    nsrc = 4000 if W == 255 and k == 1 else 6000
    L = 40
    stride = O.round_up(L, 16)
    src = stream(nsrc, L, stride, W * 100 + k * 10 + int(loss * 100))
    hdr = hdr_array(N.sw_schedule(nsrc, k, W, key0=W * k, dt=15))
    rep = O.sw_encode(src, hdr, L)
    rng = np.random.default_rng(W + k + int(loss * 1000))
    sp = (rng.random(nsrc) >= loss).astype(np.uint8)
    rp = (rng.random(len(hdr)) >= loss).astype(np.uint8)
    check_vs_oracle(ctx, src, sp, rep, rp, hdr, L)
    if loss >= 0.10 and W >= 64:
        assert max_system(sp, rp, hdr) > 200


@pytest.mark.parametrize("burst", [100, 180, 300])
@pytest.mark.parametrize("W,k", [(32, 4), (64, 8), (255, 8), (255, 1)])
def test_sw_decode_bursts_vs_oracle(ctx, burst, W, k):
    """Bursts of 100-300 consecutive lost sources plus 3 % i.i.d. loss: a burst
    longer than the window's repairs can cover leaves a linked system the
    repairs only partly determine; equal to the oracle everywhere."""
    nsrc, L = 3000, 64
    stride = O.round_up(L, 16)
    src = stream(nsrc, L, stride, burst + W)
    hdr = hdr_array(N.sw_schedule(nsrc, k, W, key0=burst, dt=15))
    rep = O.sw_encode(src, hdr, L)
    rng = np.random.default_rng(burst * W + k)
    sp = (rng.random(nsrc) >= 0.03).astype(np.uint8)
    rp = (rng.random(len(hdr)) >= 0.03).astype(np.uint8)
    b = int(rng.integers(200, nsrc - burst - 200))
    sp[b:b + burst] = 0
    check_vs_oracle(ctx, src, sp, rep, rp, hdr, L)


@pytest.mark.parametrize("dt", [0, 3, 15])
@pytest.mark.parametrize("long_min", [1, 8])
def test_sw_decode_long_path_on_every_system(dt, long_min):
    """Tuning "sw_long_min" sends small systems down the banded long-system path
    too: the two paths agree with the oracle on the same random streams,
    including sparse coefficients (DT 0, 3: rank-deficient systems)."""
    c = fecgpu.Context()
    try:
        c.set_tuning("sw_long_min", long_min)
        for seed in range(12):
            rng = np.random.default_rng(seed * 7 + dt)
            nsrc = int(rng.integers(100, 900))
            k = int(rng.integers(1, 9))
            W = int(rng.integers(k, 80))
            L = int(rng.integers(1, 200))
            stride = O.round_up(L, 16)
            src = stream(nsrc, L, stride, seed)
            hdr = hdr_array(N.sw_schedule(nsrc, k, W, key0=seed * 31, dt=dt))
            rep = O.sw_encode(src, hdr, L)
            loss = float(rng.choice([0.05, 0.15, 0.3]))
            sp = (rng.random(nsrc) >= loss).astype(np.uint8)
            rp = (rng.random(len(hdr)) >= loss).astype(np.uint8)
            check_vs_oracle(c, src, sp, rep, rp, hdr, L)
    finally:
        c.close()


def test_sw_decode_wide_symbols_long_path():
    """Long systems over 1200-B and 9000-B symbols (the replay walks 256-B column
    chunks), equal to the oracle."""
    c = fecgpu.Context()
    try:
        c.set_tuning("sw_long_min", 1)
        for L, nsrc in ((1200, 700), (9000, 250)):
            stride = O.round_up(L, 16)
            src = stream(nsrc, L, stride, L)
            hdr = hdr_array(N.sw_schedule(nsrc, 4, 40, key0=L, dt=15))
            rep = O.sw_encode(src, hdr, L)
            rng = np.random.default_rng(L)
            sp = (rng.random(nsrc) >= 0.12).astype(np.uint8)
            rp = (rng.random(len(hdr)) >= 0.05).astype(np.uint8)
            assert check_vs_oracle(c, src, sp, rep, rp, hdr, L) > 0
    finally:
        c.close()


def test_sw_decode_device_bookkeeping(ctx):
    """fecgpu_sw_decode_device (flags, headers and statuses in device memory)
    equals the host-bookkeeping decode; asynchronous without F_SYNC; a bad or
    unordered header is INVALID_ARG with F_SYNC and recovers nothing."""
    nsrc, L, k, W = 3000, 100, 4, 64
    stride = O.round_up(L, 16)
    src = stream(nsrc, L, stride, 41)
    hdr = hdr_array(N.sw_schedule(nsrc, k, W, key0=2, dt=15))
    rep = O.sw_encode(src, hdr, L)
    rng = np.random.default_rng(5)
    sp = (rng.random(nsrc) >= 0.12).astype(np.uint8)
    rp = (rng.random(len(hdr)) >= 0.05).astype(np.uint8)
    od, ost, on = oracle_decode(src, sp, rep, rp, hdr, L)
    for flags in (0, fecgpu.F_SYNC):
        d = src.copy()
        d[sp == 0] = 0xAB
        d_src = torch.from_numpy(d).cuda()
        d_rep = torch.from_numpy(rep).cuda()
        d_sp, d_rp = torch.from_numpy(sp).cuda(), torch.from_numpy(rp).cuda()
        d_hdr = torch.from_numpy(hdr.view(np.uint8).copy()).cuda()
        d_st = torch.full((nsrc,), 9, dtype=torch.uint8, device="cuda")
        n = ctx.sw_decode_device(d_src, d_sp, d_rep, d_rp, d_hdr, d_st, nsrc=nsrc, nrep=len(hdr), sym_len=L,
                                 stride=stride, flags=flags)
        torch.cuda.synchronize()
        assert n == (on if flags else 0)
        assert np.array_equal(d_st.cpu().numpy(), ost)
        assert np.array_equal(d_src.cpu().numpy()[:, :L], od[:, :L])
    bad = hdr[::-1].copy()
    d_hdr = torch.from_numpy(bad.view(np.uint8).copy()).cuda()
    with pytest.raises(fecgpu.FecError) as ei:
        ctx.sw_decode_device(d_src, d_sp, d_rep, d_rp, d_hdr, d_st, nsrc=nsrc, nrep=len(hdr), sym_len=L,
                             stride=stride, flags=fecgpu.F_SYNC)
    assert ei.value.code == fecgpu.ERR_INVALID_ARG
    assert np.array_equal(d_st.cpu().numpy(), 1 - sp)


def test_sw_decode_log_overflow_retries():
    """A long-system log reservation far too small (tuning "sw_log_entries" = 16):
    the asynchronous device call leaves the overflowing systems lost, the
    synchronous calls grow the log and finish equal to the oracle."""
    c = fecgpu.Context()
    try:
        c.set_tuning("sw_log_entries", 16)
        nsrc, L, k, W = 2000, 32, 2, 64
        stride = O.round_up(L, 16)
        src = stream(nsrc, L, stride, 8)
        hdr = hdr_array(N.sw_schedule(nsrc, k, W, key0=8, dt=15))
        rep = O.sw_encode(src, hdr, L)
        rng = np.random.default_rng(8)
        sp = (rng.random(nsrc) >= 0.2).astype(np.uint8)
        rp = np.ones(len(hdr), np.uint8)
        assert max_system(sp, rp, hdr) > 64
        od, ost, on = oracle_decode(src, sp, rep, rp, hdr, L)
        d = src.copy()
        d[sp == 0] = 0xAB
        d_src = torch.from_numpy(d).cuda()
        d_st = torch.zeros(nsrc, dtype=torch.uint8, device="cuda")
        assert c.sw_decode_device(d_src, torch.from_numpy(sp).cuda(), torch.from_numpy(rep).cuda(),
                                  torch.from_numpy(rp).cuda(), torch.from_numpy(hdr.view(np.uint8).copy()).cuda(),
                                  d_st, nsrc=nsrc, nrep=len(hdr), sym_len=L, stride=stride) == 0
        torch.cuda.synchronize()
        ast = d_st.cpu().numpy()
        got = d_src.cpu().numpy()
        assert ((ast == 0) <= (ost == 0)).all() and (ast != ost).any()  # the long systems stayed lost
        assert np.array_equal(got[ast == 0, :L], src[ast == 0, :L])
        check_vs_oracle(c, src, sp, rep, rp, hdr, L)
    finally:
        c.close()


def two_per_step(nsrc, W, key0, dt=15):
    """Two repairs after every source over the last W (distinct keys): about
    2 W received repairs cover each source."""
    h = []
    for t, (fss, nss, _, _) in enumerate(N.sw_schedule(nsrc, 1, W)):
        h += [(fss, nss, (key0 + 2 * t) & 0xFFFF, dt), (fss, nss, (key0 + 2 * t + 1) & 0xFFFF, dt)]
    return hdr_array(h)


@pytest.mark.parametrize("loss", [0.02, 0.10, 0.30])
def test_sw_decode_two_repairs_per_step_W255(ctx, loss):
    """More repairs alive at one column than the long-system pass has row slots
    (256): 2 repairs per step at W = 255, step 1, so ~500 received repairs cover
    every lost source.  The pass reduces its alive rows to a basis when the
    slots run out (fec_swdec.hip long_compact); statuses, count and every byte
    equal the banded oracle's global decode."""
    nsrc, L, W = 2500, 24, 255
    stride = O.round_up(L, 16)
    src = stream(nsrc, L, stride, 255 + int(loss * 100))
    hdr = two_per_step(nsrc, W, key0=int(loss * 1000))
    rep = O.sw_encode(src, hdr, L)
    rng = np.random.default_rng(int(loss * 1000) + 1)
    sp = (rng.random(nsrc) >= loss).astype(np.uint8)
    rp = (rng.random(len(hdr)) >= loss).astype(np.uint8)
    assert max_system(sp, rp, hdr) > (100 if loss >= 0.1 else 30)  # long systems (> 96 equations)
    assert check_vs_oracle(ctx, src, sp, rep, rp, hdr, L) > 0.9 * (sp == 0).sum()


@pytest.mark.parametrize("nsame,dt,lost", [(320, 15, 150), (700, 15, 250), (400, 2, 120), (300, 15, 255)])
def test_sw_decode_many_repairs_one_fss(ctx, nsame, dt, lost):
    """More than 300 received repairs sharing one fss (all over the same 255
    sources, `lost` of them lost) inside a regular W 32 step 4 stream: every
    one is alive at the system's first column.  DT 2 makes sparse rows (the
    shared window partly undetermined).  Equal to the banded oracle."""
    nsrc, L, W0 = 1200, 40, 255
    stride = O.round_up(L, 16)
    src = stream(nsrc, L, stride, nsame + dt)
    base = N.sw_schedule(nsrc, 4, 32, key0=7)
    fss0 = 400
    same = [(fss0, W0, (1000 + u) & 0xFFFF, dt) for u in range(nsame)]
    h = sorted(base + same, key=lambda x: x[0])   # fss nondecreasing (stable: base first)
    hdr = hdr_array(h)
    rep = O.sw_encode(src, hdr, L)
    rng = np.random.default_rng(nsame + lost)
    sp = (rng.random(nsrc) >= 0.03).astype(np.uint8)
    sp[fss0 + rng.choice(W0, lost, replace=False)] = 0
    rp = np.ones(len(hdr), np.uint8)
    rp[rng.choice(len(hdr), len(hdr) // 50, replace=False)] = 0
    check_vs_oracle(ctx, src, sp, rep, rp, hdr, L)


def test_sw_decode_compaction_with_small_log():
    """The compaction's eliminations overflow a long system's first log chunk:
    chained chunks (kOpJump) and, with a tiny reservation ("sw_log_entries" =
    4096), the synchronous retries; equal to the oracle."""
    c = fecgpu.Context()
    try:
        nsrc, L, W = 1500, 16, 255
        stride = O.round_up(L, 16)
        src = stream(nsrc, L, stride, 77)
        hdr = two_per_step(nsrc, W, key0=77)
        rep = O.sw_encode(src, hdr, L)
        rng = np.random.default_rng(77)
        sp = (rng.random(nsrc) >= 0.2).astype(np.uint8)
        rp = (rng.random(len(hdr)) >= 0.2).astype(np.uint8)
        for entries in (0, 4096):
            if entries:
                c.set_tuning("sw_log_entries", entries)
            check_vs_oracle(c, src, sp, rep, rp, hdr, L)
    finally:
        c.close()


def test_sw_decode_async_error_flags():
    """Asynchronous decodes raise their errors where the caller can read them
    (fecgpu_sw_decode_errors): with "sw_log_entries" = 16
    the long systems overflow and SW_ERR_CAPACITY is set (the flags clear on
    read); a reversed header list raises SW_ERR_HEADER; a clean call raises
    nothing."""
    c = fecgpu.Context()
    try:
        nsrc, L, k, W = 2000, 32, 2, 64
        stride = O.round_up(L, 16)
        src = stream(nsrc, L, stride, 8)
        hdr = hdr_array(N.sw_schedule(nsrc, k, W, key0=8, dt=15))
        rep = O.sw_encode(src, hdr, L)
        rng = np.random.default_rng(8)
        sp = (rng.random(nsrc) >= 0.2).astype(np.uint8)
        rp = np.ones(len(hdr), np.uint8)
        od, ost, on = oracle_decode(src, sp, rep, rp, hdr, L)

        def run(h):
            d = src.copy()
            d[sp == 0] = 0xAB
            d_src = torch.from_numpy(d).cuda()
            d_st = torch.zeros(nsrc, dtype=torch.uint8, device="cuda")
            assert c.sw_decode_device(d_src, torch.from_numpy(sp).cuda(), torch.from_numpy(rep).cuda(),
                                      torch.from_numpy(rp).cuda(), torch.from_numpy(h.view(np.uint8).copy()).cuda(),
                                      d_st, nsrc=nsrc, nrep=len(h), sym_len=L, stride=stride) == 0
            return d_src, d_st

        assert c.sw_decode_errors() == 0
        c.set_tuning("sw_log_entries", 16)
        run(hdr)
        assert c.sw_decode_errors() == fecgpu.SW_ERR_CAPACITY
        assert c.sw_decode_errors() == 0
        c.set_tuning("sw_log_entries", 0)   # automatic: grown past the overflow
        d_src, d_st = run(hdr)
        assert c.sw_decode_errors() == 0
        assert np.array_equal(d_st.cpu().numpy(), ost)
        assert np.array_equal(d_src.cpu().numpy()[:, :L], od[:, :L])
        run(hdr[::-1].copy())
        assert c.sw_decode_errors() == fecgpu.SW_ERR_HEADER
    finally:
        c.close()


@pytest.mark.parametrize("bad", ["swap", "nss300", "past_end", "dt16"])
def test_sw_decode_bad_headers_recover_nothing(bad):
    """A bad or unordered device header list: the plan's blocks
    finish their chunks' one-unknown systems before every chunk's headers are
    checked, so the combine launches must stand down and the statuses be
    restored.  Several plan chunks (nsrc > 2048), one bad header near the end:
    the asynchronous call raises SW_ERR_HEADER, every status equals the arrival
    flag and no source byte changes; the synchronous call is INVALID_ARG."""
    c = fecgpu.Context()
    try:
        nsrc, L, k, W = 9000, 64, 4, 32
        stride = O.round_up(L, 16)
        src = stream(nsrc, L, stride, 301)
        hdr = hdr_array(N.sw_schedule(nsrc, k, W, key0=11, dt=15))
        rep = O.sw_encode(src, hdr, L)
        rng = np.random.default_rng(301)
        sp = (rng.random(nsrc) >= 0.03).astype(np.uint8)   # mostly one-unknown systems
        rp = np.ones(len(hdr), np.uint8)
        t = len(hdr) - 40
        if bad == "swap":
            hdr[[t, t + 1]] = hdr[[t + 1, t]]
            assert hdr[t]["fss"] > hdr[t + 1]["fss"]
        elif bad == "nss300":
            hdr[t]["nss"] = 300
        elif bad == "past_end":
            hdr[t]["fss"], hdr[t]["nss"] = nsrc - 2, 8
        else:
            hdr[t]["dt"] = 16
        d = src.copy()
        d[sp == 0] = 0xAB
        d_src = torch.from_numpy(d).cuda()
        d_st = torch.full((nsrc,), 9, dtype=torch.uint8, device="cuda")
        args = (torch.from_numpy(sp).cuda(), torch.from_numpy(rep).cuda(), torch.from_numpy(rp).cuda(),
                torch.from_numpy(hdr.view(np.uint8).copy()).cuda(), d_st)
        assert c.sw_decode_errors() == 0
        assert c.sw_decode_device(d_src, *args, nsrc=nsrc, nrep=len(hdr), sym_len=L, stride=stride) == 0
        torch.cuda.synchronize()
        assert c.sw_decode_errors() & fecgpu.SW_ERR_HEADER
        assert np.array_equal(d_st.cpu().numpy(), 1 - sp)
        assert np.array_equal(d_src.cpu().numpy(), d)
        with pytest.raises(fecgpu.FecError) as ei:
            c.sw_decode_device(d_src, *args, nsrc=nsrc, nrep=len(hdr), sym_len=L, stride=stride,
                               flags=fecgpu.F_SYNC)
        assert ei.value.code == fecgpu.ERR_INVALID_ARG
        assert np.array_equal(d_st.cpu().numpy(), 1 - sp)
        assert np.array_equal(d_src.cpu().numpy(), d)
    finally:
        c.close()


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


@pytest.mark.parametrize("loss,nsrc", [(0.02, 131072), (0.10, 131072), (0.02, 524288)])
def test_sw_full_size_roundtrip(ctx, loss, nsrc):
    """131,072 or 524,288 (config 7's stream: 256 chunks of the plan's look-back)
    sources of 1200 B, a repair after every 8 over the last 32, 2 %
    (config 7's rate) or 10 % i.i.d. loss of sources and repairs: every source the
    decoder reports recovered equals the original, and every status equals the
    oracle's global decode over the whole stream (at 10 % the repairs, 1 per 8
    sources, no longer cover the losses: long linked systems, mostly rank deficient)."""
    L, stride, k, W = 1200, 1200, 8, 32  # 524,288: config 7's stream (256 plan chunks)
    g = torch.Generator(device="cuda").manual_seed(7)
    d_src = torch.randint(0, 256, (nsrc, stride), dtype=torch.uint8, device="cuda", generator=g)
    h = N.sw_schedule(nsrc, k, W, key0=0)
    hdr = hdr_array(h)
    d_hdr = torch.from_numpy(hdr.view(np.uint8).copy()).cuda()
    d_rep = torch.empty((len(h), stride), dtype=torch.uint8, device="cuda")
    ctx.sw_encode(d_src, d_rep, d_hdr, nsrc=nsrc, nrep=len(h), sym_len=L, stride=stride, max_window=W)
    orig = d_src.clone()
    rng = np.random.default_rng(1)
    sp = (rng.random(nsrc) >= loss).astype(np.uint8)
    rp = (rng.random(len(h)) >= loss).astype(np.uint8)
    lost = torch.from_numpy(sp == 0).cuda()
    d_src[lost] = 0xCD
    st = np.zeros(nsrc, np.uint8)
    n = ctx.sw_decode(d_src, sp, d_rep, rp, hdr, st, nsrc=nsrc, nrep=len(h), sym_len=L, stride=stride)
    torch.cuda.synchronize()
    ok = torch.from_numpy(st == 0).cuda()
    assert torch.equal(d_src[ok], orig[ok])
    assert n == int(((sp == 0) & (st == 0)).sum()) and n > (0.9 if loss < 0.05 else 0.0) * (sp == 0).sum()
    # the whole stream against the banded oracle (equal to the dense one, test_sw_oracle.py)
    full = orig.cpu().numpy()
    od = full.copy()
    od[sp == 0] = 0xAB
    ost, on = O.sw_decode_banded(od, sp, d_rep.cpu().numpy(), rp, hdr, L)
    assert np.array_equal(st, ost) and n == on
    assert np.array_equal(od[ost == 0], full[ost == 0])


def test_sw_decode_device_config7_scale(ctx):
    """The bench's path at config 7's size: asynchronous fecgpu_sw_decode_device
    (bookkeeping on the device) raises no error flag and leaves exactly the
    statuses and bytes of the synchronous host-bookkeeping decode."""
    nsrc, L, stride, k, W = 524288, 1200, 1200, 8, 32
    g = torch.Generator(device="cuda").manual_seed(11)
    d_src = torch.randint(0, 256, (nsrc, stride), dtype=torch.uint8, device="cuda", generator=g)
    hdr = hdr_array(N.sw_schedule(nsrc, k, W, key0=3))
    d_hdr = torch.from_numpy(hdr.view(np.uint8).copy()).cuda()
    d_rep = torch.empty((len(hdr), stride), dtype=torch.uint8, device="cuda")
    ctx.sw_encode(d_src, d_rep, d_hdr, nsrc=nsrc, nrep=len(hdr), sym_len=L, stride=stride, max_window=W)
    rng = np.random.default_rng(2)
    sp = (rng.random(nsrc) >= 0.02).astype(np.uint8)
    rp = (rng.random(len(hdr)) >= 0.02).astype(np.uint8)
    lost = torch.from_numpy(sp == 0).cuda()
    orig = d_src.clone()
    d_src[lost] = 0xCD
    a_src = d_src.clone()
    st = np.zeros(nsrc, np.uint8)
    n = ctx.sw_decode(d_src, sp, d_rep, rp, hdr, st, nsrc=nsrc, nrep=len(hdr), sym_len=L, stride=stride)
    assert ctx.sw_decode_errors() == 0
    d_st = torch.full((nsrc,), 9, dtype=torch.uint8, device="cuda")
    for _ in range(3):  # back to back, as the bench's timed loop
        assert ctx.sw_decode_device(a_src, torch.from_numpy(sp).cuda(), d_rep, torch.from_numpy(rp).cuda(), d_hdr,
                                    d_st, nsrc=nsrc, nrep=len(hdr), sym_len=L, stride=stride) == 0
    assert ctx.sw_decode_errors() == 0
    torch.cuda.synchronize()
    assert np.array_equal(d_st.cpu().numpy(), st)
    assert torch.equal(a_src, d_src)
    ok = torch.from_numpy(st == 0).cuda()
    assert torch.equal(d_src[ok], orig[ok]) and n > 0.9 * (sp == 0).sum()


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
