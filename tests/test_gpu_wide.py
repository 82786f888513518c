"""GPU parity of GF(2^8) block codes with k + r > 64 (fec_wide.hip): repairs
equal the numpy oracle's (oracle/np_oracle.py encode) byte for byte; decode
recovers every window whose missing sources its present repairs determine,
bit-exact against the originals, with the oracle's status (np_oracle.decode,
which for RLC eliminates every received row); missing rows are poisoned
first.  Present masks are ceil((k + r) / 64) words per window.
PARITY UNPINNED vs the reference fec branch."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import fecgpu  # noqa: E402
import np_oracle as N  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    c = fecgpu.Context()
    yield c
    c.close()


def _scheme(matrix, key, dt):
    return {"cauchy": "gf", "vandermonde": "gf-vdm"}.get(matrix, f"rlc:{key}:{dt}")


def _masks(pres_bits: np.ndarray) -> np.ndarray:
    """[nwin, n] bool -> [nwin, words] u64 (bit i of word i // 64)."""
    nwin, n = pres_bits.shape
    words = (n + 63) // 64
    out = np.zeros((nwin, words), np.uint64)
    for i in range(n):
        out[:, i // 64] |= pres_bits[:, i].astype(np.uint64) << np.uint64(i % 64)
    return out


def _run(ctx, k, r, matrix, L, nwin, pres_bits, key=5, dt=15, sym_len=None, seed=0, m=fecgpu):
    n = k + r
    stride = (L + 15) // 16 * 16
    rng = np.random.default_rng(seed + k * 7 + r)
    wins = np.zeros((nwin, n, stride), np.uint8)
    wins[:, :k, :L] = rng.integers(0, 256, (nwin, k, L), dtype=np.uint8)
    code = m.Code("gf256", k, r, matrix=matrix, rlc_key=key, rlc_dt=dt)
    d = torch.from_numpy(wins.copy()).cuda()
    sl = None if sym_len is None else torch.from_numpy(sym_len).cuda()
    ctx.encode_batch(code, d, nwin=nwin, stride=stride, sym_len_all=L if sym_len is None else 0, sym_len=sl)
    torch.cuda.synchronize()
    enc = d.cpu().numpy()
    scheme = _scheme(matrix, key, dt)
    for w in range(nwin):
        S = L if sym_len is None else int(sym_len[w])
        ref = N.encode(scheme, k, r, wins[w, :k, :S])
        assert np.array_equal(enc[w, k:, :S], ref), f"window {w}: repairs differ"
    mask = torch.from_numpy(pres_bits).cuda()
    d[~mask] = 0xAB  # poison every missing symbol
    st = torch.full((nwin,), 7, dtype=torch.uint8, device="cuda")
    pres = torch.from_numpy(_masks(pres_bits).view(np.int64)).cuda()
    ctx.decode_batch(code, d, pres, st, nwin=nwin, stride=stride, sym_len_all=L if sym_len is None else 0,
                     sym_len=sl)
    torch.cuda.synchronize()
    got, gst = d.cpu().numpy(), st.cpu().numpy()
    for w in range(nwin):
        p = 0
        for i in np.flatnonzero(pres_bits[w]):
            p |= 1 << int(i)
        S = L if sym_len is None else int(sym_len[w])  # bytes past S_w are padding (fecgpu.h)
        sym = enc[w, :, :S].copy()
        sym[~pres_bits[w]] = 0xAB
        ref, ok = N.decode(scheme, k, r, sym, p)
        assert gst[w] == (0 if ok else 1), f"window {w}: status {gst[w]}, oracle ok={ok}"
        if ok:
            assert np.array_equal(got[w, :k, :S], wins[w, :k, :S]), f"window {w}: recovered bytes differ"
            assert np.array_equal(ref, wins[w, :k, :S])
    return gst


def _erasures(nwin, k, r, rng, max_e=None):
    """Per window: e in 0..r+1 missing sources, and 0..2 missing repairs."""
    n = k + r
    bits = np.ones((nwin, n), bool)
    for w in range(nwin):
        e = int(rng.integers(0, (max_e if max_e is not None else r + 1) + 1))
        bits[w, rng.choice(k, e, replace=False)] = False
        lr = int(rng.integers(0, min(3, r + 1)))
        if lr:
            bits[w, k + rng.choice(r, lr, replace=False)] = False
    return bits


@pytest.mark.parametrize("k,r,matrix,L", [(60, 8, "cauchy", 1200), (100, 4, "cauchy", 40),
                                          (200, 8, "cauchy", 1200), (248, 8, "cauchy", 300),
                                          (90, 6, "vandermonde", 1200), (150, 8, "rlc", 1200),
                                          (250, 6, "rlc", 64), (75, 5, "cauchy", 200),
                                          (180, 7, "vandermonde", 1200), (68, 4, "rlc", 16),
                                          # r < 4: the combine-job passes (the bit-sliced kernel takes r >= 4)
                                          (70, 2, "cauchy", 1200), (130, 3, "rlc", 500), (65, 1, "cauchy", 100)])
def test_wide_encode_decode_vs_oracle(ctx, k, r, matrix, L):
    nwin = 12
    rng = np.random.default_rng(k * 31 + r)
    bits = _erasures(nwin, k, r, rng)
    bits[0] = True            # nothing missing
    bits[1] = True
    bits[1, :r] = False       # exactly r sources, every repair present
    gst = _run(ctx, k, r, matrix, L, nwin, bits)
    assert gst[0] == 0 and gst[1] == 0


def test_wide_many_windows(ctx):
    """600 windows of k 120 r 8 (the bench's shape): the bit-sliced passes'
    flat unit space over many workgroups, and the two-stage decode's syndrome
    scratch past one workgroup's windows."""
    k, r, nwin = 120, 8, 600
    rng = np.random.default_rng(17)
    bits = _erasures(nwin, k, r, rng, max_e=r)
    gst = _run(ctx, k, r, "cauchy", 1200, nwin, bits)
    assert (gst == 0).sum() > nwin // 2


def test_wide_every_erasure_count(ctx):
    """k 120 r 8 Cauchy: e = 0..8 missing sources with every repair present (all
    recoverable), then e = 9 (never)."""
    k, r = 120, 8
    bits = np.ones((10, k + r), bool)
    rng = np.random.default_rng(3)
    for e in range(10):
        bits[e, rng.choice(k, e, replace=False)] = False
    gst = _run(ctx, k, r, "cauchy", 1200, 10, bits)
    assert list(gst) == [0] * 9 + [1]


def test_wide_per_window_lengths(ctx):
    """Per-window symbol lengths (sym_len): every byte below each window's length."""
    k, r, nwin, L = 80, 8, 8, 1200
    rng = np.random.default_rng(9)
    bits = _erasures(nwin, k, r, rng, max_e=r)
    sl = rng.integers(100, L + 1, nwin).astype(np.uint32)
    _run(ctx, k, r, "cauchy", L, nwin, bits, sym_len=sl)


@pytest.mark.parametrize("k,r,matrix,L", [(60, 8, "cauchy", 1200), (100, 4, "cauchy", 40),
                                          (200, 8, "cauchy", 1200), (248, 8, "cauchy", 300),
                                          (90, 6, "vandermonde", 1200), (150, 8, "rlc", 1200),
                                          (250, 6, "rlc", 64), (75, 5, "cauchy", 200),
                                          (180, 7, "vandermonde", 1200), (68, 4, "rlc", 16),
                                          # r < 4: the combine-job passes (the bit-sliced kernel takes r >= 4)
                                          (70, 2, "cauchy", 1200), (130, 3, "rlc", 500), (65, 1, "cauchy", 100)])
def test_wide_encode_decode_vs_oracle(ctx, k, r, matrix, L):
    nwin = 12
    rng = np.random.default_rng(k * 31 + r)
    bits = _erasures(nwin, k, r, rng)
    bits[0] = True            # nothing missing
    bits[1] = True
    bits[1, :r] = False       # exactly r sources, every repair present
    gst = _run(ctx, k, r, matrix, L, nwin, bits)
    assert gst[0] == 0 and gst[1] == 0


def test_wide_many_windows(ctx):
    """600 windows of k 120 r 8 (the bench's shape): the bit-sliced passes'
    flat unit space over many workgroups, and the two-stage decode's syndrome
    scratch past one workgroup's windows."""
    k, r, nwin = 120, 8, 600
    rng = np.random.default_rng(17)
    bits = _erasures(nwin, k, r, rng, max_e=r)
    gst = _run(ctx, k, r, "cauchy", 1200, nwin, bits)
    assert (gst == 0).sum() > nwin // 2


def test_wide_every_erasure_count(ctx):
    """k 120 r 8 Cauchy: e = 0..8 missing sources with every repair present (all
    recoverable), then e = 9 (never)."""
    k, r = 120, 8
    bits = np.ones((10, k + r), bool)
    rng = np.random.default_rng(3)
    for e in range(10):
        bits[e, rng.choice(k, e, replace=False)] = False
    gst = _run(ctx, k, r, "cauchy", 1200, 10, bits)
    assert list(gst) == [0] * 9 + [1]


def test_wide_per_window_lengths(ctx):
    """Per-window symbol lengths (sym_len): every byte below each window's length."""
    k, r, nwin, L = 80, 8, 8, 1200
    rng = np.random.default_rng(9)
    bits = _erasures(nwin, k, r, rng, max_e=r)
    sl = rng.integers(100, L + 1, nwin).astype(np.uint32)
    _run(ctx, k, r, "cauchy", L, nwin, bits, sym_len=sl)


@pytest.fixture(scope="module")
def bsctx():
    """A ctx with the bit-sliced wide decode on (tuning "bsd_min_e" > 0)."""
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    c = fecgpu.Context()
    c.set_tuning("bsd_min_e", 6)
    yield c
    c.close()


@pytest.mark.parametrize("k,r,matrix,L", [(60, 8, "cauchy", 1200), (120, 8, "cauchy", 1200), (248, 8, "cauchy", 300),
                                          (90, 6, "vandermonde", 1200), (150, 8, "rlc", 1200), (250, 6, "rlc", 64),
                                          (75, 5, "cauchy", 200), (68, 4, "rlc", 16)])
def test_wide_codes_every_erasure_count(ctx, k, r, matrix, L):
    """The wide decode (two stages, fec_wide.hip): bytes and statuses as the
    oracle's for every erasure count 0..r+1, then per-window lengths."""
    nwin = 40
    rng = np.random.default_rng(k * 13 + r)
    bits = _erasures(nwin, k, r, rng)
    for e in range(min(r + 2, nwin)):
        bits[e] = True
        bits[e, rng.choice(k, e, replace=False)] = False
    gst = _run(ctx, k, r, matrix, L, nwin, bits)
    if matrix == "cauchy":  # MDS: any e <= r present repairs suffice
        assert list(gst[:r + 2]) == [0] * (r + 1) + [1]
    sl = rng.integers(1, L + 1, nwin).astype(np.uint32)
    _run(ctx, k, r, matrix, L, nwin, bits, sym_len=sl, seed=1)


def test_wide_two_stage_path():
    """With the bit-sliced kernels off (tuning "bitslice" 0) the wide decode's two
    stages run as combine passes (fec_wide.hip): the same bytes and statuses."""
    c = fecgpu.Context()
    try:
        c.set_tuning("bitslice", 0)
        k, r, nwin = 120, 8, 24
        bits = _erasures(nwin, k, r, np.random.default_rng(21))
        _run(c, k, r, "cauchy", 700, nwin, bits)
    finally:
        c.close()


def test_wide_narrow_only_entry_points(ctx):
    """Per-connection objects, encode_split and the workload helpers keep k + r <= 64."""
    code = fecgpu.Code("gf256", 100, 4)
    with pytest.raises(fecgpu.FecError) as ei:
        fecgpu.Encoder(ctx, code, 1200, 4)
    assert ei.value.code == fecgpu.ERR_UNSUPPORTED
    src = torch.zeros((2, 100, 1200), dtype=torch.uint8, device="cuda")
    rep = torch.zeros((2, 4, 1200), dtype=torch.uint8, device="cuda")
    with pytest.raises(fecgpu.FecError) as ei:
        ctx.encode_split(code, src, rep, nwin=2, stride=1200, sym_len_all=1200)
    assert ei.value.code == fecgpu.ERR_UNSUPPORTED
    win = torch.zeros((2, 104, 1200), dtype=torch.uint8, device="cuda")
    with pytest.raises(fecgpu.FecError) as ei:
        ctx.encode_batch(code, win.cpu().numpy(), nwin=2, stride=1200, sym_len_all=1200, flags=fecgpu.F_HOST_PTRS)
    assert ei.value.code == fecgpu.ERR_UNSUPPORTED
