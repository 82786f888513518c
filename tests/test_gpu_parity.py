"""GPU parity: libfecgpu.so (gfx950 kernels, through the C ABI) vs the CPU oracle.

Bit-exact on every emitted byte [0, S) of every symbol; byte work has no
tolerance.  Sizes: small windows the oracle finishes in seconds, the committed
golden fixtures, and the BASELINE.json full sizes through size-independent
properties (encode -> erase -> decode round trip on every window, linearity)
plus sampled windows against the oracle.
PARITY UNPINNED vs the reference fec branch (not mounted).
"""
import glob
import itertools
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import fecgpu  # noqa: E402
import oracle as O  # noqa: E402
from fecgpu import workloads as WL  # noqa: E402

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
SEED = 1234567


@pytest.fixture(scope="module")
def ctx():
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    O.build()
    c = fecgpu.Context()
    yield c
    c.close()


def _scheme(s):
    return O.XOR if s == "xor" else O.GF256


def _cmp_emitted(a: np.ndarray, b: np.ndarray, S: np.ndarray, what: str):
    """Compare bytes [0, S_w) of every symbol of every window."""
    for w in range(a.shape[0]):
        s = int(S[w])
        if not np.array_equal(a[w, :, :s], b[w, :, :s]):
            bad = np.argwhere(a[w, :, :s] != b[w, :, :s])
            raise AssertionError(f"{what}: window {w} differs at (sym, byte) {bad[:5].tolist()}")


def gpu_run(ctx, scheme, k, r, wins, S, present, uniform: bool, poison=0xAB, matrix="cauchy",
            rlc=(0, 15)):
    """Encode on the GPU, poison erased symbols, decode on the GPU.
    Returns (encoded, decoded, status) as numpy.  rlc: (key, dt) of matrix 'rlc'."""
    nwin, n, stride = wins.shape
    code = fecgpu.Code(scheme, k, r, matrix=matrix, rlc_key=rlc[0], rlc_dt=rlc[1])
    d = torch.from_numpy(wins.copy()).cuda()
    sl = torch.from_numpy(S.astype(np.int32)).cuda()
    kw = dict(sym_len=None, sym_len_all=int(S[0])) if uniform else dict(sym_len=sl)
    ctx.encode_batch(code, d, nwin=nwin, stride=stride, **kw)
    torch.cuda.synchronize()
    enc = d.cpu().numpy()
    pres_t = torch.from_numpy(present.astype(np.int64)).cuda()
    mask = torch.from_numpy(np.array([[(int(p) >> i) & 1 for i in range(n)] for p in present],
                                     dtype=bool)).cuda()
    d[~mask] = poison
    status = torch.full((nwin,), 7, dtype=torch.uint8, device="cuda")
    ctx.decode_batch(code, d, pres_t, status, nwin=nwin, stride=stride, **kw)
    torch.cuda.synchronize()
    return enc, d.cpu().numpy(), status.cpu().numpy()


def oracle_run(scheme, k, r, wins, S, present, poison=0xAB, oscheme=None):
    osc = _scheme(scheme) if oscheme is None else oscheme
    enc = wins.copy()
    O.encode_batch(osc, k, r, S, enc, 4)
    dec = enc.copy()
    O.erase(dec, present, k, r, fill=poison)
    st = O.decode_batch(osc, k, r, S, dec, present, 4)
    return enc, dec, st


CASES = [
    # scheme, k, r, workload, L, erasure, nwin
    ("xor", 8, 2, 0, 1200, 1, 64),
    ("xor", 4, 1, 0, 100, 1, 33),
    ("xor", 5, 3, 0, 17, 2, 64),
    ("xor", 8, 2, 1, 0, 2, 12),
    ("xor", 8, 8, 0, 48, 2, 40),
    ("gf256", 16, 4, 0, 1200, 1, 64),
    ("gf256", 32, 8, 1, 0, 2, 12),
    ("gf256", 1, 1, 0, 1, 1, 5),
    ("gf256", 56, 8, 0, 64, 1, 9),
    ("gf256", 10, 7, 0, 33, 2, 70),
    ("gf256", 3, 5, 0, 16, 1, 8),
    ("gf256", 8, 2, 0, 1500, 2, 100),
    ("gf256", 20, 6, 1, 0, 1, 6),
]


@pytest.mark.parametrize("scheme,k,r,wl,L,era,nwin", CASES)
def test_encode_decode_vs_oracle(ctx, scheme, k, r, wl, L, era, nwin):
    S = O.sym_lens(wl, SEED, 0, nwin, k, L)
    stride = O.round_up(int(S.max()), 16) + (16 if wl == 0 else 0)
    wins = O.make_windows(wl, SEED, 0, nwin, k, r, L, stride)
    present = O.presents(era, SEED, 0, nwin, _scheme(scheme), k, r)
    ge, gd, gs = gpu_run(ctx, scheme, k, r, wins, S, present, uniform=(wl == 0))
    oe, od, os_ = oracle_run(scheme, k, r, wins, S, present)
    _cmp_emitted(ge, oe, S, "encode")
    assert np.array_equal(gs, os_), (gs, os_)
    _cmp_emitted(gd, od, S, "decode")
    # recovered windows equal the original sources
    for w in range(nwin):
        if gs[w] == 0:
            s = int(S[w])
            assert np.array_equal(gd[w, :k, :s], wins[w, :k, :s])


@pytest.mark.parametrize("scheme,k,r", [("gf256", 4, 3), ("xor", 6, 3), ("gf256", 5, 2),
                                        ("xor", 3, 1)])
def test_every_erasure_pattern(ctx, scheme, k, r):
    """All 2^(k+r) present masks, one window each: status and bytes vs oracle."""
    n = k + r
    nwin = 1 << n
    L = 40
    wins = O.make_windows(0, SEED, 7, 1, k, r, L, 48)
    wins = np.repeat(wins, nwin, axis=0)
    S = np.full(nwin, L, np.uint32)
    present = np.arange(nwin, dtype=np.uint64)
    ge, gd, gs = gpu_run(ctx, scheme, k, r, wins, S, present, uniform=True)
    oe, od, os_ = oracle_run(scheme, k, r, wins, S, present)
    _cmp_emitted(ge, oe, S, "encode")
    assert np.array_equal(gs, os_)
    _cmp_emitted(gd, od, S, "decode")
    if scheme == "gf256":  # MDS: recoverable iff missing sources <= present repairs
        for p in range(nwin):
            miss = sum(1 for j in range(k) if not (p >> j) & 1)
            reps = sum(1 for i in range(r) if (p >> (k + i)) & 1)
            assert gs[p] == (0 if miss <= reps else 1)


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(HERE, "golden", "*.npz"))),
                         ids=lambda p: os.path.basename(p)[:-4])
def test_golden_fixtures(ctx, path):
    z = np.load(path)
    scheme_id, k, r, L, era, nwin, w0, seed = (int(x) for x in z["meta"])
    scheme = "xor" if scheme_id == 0 else "gf256"
    matrix = {2: "vandermonde", 3: "rlc"}.get(scheme_id & 0xF, "cauchy")
    rlc = ((scheme_id >> 8) & 0xFFFF, (scheme_id >> 4) & 0xF)
    stride = O.round_up(L, 16)
    wins = np.zeros((nwin, k + r, stride), np.uint8)
    wins[:, :k, :L] = z["src"]
    S = np.full(nwin, L, np.uint32)
    ge, gd, gs = gpu_run(ctx, scheme, k, r, wins, S, z["present"], uniform=True, matrix=matrix, rlc=rlc)
    assert np.array_equal(ge[:, k:, :L], z["repair"])
    assert np.array_equal(gs, z["status"])
    ok = z["status"] == 0
    assert np.array_equal(gd[ok, :k, :L], z["decoded"][ok])


def test_ragged_layout(ctx):
    """win_off != NULL: per-window stride round_up(S_w, 16), windows at arbitrary 16-B offsets."""
    k, r, nwin = 6, 3, 17
    rng = np.random.default_rng(5)
    S = rng.integers(1, 300, nwin).astype(np.uint32)
    strides = [O.round_up(int(s), 16) for s in S]
    offs, pos = [], 0
    for w in range(nwin):
        pos += 16 * int(rng.integers(0, 4))
        offs.append(pos)
        pos += (k + r) * strides[w]
    for scheme in ("gf256", "xor"):
        buf = np.zeros(pos + 64, np.uint8)
        ref = []
        for w in range(nwin):
            win = np.zeros((k + r, strides[w]), np.uint8)
            win[:k, :S[w]] = rng.integers(0, 256, (k, int(S[w])), dtype=np.uint8)
            ref.append(win)
            buf[offs[w]:offs[w] + win.size] = win.ravel()
        present = O.presents(1, SEED, 0, nwin, _scheme(scheme), k, r)
        d = torch.from_numpy(buf).cuda()
        off_t = torch.tensor(offs, dtype=torch.int64).cuda()
        sl = torch.from_numpy(S.astype(np.int32)).cuda()
        code = fecgpu.Code(scheme, k, r)
        ctx.encode_batch(code, d, nwin=nwin, stride=0, sym_len=sl, win_off=off_t)
        st = torch.zeros(nwin, dtype=torch.uint8, device="cuda")
        enc = d.cpu().numpy()
        for w in range(nwin):  # erase in place on device
            for i in range(k + r):
                if not (int(present[w]) >> i) & 1:
                    a = offs[w] + i * strides[w]
                    d[a:a + strides[w]] = 0xCD
        ctx.decode_batch(code, d, torch.from_numpy(present.astype(np.int64)).cuda(), st,
                         nwin=nwin, stride=0, sym_len=sl, win_off=off_t)
        out = d.cpu().numpy()
        for w in range(nwin):
            o = ref[w].copy()
            O.encode_batch(_scheme(scheme), k, r, np.array([S[w]], np.uint32), o[None], 1)
            got = enc[offs[w]:offs[w] + o.size].reshape(o.shape)
            assert np.array_equal(got[:, :S[w]], o[:, :S[w]]), (scheme, w)
            rec = out[offs[w]:offs[w] + o.size].reshape(o.shape)
            assert st[w].item() == 0
            assert np.array_equal(rec[:k, :S[w]], o[:k, :S[w]]), (scheme, w)


def test_host_pointer_mode(ctx):
    k, r, nwin, L = 16, 4, 50, 1200
    S = np.full(nwin, L, np.uint32)
    wins = O.make_windows(0, SEED, 0, nwin, k, r, L, 1216)
    present = O.presents(1, SEED, 0, nwin, O.GF256, k, r)
    code = fecgpu.Code("gf256", k, r)
    h = wins.copy()
    ctx.encode_batch(code, h, nwin=nwin, stride=1216, sym_len_all=L, flags=fecgpu.F_HOST_PTRS)
    oe, od, os_ = oracle_run("gf256", k, r, wins, S, present)
    _cmp_emitted(h, oe, S, "host encode")
    O.erase(h, present, k, r, fill=0x11)
    st = np.zeros(nwin, np.uint8)
    ctx.decode_batch(code, h, present, st, nwin=nwin, stride=1216, sym_len_all=L,
                     flags=fecgpu.F_HOST_PTRS)
    assert np.array_equal(st, os_)
    _cmp_emitted(h, od, S, "host decode")


@pytest.mark.parametrize("cfgid,direct", [(5, 6), (6, 6), (5, 0), (6, 0), (6, 3), (5, 7), (6, 7)])
def test_pinned_host_pipeline_matches_device_path(ctx, cfgid, direct):
    """FECGPU_F_HOST_PTRS over pinned memory, > 3 pipeline chunks (slot reuse): repairs
    and recovered sources equal the device-resident path on the same windows, with
    the kernels storing straight into the mapped host windows (direct bit 0 encode,
    bit 1 decode), reading them too (bit 2), and with H2D/D2H copies only (0)."""
    ctx.set_tuning("host_direct", direct)
    cfg = WL.CONFIGS[cfgid]
    nwin = 40000  # 480 MB of windows -> 8 chunks of 64 MB
    hb = WL.HostBatch.allocate(cfg, nwin, torch.device("cuda"))
    hb.synthesize(ctx, 77)
    db = WL.Batch.allocate(cfg, nwin, torch.device("cuda"))
    db.synthesize(ctx, 77)
    db.make_erasures(ctx, 77)
    assert np.array_equal(hb.present, db.present.cpu().numpy().view(np.uint64))
    hb.encode(ctx)
    db.encode(ctx)
    torch.cuda.synchronize()
    assert np.array_equal(hb.buf.array, db.win.cpu().numpy())
    res = hb.verify(ctx, 77)
    ctx.set_tuning("host_direct", 6)
    assert res["ok"] and res["unrecoverable"] == 0, res
    hb.buf.close()


@pytest.mark.parametrize("scheme,k,r", [("gf256", 32, 8), ("xor", 8, 2)])
@pytest.mark.parametrize("direct", [0, 6, 7])
def test_pinned_host_mixed_mtu_vs_oracle(ctx, scheme, k, r, direct):
    """Host pipeline on per-window symbol lengths (mixed MTU, LENPREFIX, i.i.d.
    erasures), 1 MiB chunks so the 3 staging slots are reused many times: encode and
    decode through pinned host windows equal the oracle, for copies only, zero-copy
    decode, and zero-copy + direct stores on both sides."""
    nwin = 150
    S = O.sym_lens(1, SEED, 0, nwin, k, 0)
    stride = O.round_up(int(S.max()), 16)
    wins = O.make_windows(1, SEED, 0, nwin, k, r, 0, stride)
    present = O.presents(2, SEED, 0, nwin, _scheme(scheme), k, r)
    oe, od, os_ = oracle_run(scheme, k, r, wins, S, present)
    code = fecgpu.Code(scheme, k, r)
    buf = fecgpu.PinnedBuffer(wins.nbytes)
    h = buf.array.reshape(wins.shape)
    h[:] = wins
    ctx.set_tuning("host_direct", direct)
    ctx.set_tuning("host_chunk_mb", 1)
    try:
        ctx.encode_batch(code, h, nwin=nwin, stride=stride, sym_len=S, flags=fecgpu.F_HOST_PTRS)
        enc = h.copy()
        O.erase(h, present, k, r, fill=0xAB)  # the oracle_run poison
        st = np.full(nwin, 9, np.uint8)
        ctx.decode_batch(code, h, present, st, nwin=nwin, stride=stride, sym_len=S,
                         flags=fecgpu.F_HOST_PTRS)
        dec = h.copy()
    finally:
        ctx.set_tuning("host_direct", 6)
        ctx.set_tuning("host_chunk_mb", 128)
        del h
        buf.close()  # no view of the freed pages may outlive this (pytest reprs locals)
    _cmp_emitted(enc, oe, S, "host encode")
    assert np.array_equal(st, os_), np.nonzero(st != os_)
    _cmp_emitted(dec, od, S, "host decode")


@pytest.mark.parametrize("scheme,k,r,wl,L", [("xor", 8, 2, 0, 1200), ("gf256", 16, 4, 0, 1200),
                                              ("gf256", 32, 8, 1, 0), ("xor", 5, 3, 1, 0),
                                              ("gf256", 4, 7, 0, 100)])
def test_encode_split_layout_vs_oracle(ctx, scheme, k, r, wl, L):
    """fecgpu_encode_split (SURVEY §8b form: src[W][k][stride] in, repair[W][r][stride]
    out) equals the oracle's repairs and leaves the sources untouched (r > k too)."""
    nwin = 37
    S = O.sym_lens(wl, SEED, 0, nwin, k, L)
    stride = O.round_up(int(S.max()), 16)
    wins = O.make_windows(wl, SEED, 0, nwin, k, r, L, stride)
    oe, _, _ = oracle_run(scheme, k, r, wins, S, np.full(nwin, (1 << (k + r)) - 1, np.uint64))
    src = torch.from_numpy(np.ascontiguousarray(wins[:, :k])).cuda()
    rep = torch.full((nwin, r, stride), 0x77, dtype=torch.uint8, device="cuda")
    kw = dict(sym_len_all=int(S[0])) if wl == 0 else dict(sym_len=torch.from_numpy(S.astype(np.int32)).cuda())
    ctx.encode_split(fecgpu.Code(scheme, k, r), src, rep, nwin=nwin, stride=stride, **kw)
    torch.cuda.synchronize()
    got = np.concatenate([src.cpu().numpy(), rep.cpu().numpy()], axis=1)
    assert np.array_equal(got[:, :k], wins[:, :k])
    _cmp_emitted(got, oe, S, "encode_split")


VDM_CASES = [(5, 5, 0, 2, 1, 9), (8, 2, 0, 1200, 1, 64), (16, 4, 0, 1200, 2, 64),
             (32, 8, 1, 0, 2, 12), (56, 8, 0, 64, 1, 9), (3, 7, 0, 33, 2, 40)]


@pytest.mark.parametrize("k,r,wl,L,era,nwin", VDM_CASES)
def test_vandermonde_matrix_vs_oracle(ctx, k, r, wl, L, era, nwin):
    """FECGPU_MATRIX_VANDERMONDE (systematic Vandermonde rows, decode through the
    general-matrix Gauss-Jordan plan) vs the oracle: repairs, status and recovered
    bytes."""
    S = O.sym_lens(wl, SEED, 0, nwin, k, L)
    stride = O.round_up(int(S.max()), 16)
    wins = O.make_windows(wl, SEED, 0, nwin, k, r, L, stride)
    present = O.presents(era, SEED, 0, nwin, O.GF256_VDM, k, r)
    code = fecgpu.Code("gf256", k, r, matrix="vandermonde")
    d = torch.from_numpy(wins.copy()).cuda()
    kw = dict(sym_len_all=int(S[0])) if wl == 0 else dict(sym_len=torch.from_numpy(S.astype(np.int32)).cuda())
    ctx.encode_batch(code, d, nwin=nwin, stride=stride, **kw)
    torch.cuda.synchronize()
    ge = d.cpu().numpy()
    oe = wins.copy()
    O.encode_batch(O.GF256_VDM, k, r, S, oe, 4)
    _cmp_emitted(ge, oe, S, "vdm encode")
    od = oe.copy()
    O.erase(od, present, k, r, fill=0xAB)
    os_ = O.decode_batch(O.GF256_VDM, k, r, S, od, present, 4)
    mask = torch.from_numpy(np.array([[(int(p) >> i) & 1 for i in range(k + r)] for p in present],
                                     dtype=bool)).cuda()
    d[~mask] = 0xAB
    st = torch.full((nwin,), 7, dtype=torch.uint8, device="cuda")
    ctx.decode_batch(code, d, torch.from_numpy(present.astype(np.int64)).cuda(), st, nwin=nwin,
                     stride=stride, **kw)
    torch.cuda.synchronize()
    assert np.array_equal(st.cpu().numpy(), os_)
    _cmp_emitted(d.cpu().numpy(), od, S, "vdm decode")


def test_vandermonde_kat_on_gpu(ctx):
    """The published 5+5 known answer through the GPU encode."""
    code = fecgpu.Code("gf256", 5, 5, matrix="vandermonde")
    win = np.zeros((1, 10, 16), np.uint8)
    win[0, :5, :2] = [[0, 1], [4, 5], [2, 3], [6, 7], [8, 9]]
    d = torch.from_numpy(win).cuda()
    ctx.encode_batch(code, d, nwin=1, stride=16, sym_len_all=2)
    torch.cuda.synchronize()
    assert d.cpu().numpy()[0, 5:, :2].tolist() == [[12, 13], [10, 11], [14, 15], [90, 91], [94, 95]]


@pytest.mark.parametrize("k,r", [(4, 3), (5, 5), (6, 2)])
def test_vandermonde_every_erasure_pattern(ctx, k, r):
    n = k + r
    nwin = 1 << n
    wins = np.repeat(O.make_windows(0, SEED, 3, 1, k, r, 40, 48), nwin, axis=0)
    S = np.full(nwin, 40, np.uint32)
    present = np.arange(nwin, dtype=np.uint64)
    code = fecgpu.Code("gf256", k, r, matrix="vandermonde")
    d = torch.from_numpy(wins.copy()).cuda()
    ctx.encode_batch(code, d, nwin=nwin, stride=48, sym_len_all=40)
    torch.cuda.synchronize()
    enc = d.cpu().numpy()
    mask = torch.from_numpy(np.array([[(p >> i) & 1 for i in range(n)] for p in range(nwin)],
                                     dtype=bool)).cuda()
    d[~mask] = 0x3C
    st = torch.full((nwin,), 7, dtype=torch.uint8, device="cuda")
    ctx.decode_batch(code, d, torch.from_numpy(present.astype(np.int64)).cuda(), st, nwin=nwin,
                     stride=48, sym_len_all=40)
    torch.cuda.synchronize()
    got, st = d.cpu().numpy(), st.cpu().numpy()
    for p in range(nwin):
        miss = sum(1 for j in range(k) if not (p >> j) & 1)
        reps = sum(1 for i in range(r) if (p >> (k + i)) & 1)
        assert st[p] == (0 if miss <= reps else 1), p
        if st[p] == 0:
            assert np.array_equal(got[p, :k, :40], enc[p, :k, :40]), p


@pytest.mark.parametrize("devs", [[0, 0], [0, 0, 0]])
def test_multi_device_ctx_host_batches(ctx, devs):
    """A ctx over several devices splits host-pointer batches into contiguous
    window ranges, one host thread and pipeline per device (the one-GPU box lists
    device 0 several times): same repairs, status and recovered bytes as the
    oracle, for uniform and per-window lengths."""
    multi = fecgpu.Context(devs)
    try:
        for scheme, k, r, wl, L, era in (("xor", 8, 2, 0, 1200, 1), ("gf256", 32, 8, 1, 0, 2)):
            nwin = 61
            S = O.sym_lens(wl, SEED, 5, nwin, k, L)
            stride = O.round_up(int(S.max()), 16)
            wins = O.make_windows(wl, SEED, 5, nwin, k, r, L, stride)
            present = O.presents(era, SEED, 5, nwin, _scheme(scheme), k, r)
            oe, od, os_ = oracle_run(scheme, k, r, wins, S, present)
            code = fecgpu.Code(scheme, k, r)
            buf = fecgpu.PinnedBuffer(wins.nbytes)
            h = buf.array.reshape(wins.shape)
            h[:] = wins
            kw = dict(sym_len_all=L) if wl == 0 else dict(sym_len=S)
            multi.set_tuning("host_chunk_mb", 1)
            multi.encode_batch(code, h, nwin=nwin, stride=stride, flags=fecgpu.F_HOST_PTRS, **kw)
            enc = h.copy()
            O.erase(h, present, k, r, fill=0xAB)
            st = np.full(nwin, 9, np.uint8)
            multi.decode_batch(code, h, present, st, nwin=nwin, stride=stride,
                               flags=fecgpu.F_HOST_PTRS, **kw)
            dec = h.copy()
            del h
            buf.close()
            _cmp_emitted(enc, oe, S, f"multi encode {scheme}")
            assert np.array_equal(st, os_)
            _cmp_emitted(dec, od, S, f"multi decode {scheme}")
    finally:
        multi.close()


def test_zero_windows_and_errors(ctx):
    code = fecgpu.Code("gf256", 4, 2)
    d = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    assert ctx.encode_batch(code, d, nwin=0, stride=64, sym_len_all=10) == 0
    with pytest.raises(fecgpu.FecError) as e:
        ctx.encode_batch(code, d, nwin=1, stride=60, sym_len_all=10)  # stride % 16
    assert e.value.code == fecgpu.ERR_INVALID_ARG
    with pytest.raises(fecgpu.FecError) as e:
        ctx.encode_batch(code, d, nwin=1, stride=64, sym_len_all=100)  # S > stride
    assert e.value.code == fecgpu.ERR_BUFFER_TOO_SHORT
    with pytest.raises(fecgpu.FecError) as e:
        ctx.encode_batch(fecgpu.Code("gf256", 60, 9), d, nwin=1, stride=64, sym_len_all=10)
    assert e.value.code == fecgpu.ERR_UNSUPPORTED
    with pytest.raises(fecgpu.FecError) as e:  # pitch over FECGPU_MAX_SYMBOL (16 MiB)
        ctx.encode_batch(code, d, nwin=1, stride=1 << 25, sym_len_all=10)
    assert e.value.code == fecgpu.ERR_UNSUPPORTED


@pytest.mark.parametrize("scheme,k,r,L", [("xor", 8, 2, 1200), ("gf256", 16, 4, 1200),
                                          ("gf256", 32, 8, 1200), ("gf256", 32, 8, 9000),
                                          ("xor", 1, 1, 16), ("gf256", 64 - 8, 8, 33)])
@pytest.mark.parametrize("uniform", [True, False])
def test_single_window(ctx, scheme, k, r, L, uniform):
    """One window: the tiny-grid paths (fewer work units than XCD regions) of the
    flat, group and bit-sliced kernels, encode and decode vs the oracle."""
    S = np.full(1, L, np.uint32)
    stride = O.round_up(L, 16)
    wins = O.make_windows(0, SEED + 3, 0, 1, k, r, L, stride)
    present = O.presents(1, SEED + 3, 0, 1, _scheme(scheme), k, r)
    ge, gd, gs = gpu_run(ctx, scheme, k, r, wins, S, present, uniform)
    oe, od, os_ = oracle_run(scheme, k, r, wins, S, present)
    _cmp_emitted(ge, oe, S, "encode")
    assert np.array_equal(gs, os_)
    _cmp_emitted(gd, od, S, "decode")


@pytest.mark.parametrize("scheme,k,r", [("xor", 4, 2), ("gf256", 4, 2), ("gf256", 16, 8)])
def test_megabyte_symbols(ctx, scheme, k, r):
    """Symbols far above any MTU (1 MiB + 5 B, 3 windows): 64-bit window offsets,
    long column loops, the last partial 16-B column."""
    L = (1 << 20) + 5
    stride = O.round_up(L, 16)
    nwin = 3
    S = np.full(nwin, L, np.uint32)
    wins = O.make_windows(0, SEED + 5, 0, nwin, k, r, L, stride)
    present = O.presents(1, SEED + 5, 0, nwin, _scheme(scheme), k, r)
    ge, gd, gs = gpu_run(ctx, scheme, k, r, wins, S, present, True)
    oe, od, os_ = oracle_run(scheme, k, r, wins, S, present)
    _cmp_emitted(ge, oe, S, "encode")
    assert np.array_equal(gs, os_)
    _cmp_emitted(gd, od, S, "decode")


def _random_cases(n, seed):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        scheme = ["xor", "gf256", "gf256"][int(rng.integers(0, 3))]
        k = int(rng.integers(1, 57))
        r = int(rng.integers(1, min(8, 64 - k, k if scheme == "xor" else 8) + 1))
        matrix = "vandermonde" if scheme == "gf256" and rng.random() < 0.3 else "cauchy"
        out.append((scheme, matrix, k, r, int(rng.integers(1, 3001)), int(rng.integers(1, 41)),
                    bool(rng.random() < 0.5), int(rng.integers(1, 3))))
    return out


@pytest.mark.parametrize("scheme,matrix,k,r,L,nwin,uniform,era", _random_cases(40, 2026))
def test_random_shapes_vs_oracle(ctx, scheme, matrix, k, r, L, nwin, uniform, era):
    """Seeded random codes and shapes (k 1..56, r 1..8, S 1..3000, 1..40 windows, both
    matrices, uniform or per-window S, exact-r or i.i.d. erasures) vs the oracle."""
    sid = _scheme(scheme) if matrix == "cauchy" else O.GF256_VDM
    rng = np.random.default_rng(k * 1000 + L)
    S = np.full(nwin, L, np.uint32) if uniform else rng.integers(1, L + 1, nwin).astype(np.uint32)
    stride = O.round_up(int(S.max()), 16)
    wins = np.zeros((nwin, k + r, stride), np.uint8)
    for w in range(nwin):
        wins[w, :k, :S[w]] = rng.integers(0, 256, (k, int(S[w])), dtype=np.uint8)
    present = O.presents(era, SEED + k, 0, nwin, sid, k, r)
    ge, gd, gs = gpu_run(ctx, scheme, k, r, wins, S, present, uniform, matrix=matrix)
    oe = wins.copy()
    O.encode_batch(sid, k, r, S, oe, 4)
    od = oe.copy()
    O.erase(od, present, k, r, fill=0xAB)
    os_ = O.decode_batch(sid, k, r, S, od, present, 4)
    _cmp_emitted(ge, oe, S, "encode")
    assert np.array_equal(gs, os_)
    _cmp_emitted(gd, od, S, "decode")


# ------------------------------------------------ workload generators ---
@pytest.mark.parametrize("cfgid", [2, 3, 4])
def test_synth_erasure_digest_vs_oracle(ctx, cfgid):
    cfg = WL.CONFIGS[cfgid]
    nwin, w0 = 24, 1000
    b = WL.Batch.allocate(cfg, nwin, torch.device("cuda"))
    b.synthesize(ctx, w0)
    b.make_erasures(ctx, w0)
    torch.cuda.synchronize()
    S = O.sym_lens(cfg.workload, WL.SEED, w0, nwin, cfg.k, cfg.L)
    wins = O.make_windows(cfg.workload, WL.SEED, w0, nwin, cfg.k, cfg.r, cfg.L, cfg.stride)
    got = b.view.cpu().numpy()
    assert np.array_equal(got[:, :cfg.k], wins[:, :cfg.k])
    if cfg.workload == 1:
        assert np.array_equal(b.sym_len.cpu().numpy().astype(np.uint32), S)
    pres = O.presents(cfg.erasure, WL.SEED, w0, nwin, _scheme(cfg.scheme), cfg.k, cfg.r)
    assert np.array_equal(b.present.cpu().numpy().astype(np.uint64), pres)
    b.encode(ctx)
    dg = torch.zeros(1, dtype=torch.int64, device="cuda")
    ctx.digest_batch(cfg.code, b.win, dg, nwin=nwin, stride=cfg.stride, w0=w0,
                     **b._len_args())
    O.encode_batch(_scheme(cfg.scheme), cfg.k, cfg.r, S, wins, 4)
    want = O.batch_digest(cfg.k, cfg.r, S, wins, w0)
    assert (int(dg.item()) & (2**64 - 1)) == want


# --------------------------------------------------- full BASELINE sizes ---
@pytest.mark.parametrize("cfgid,nwin", [(2, 65536), (3, 262144), (4, 131072)])
def test_full_size_roundtrip(ctx, cfgid, nwin):
    """Every window: encode -> poison erased -> decode == original sources, status as
    predicted from the masks; 64 sampled windows bit-exact vs the oracle.  cfg4 runs
    its real per-GPU shard (1M windows / 8 GPUs = 131,072 windows, 47 GB + a 38 GB
    saved copy of the sources in HBM)."""
    cfg = WL.CONFIGS[cfgid]
    b = WL.Batch.allocate(cfg, nwin, torch.device("cuda"))
    b.synthesize(ctx, 0)
    b.make_erasures(ctx, 0)
    b.encode(ctx)
    torch.cuda.synchronize()
    rng = np.random.default_rng(cfgid)
    sample = np.sort(rng.choice(nwin, 64, replace=False))
    enc = b.view[torch.from_numpy(sample).cuda()].cpu().numpy()
    res = b.verify(ctx, 0)
    assert res["ok"], res
    if cfgid != 4:
        assert res["unrecoverable"] == 0
    for i, w in enumerate(sample):
        S = O.sym_lens(cfg.workload, WL.SEED, int(w), 1, cfg.k, cfg.L)
        win = O.make_windows(cfg.workload, WL.SEED, int(w), 1, cfg.k, cfg.r, cfg.L, cfg.stride)
        O.encode_batch(_scheme(cfg.scheme), cfg.k, cfg.r, S, win, 1)
        _cmp_emitted(enc[i:i + 1], win, S, f"cfg{cfgid} window {w}")


def test_linearity_full_size(ctx):
    """encode(A xor B) == encode(A) xor encode(B) over 262,144 k=16 r=4 windows."""
    cfg = WL.CONFIGS[3]
    nwin = 262144
    a = WL.Batch.allocate(cfg, nwin, torch.device("cuda"))
    a.synthesize(ctx, 0)
    bsrc = a.view[:, :cfg.k].roll(1, dims=0).clone()
    a.encode(ctx)
    ra = a.view[:, cfg.k:].clone()
    a.view[:, :cfg.k] = bsrc
    a.encode(ctx)
    rb = a.view[:, cfg.k:].clone()
    a.synthesize(ctx, 0)
    a.view[:, :cfg.k] ^= bsrc
    a.encode(ctx)
    assert torch.equal(a.view[:, cfg.k:], ra ^ rb)


# (16|24|32, 8) and (16, 4): compiled masks (16, 4 on uniform short rows with the
# repairs gathered in LDS, gf_encode_bs_gs_kernel); r >= 5 otherwise: runtime
# masks (rbs); (8, 8): table kernel
BS_CODES = [(16, 8), (24, 8), (32, 8), (8, 8), (16, 4), (1, 5), (13, 6), (45, 7), (56, 8)]


@pytest.fixture(scope="module")
def ctx_tables():
    """A second context with the bit-sliced encode switched off (table multiply)."""
    c = fecgpu.Context()
    c.set_tuning("bitslice", 0)
    yield c
    c.close()


@pytest.mark.parametrize("matrix", ["cauchy", "vandermonde"])
@pytest.mark.parametrize("k,r", BS_CODES)
@pytest.mark.parametrize("wl,L,nwin", [(0, 1200, 70), (1, 0, 9), (0, 16, 33), (0, 1, 5), (0, 9000, 6)])
def test_bitslice_encode_vs_oracle(ctx, ctx_tables, k, r, wl, L, nwin, matrix):
    """The bit-sliced GF encodes (compile-time parity rows, Cauchy or systematic
    Vandermonde, and runtime plane masks for the other codes with r >= 5,
    DESIGN.md §GF bit-slicing) emit the oracle's repairs for every code: odd column counts (1200 B: 75 columns, the last unit without a
    second column), one column (16 B), S = 1, per-window lengths (mixed MTU,
    LENPREFIX) and 9000-B symbols; and the same bytes as the table-multiply kernel."""
    S = O.sym_lens(wl, SEED + k, 0, nwin, k, L)
    stride = O.round_up(int(S.max()), 16) + (16 if wl == 0 else 0)
    wins = O.make_windows(wl, SEED + k, 0, nwin, k, r, L, stride)
    oe = wins.copy()
    O.encode_batch(O.GF256 if matrix == "cauchy" else O.GF256_VDM, k, r, S, oe, 4)
    code = fecgpu.Code("gf256", k, r, matrix=matrix)
    outs = []
    for c in (ctx, ctx_tables):
        d = torch.from_numpy(wins.copy()).cuda()
        kw = dict(sym_len_all=int(S[0])) if wl == 0 else dict(sym_len=torch.from_numpy(S.astype(np.int32)).cuda())
        c.encode_batch(code, d, nwin=nwin, stride=stride, **kw)
        torch.cuda.synchronize()
        outs.append(d.cpu().numpy())
    _cmp_emitted(outs[0], oe, S, "bit-sliced encode")
    _cmp_emitted(outs[1], oe, S, "table encode")


@pytest.mark.parametrize("k,r", [(16, 8), (32, 8), (8, 8), (20, 5), (16, 4)])
def test_bitslice_ragged_and_split(ctx, k, r):
    """Bit-sliced encode through the ragged (win_off) and split (src / repair arrays) layouts."""
    nwin = 11
    rng = np.random.default_rng(k)
    S = rng.integers(1, 2000, nwin).astype(np.uint32)
    strides = [O.round_up(int(s), 16) for s in S]
    offs, pos = [], 0
    for w in range(nwin):
        pos += 16 * int(rng.integers(0, 3))
        offs.append(pos)
        pos += (k + r) * strides[w]
    buf = np.zeros(pos + 64, np.uint8)
    ref = []
    for w in range(nwin):
        win = np.zeros((k + r, strides[w]), np.uint8)
        win[:k, :S[w]] = rng.integers(0, 256, (k, int(S[w])), dtype=np.uint8)
        buf[offs[w]:offs[w] + win.size] = win.ravel()
        O.encode_batch(O.GF256, k, r, np.array([S[w]], np.uint32), win[None], 1)
        ref.append(win)
    d = torch.from_numpy(buf).cuda()
    ctx.encode_batch(fecgpu.Code("gf256", k, r), d, nwin=nwin, stride=0,
                     sym_len=torch.from_numpy(S.astype(np.int32)).cuda(),
                     win_off=torch.tensor(offs, dtype=torch.int64).cuda())
    out = d.cpu().numpy()
    for w in range(nwin):
        got = out[offs[w]:offs[w] + ref[w].size].reshape(ref[w].shape)
        assert np.array_equal(got[:, :S[w]], ref[w][:, :S[w]]), w
    # split layout, uniform S
    Su = np.full(nwin, 1100, np.uint32)
    wins = O.make_windows(0, SEED, 0, nwin, k, r, 1100, 1104)
    oe = wins.copy()
    O.encode_batch(O.GF256, k, r, Su, oe, 2)
    src = torch.from_numpy(np.ascontiguousarray(wins[:, :k])).cuda()
    rep = torch.full((nwin, r, 1104), 0x55, dtype=torch.uint8, device="cuda")
    ctx.encode_split(fecgpu.Code("gf256", k, r), src, rep, nwin=nwin, stride=1104, sym_len_all=1100)
    torch.cuda.synchronize()
    assert np.array_equal(rep.cpu().numpy()[:, :, :1100], oe[:, k:, :1100])


@pytest.mark.parametrize("matrix", ["cauchy", "vandermonde"])
@pytest.mark.parametrize("L,stride,nwin", [(1200, 1200, 1000), (1200, 1264, 301), (496, 496, 777), (4096, 4096, 40),
                                           (4112, 4112, 9), (16, 16, 2000)])
def test_bitslice_gathered_stores_vs_oracle(ctx, ctx_tables, matrix, L, stride, nwin):
    """k 16 r 4 on uniform windows (gf_encode_bs_gs_kernel):
    many steps of whole windows, a last step with fewer windows, strides above
    the row length, rows up to 256 units (4096 B: one window per step) and just
    past it (4112 B: the flat kernel); bytes equal the oracle's and the table
    kernel's."""
    k, r = 16, 4
    S = np.full(nwin, L, np.uint32)
    wins = O.make_windows(0, SEED + L, 0, nwin, k, r, L, stride)
    oe = wins.copy()
    O.encode_batch(O.GF256 if matrix == "cauchy" else O.GF256_VDM, k, r, S, oe, 4)
    code = fecgpu.Code("gf256", k, r, matrix=matrix)
    for c, what in ((ctx, "gathered-store encode"), (ctx_tables, "table encode")):
        d = torch.from_numpy(wins.copy()).cuda()
        c.encode_batch(code, d, nwin=nwin, stride=stride, sym_len_all=L)
        torch.cuda.synchronize()
        _cmp_emitted(d.cpu().numpy(), oe, S, what)


# ---- FECGPU_MATRIX_RLC: RFC 8681 random linear code rows (tests/test_rlc_spec.py pins the
# generator on CPU).  Not MDS: status is the rank of the present repairs on the missing
# columns, which the plan finds by Gauss-Jordan with pivot search over every present repair.
RLC_CASES = [
    # k, r, key, dt, workload, L, erasure, nwin
    (16, 4, 0, 15, 0, 1200, 1, 64),
    (8, 2, 77, 15, 0, 1200, 2, 200),
    (32, 8, 4660, 15, 1, 0, 2, 12),     # mixed MTU, LENPREFIX, i.i.d. erasures
    (10, 6, 4660, 7, 0, 33, 2, 300),
    (6, 6, 65535, 1, 0, 20, 2, 400),    # sparse: many singular windows
    (12, 8, 9, 0, 0, 48, 2, 300),       # density 1/16
    (56, 8, 65530, 3, 0, 64, 2, 40),    # repair keys wrap at 2^16
    (1, 1, 5, 15, 0, 1, 1, 5),
]


@pytest.mark.parametrize("k,r,key,dt,wl,L,era,nwin", RLC_CASES)
def test_rlc_encode_decode_vs_oracle(ctx, k, r, key, dt, wl, L, era, nwin):
    S = O.sym_lens(wl, SEED, 0, nwin, k, L)
    stride = O.round_up(int(S.max()), 16) + (16 if wl == 0 else 0)
    wins = O.make_windows(wl, SEED, 0, nwin, k, r, L, stride)
    osc = O.RLC(key, dt)
    present = O.presents(era, SEED, 0, nwin, osc, k, r)
    ge, gd, gs = gpu_run(ctx, "gf256", k, r, wins, S, present, uniform=(wl == 0), matrix="rlc",
                         rlc=(key, dt))
    oe, od, os_ = oracle_run("gf256", k, r, wins, S, present, oscheme=osc)
    _cmp_emitted(ge, oe, S, "encode")
    assert np.array_equal(gs, os_), np.argwhere(gs != os_)[:5].tolist()
    _cmp_emitted(gd, od, S, "decode")
    for w in range(nwin):
        if gs[w] == 0:
            s = int(S[w])
            assert np.array_equal(gd[w, :k, :s], wins[w, :k, :s])


@pytest.mark.parametrize("k,r,key,dt", [(4, 4, 3, 2), (5, 3, 77, 0), (4, 3, 9, 15), (3, 5, 1, 5)])
def test_rlc_every_erasure_pattern(ctx, k, r, key, dt):
    """All 2^(k+r) present masks: GPU status (pivoting plan over every present repair)
    and bytes equal the oracle's (greedy independent repairs); recovered == original."""
    n = k + r
    nwin = 1 << n
    L = 40
    wins = O.make_windows(0, SEED, 11, 1, k, r, L, 48)
    wins = np.repeat(wins, nwin, axis=0)
    S = np.full(nwin, L, np.uint32)
    present = np.arange(nwin, dtype=np.uint64)
    osc = O.RLC(key, dt)
    ge, gd, gs = gpu_run(ctx, "gf256", k, r, wins, S, present, uniform=True, matrix="rlc", rlc=(key, dt))
    oe, od, os_ = oracle_run("gf256", k, r, wins, S, present, oscheme=osc)
    _cmp_emitted(ge, oe, S, "encode")
    assert np.array_equal(gs, os_)
    _cmp_emitted(gd, od, S, "decode")
    ok = gs == 0
    assert np.array_equal(gd[ok, :k, :L], wins[ok, :k, :L])
