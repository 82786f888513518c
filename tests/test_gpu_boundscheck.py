"""Bounds-checked debug build (GPU AddressSanitizer is not available
on this pool, so lib/libfecgpu_check.so, built with FECGPU_CHECK=1, checks every
symbol load / store of every batch kernel against the byte ranges of the launch's
windows and fails the call with FECGPU_ERR_DEVICE when one falls outside).

The layouts and codes of the parity suite run on that build: their outputs equal
the oracle's AND no kernel touched a byte outside its windows.  check_shrink
takes bytes off the end of the checked ranges, so the checker is seen to fire.
"""
import importlib.util
import os
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import fecgpu  # noqa: E402
import oracle as O  # noqa: E402

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "quic-fec-eps_amd")
CHECK_LIB = os.path.join(PKG, "lib", "libfecgpu_check.so")
SEED = 97531


def _load_check_module():
    """A second copy of the fecgpu package bound to the bounds-checked library."""
    assert os.path.exists(CHECK_LIB), "build first: make -C quic-fec-eps_amd"
    os.environ["FECGPU_LIB"] = CHECK_LIB
    try:
        spec = importlib.util.spec_from_file_location("fecgpu_check", os.path.join(PKG, "fecgpu", "__init__.py"))
        mod = importlib.util.module_from_spec(spec)
        sys.modules[spec.name] = mod
        spec.loader.exec_module(mod)
    finally:
        del os.environ["FECGPU_LIB"]
    assert mod.LIB_PATH == CHECK_LIB
    return mod


@pytest.fixture(scope="module")
def chk():
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    O.build()
    m = _load_check_module()
    c = m.Context()
    yield m, c
    c.close()


def _scheme(s):
    return O.XOR if s == "xor" else O.GF256


def _oracle(scheme, k, r, wins, S, present, poison=0xAB):
    enc = wins.copy()
    O.encode_batch(_scheme(scheme), k, r, S, enc, 4)
    dec = enc.copy()
    O.erase(dec, present, k, r, fill=poison)
    st = O.decode_batch(_scheme(scheme), k, r, S, dec, present, 4)
    return enc, dec, st


def _emitted_equal(a, b, S):
    return all(np.array_equal(a[w, :, :int(S[w])], b[w, :, :int(S[w])]) for w in range(a.shape[0]))


CASES = [
    # scheme, k, r, workload, L, erasure, nwin: flat and group modes, per-window S,
    # tiny and large symbols, r > k, the bit-sliced codes (k 16 r 4 at 1200 B: the
    # gathered-store kernel, 64 windows = 10 steps of 6 and one of 4)
    ("xor", 8, 2, 0, 1200, 1, 64),
    ("xor", 5, 3, 0, 17, 2, 64),
    ("xor", 8, 2, 1, 0, 2, 12),
    ("gf256", 16, 4, 0, 1200, 1, 64),
    ("gf256", 32, 8, 1, 0, 2, 12),
    ("gf256", 32, 8, 0, 1200, 2, 40),
    ("gf256", 16, 8, 0, 16, 1, 33),
    ("gf256", 1, 1, 0, 1, 1, 5),
    ("gf256", 56, 8, 0, 64, 1, 9),
    ("gf256", 3, 5, 0, 16, 1, 8),
]


@pytest.mark.parametrize("scheme,k,r,wl,L,era,nwin", CASES)
def test_checked_encode_decode_vs_oracle(chk, scheme, k, r, wl, L, era, nwin):
    """Windows in a tensor of exactly nwin x (k + r) x stride bytes: every access of
    encode and decode stays inside (else the call raises) and the bytes equal the oracle."""
    m, ctx = chk
    S = O.sym_lens(wl, SEED, 0, nwin, k, L)
    stride = O.round_up(int(S.max()), 16)
    wins = O.make_windows(wl, SEED, 0, nwin, k, r, L, stride)
    present = O.presents(era, SEED, 0, nwin, _scheme(scheme), k, r)
    oe, od, os_ = _oracle(scheme, k, r, wins, S, present)
    code = m.Code(scheme, k, r)
    d = torch.from_numpy(wins.copy()).cuda()
    kw = dict(sym_len_all=int(S[0])) if wl == 0 else dict(sym_len=torch.from_numpy(S.astype(np.int32)).cuda())
    ctx.encode_batch(code, d, nwin=nwin, stride=stride, **kw)
    torch.cuda.synchronize()
    enc = d.cpu().numpy()
    assert _emitted_equal(enc, oe, S)
    mask = torch.from_numpy(np.array([[(int(p) >> i) & 1 for i in range(k + r)] for p in present], bool)).cuda()
    d[~mask] = 0xAB
    st = torch.full((nwin,), 7, dtype=torch.uint8, device="cuda")
    ctx.decode_batch(code, d, torch.from_numpy(present.astype(np.int64)).cuda(), st, nwin=nwin,
                     stride=stride, **kw)
    torch.cuda.synchronize()
    assert np.array_equal(st.cpu().numpy(), os_)
    assert _emitted_equal(d.cpu().numpy(), od, S)


@pytest.mark.parametrize("pitch", [0, 320])
def test_checked_ragged_layout(chk, pitch):
    """win_off windows, packed (pitch 0: stride round_up(S_w, 16)) or fixed pitch,
    at scattered offsets with gaps: the checked range is derived from win_off."""
    m, ctx = chk
    k, r, nwin = 6, 3, 17
    rng = np.random.default_rng(11)
    S = rng.integers(1, 300, nwin).astype(np.uint32)
    strides = [pitch or O.round_up(int(s), 16) for s in S]
    offs, pos = [], 0
    for w in range(nwin):
        pos += 16 * int(rng.integers(0, 4))
        offs.append(pos)
        pos += (k + r) * strides[w]
    for scheme in ("gf256", "xor"):
        buf = np.zeros(pos, np.uint8)
        for w in range(nwin):
            win = np.zeros((k + r, strides[w]), np.uint8)
            win[:k, :S[w]] = rng.integers(0, 256, (k, int(S[w])), dtype=np.uint8)
            buf[offs[w]:offs[w] + win.size] = win.ravel()
        present = O.presents(1, SEED, 0, nwin, _scheme(scheme), k, r)
        d = torch.from_numpy(buf).cuda()
        off_t = torch.tensor(offs, dtype=torch.int64).cuda()
        sl = torch.from_numpy(S.astype(np.int32)).cuda()
        code = m.Code(scheme, k, r)
        ctx.encode_batch(code, d, nwin=nwin, stride=pitch, sym_len=sl, win_off=off_t)
        enc = d.cpu().numpy()
        for w in range(nwin):
            for i in range(k + r):
                if not (int(present[w]) >> i) & 1:
                    a = offs[w] + i * strides[w]
                    d[a:a + strides[w]] = 0xCD
        st = torch.zeros(nwin, dtype=torch.uint8, device="cuda")
        ctx.decode_batch(code, d, torch.from_numpy(present.astype(np.int64)).cuda(), st,
                         nwin=nwin, stride=pitch, sym_len=sl, win_off=off_t)
        out = d.cpu().numpy()
        assert int(st.sum().item()) == 0
        for w in range(nwin):
            o = np.frombuffer(enc[offs[w]:offs[w] + (k + r) * strides[w]].tobytes(), np.uint8)
            o = o.reshape(k + r, strides[w]).copy()
            ref = o.copy()
            O.encode_batch(_scheme(scheme), k, r, np.array([S[w]], np.uint32), ref[None], 1)
            assert np.array_equal(o[:, :S[w]], ref[:, :S[w]]), (scheme, w)
            rec = out[offs[w]:offs[w] + o.size].reshape(o.shape)
            assert np.array_equal(rec[:k, :S[w]], ref[:k, :S[w]]), (scheme, w)


@pytest.mark.parametrize("scheme,k,r,wl,L", [("xor", 8, 2, 0, 1200), ("gf256", 16, 4, 0, 1200),
                                              ("gf256", 32, 8, 1, 0), ("gf256", 4, 7, 0, 100)])
def test_checked_encode_split(chk, scheme, k, r, wl, L):
    """Split layout: sources read only inside src, repairs written only inside repair."""
    m, ctx = chk
    nwin = 37
    S = O.sym_lens(wl, SEED, 0, nwin, k, L)
    stride = O.round_up(int(S.max()), 16)
    wins = O.make_windows(wl, SEED, 0, nwin, k, r, L, stride)
    oe, _, _ = _oracle(scheme, k, r, wins, S, np.full(nwin, (1 << (k + r)) - 1, np.uint64))
    src = torch.from_numpy(np.ascontiguousarray(wins[:, :k])).cuda()
    rep = torch.full((nwin, r, stride), 0x77, dtype=torch.uint8, device="cuda")
    kw = dict(sym_len_all=int(S[0])) if wl == 0 else dict(sym_len=torch.from_numpy(S.astype(np.int32)).cuda())
    ctx.encode_split(m.Code(scheme, k, r), src, rep, nwin=nwin, stride=stride, **kw)
    torch.cuda.synchronize()
    got = np.concatenate([src.cpu().numpy(), rep.cpu().numpy()], axis=1)
    assert np.array_equal(got[:, :k], wins[:, :k])
    assert _emitted_equal(got, oe, S)


@pytest.mark.parametrize("direct", [0, 6, 7])
def test_checked_host_pipeline(chk, direct):
    """Pinned host windows through the chunked pipeline (staging slots reused, outputs
    stored into the mapped host windows for direct != 0): each launch's range is its
    chunk."""
    m, ctx = chk
    k, r, nwin = 32, 8, 120
    S = O.sym_lens(1, SEED, 0, nwin, k, 0)
    stride = O.round_up(int(S.max()), 16)
    wins = O.make_windows(1, SEED, 0, nwin, k, r, 0, stride)
    present = O.presents(2, SEED, 0, nwin, O.GF256, k, r)
    oe, od, os_ = _oracle("gf256", k, r, wins, S, present)
    buf = m.PinnedBuffer(wins.nbytes)
    h = buf.array.reshape(wins.shape)
    h[:] = wins
    ctx.set_tuning("host_direct", direct)
    ctx.set_tuning("host_chunk_mb", 1)
    try:
        code = m.Code("gf256", k, r)
        ctx.encode_batch(code, h, nwin=nwin, stride=stride, sym_len=S, flags=m.F_HOST_PTRS)
        enc = h.copy()
        O.erase(h, present, k, r, fill=0xAB)
        st = np.full(nwin, 9, np.uint8)
        ctx.decode_batch(code, h, present, st, nwin=nwin, stride=stride, sym_len=S, flags=m.F_HOST_PTRS)
        dec = h.copy()
    finally:
        ctx.set_tuning("host_direct", 6)
        ctx.set_tuning("host_chunk_mb", 128)
        del h
        buf.close()
    assert _emitted_equal(enc, oe, S)
    assert np.array_equal(st, os_)
    assert _emitted_equal(dec, od, S)


@pytest.mark.parametrize("scheme,k,r,L", [("xor", 8, 2, 1200), ("gf256", 16, 4, 1200), ("gf256", 32, 8, 1200)])
def test_checker_fires_when_the_range_is_short(chk, scheme, k, r, L):
    """check_shrink=16 hides the last 16-byte column of the batch from the checker:
    the kernel's (correct) access to it must be reported as a fault."""
    m, ctx = chk
    nwin = 8
    wins = O.make_windows(0, SEED, 0, nwin, k, r, L, L)
    d = torch.from_numpy(wins).cuda()
    code = m.Code(scheme, k, r)
    ctx.set_tuning("check_shrink", 16)
    try:
        with pytest.raises(m.FecError, match="bounds check"):
            ctx.encode_batch(code, d, nwin=nwin, stride=L, sym_len_all=L)
    finally:
        ctx.set_tuning("check_shrink", 0)
    ctx.encode_batch(code, d, nwin=nwin, stride=L, sym_len_all=L)  # and clean again


@pytest.mark.parametrize("scheme,k,r,framing,mtu,loss,batch,vary", [
    ("xor", 4, 1, "lenprefix", 1200, 0.03, 16, False),
    ("gf256", 16, 4, "lenprefix", 1350, 0.08, 32, True),
    ("gf256", 8, 3, "fixed", 1000, 0.1, 8, False),
])
def test_checked_per_connection(chk, scheme, k, r, framing, mtu, loss, batch, vary):
    """Per-connection encoder / decoder on the checked build: their launches run on
    windows in mapped pinned memory (remote plan, ragged fixed-pitch decode of
    pooled slots with offsets that wrap below the base)."""
    from test_gpu_conn import _run, _stream
    m, ctx = chk
    data = _stream(600 * 1000, 21)
    _run(ctx, m.Code(scheme, k, r, framing), data, mtu, loss, 9, batch=batch, vary=vary, m=m)


def test_checked_flush_many(chk):
    """fecgpu_decoder_flush_many on the checked build: one launch over windows of 20
    decoders' separate pinned pools (offsets from one base, wrapping)."""
    m, _ = chk
    c = m.Context()
    code = m.Code("gf256", 8, 2, "lenprefix")
    rng = np.random.default_rng(3)
    encs = [m.Encoder(c, code, max_len=700, batch=2) for _ in range(20)]
    decs = [m.Decoder(c, code, max_len=700, batch=64) for _ in range(20)]
    sent = []
    for e, d in zip(encs, decs):
        pk = [rng.integers(0, 256, int(rng.integers(1, 701)), dtype=np.uint8).tobytes() for _ in range(24)]
        ids = [e.add_source(p) for p in pk]
        e.flush()
        for (w, j), p in zip(ids, pk):
            if j not in (2, 5):
                assert d.add_source(w, j, p) == 0
        for w in {w for w, _ in ids}:
            for t in range(2):
                assert d.add_repair(w, t, e.repair(w, t)) == 0
        sent.append((ids, pk))
    assert m.decoder_flush_many(decs) == 20 * 3 * 2
    e2 = [m.Encoder(c, code, max_len=700, batch=64) for _ in range(20)]  # queued, not launched
    for e, (ids, pk) in zip(e2, sent):
        for p in pk:
            e.add_source(p)
    assert m.encoder_flush_many(e2) == 20 * 3
    for e, ee, (ids, pk) in zip(e2, encs, sent):
        for w in {w for w, _ in ids}:
            assert [e.repair(w, t) for t in range(2)] == [ee.repair(w, t) for t in range(2)]
        e.close()
    for d, (ids, pk) in zip(decs, sent):
        assert all(d.recovered(w, j) == p for (w, j), p in zip(ids, pk))
    for o in encs + decs:
        o.close()
    c.close()


def test_release_build_has_no_checker():
    ctx = fecgpu.Context()
    try:
        with pytest.raises(fecgpu.FecError) as e:
            ctx.set_tuning("check_shrink", 16)
        assert e.value.code == fecgpu.ERR_UNSUPPORTED
    finally:
        ctx.close()


def test_checked_encoder_failed_launch_recovers(chk):
    """when the launch of a full batch fails, the encoder must not file
    the next source past the end of that batch.  check_shrink makes the launch fail
    (bounds check); add_source retries it and keeps failing without writing out of
    bounds; once the checker is relaxed the same batch launches and every repair
    matches the oracle."""
    import np_oracle as N
    m, ctx = chk
    code = m.Code("gf256", 4, 2, "fixed")
    pk = [bytes([(13 * n + t) & 0xFF for t in range(256)]) for n in range(16)]
    enc = m.Encoder(ctx, code, max_len=256, batch=2)
    for p in pk[:4]:
        enc.add_source(p)                           # window 0 closed, batch not full
    ctx.set_tuning("check_shrink", 16)
    try:
        for p in pk[4:7]:
            enc.add_source(p)
        with pytest.raises(m.FecError, match="bounds check"):
            enc.add_source(pk[7])                   # closes window 1: the launch fails
        for _ in range(3):                          # retried, never filed past the batch
            with pytest.raises(m.FecError, match="bounds check"):
                enc.add_source(pk[8])
        assert enc.repair(0, 0) is None             # not encoded
    finally:
        ctx.set_tuning("check_shrink", 0)
    assert enc.add_source(pk[8]) == (2, 0)          # launches batch 0, starts window 2
    for p in pk[9:12]:
        enc.add_source(p)
    enc.flush()
    for w in range(3):
        ref = N.encode("gf", 4, 2, np.frombuffer(b"".join(pk[4 * w:4 * w + 4]), np.uint8).reshape(4, 256))
        assert [enc.repair(w, i) for i in range(2)] == [ref[i].tobytes() for i in range(2)], w
    enc.close()


# ---- sliding-window and wide kernels ----
# The checked build also bounds the sliding-window kernels (fec_swdec.hip,
# fec_swenc.hip: every row, job slot, look-back record, start-list entry and
# operation-log entry an index addresses, against its allocation), the combine
# launches (their rows against the call's arrays) and the wide plan.  Each case
# below runs equal to the oracle AND clean.

def _sw():
    import test_gpu_sw as T
    return T


def test_checked_sw_decode_config7_scale(chk):
    """Config 7's stream shape at full length (524,288 sources: the plan's 256
    look-back chunks), short symbols; encode and decode on the checked build."""
    T = _sw()
    m, ctx = chk
    nsrc, L, k, W = 524288, 32, 8, 32
    stride = O.round_up(L, 16)
    src = T.stream(nsrc, L, stride, 7)
    hdr = T.hdr_array(T.N.sw_schedule(nsrc, k, W, key0=1, dt=15))
    rep = T.gpu_encode(ctx, src, hdr, L, max_window=W)
    assert np.array_equal(rep[:, :L], O.sw_encode(src, hdr, L)[:, :L])
    rng = np.random.default_rng(7)
    sp = (rng.random(nsrc) >= 0.02).astype(np.uint8)
    rp = (rng.random(len(hdr)) >= 0.02).astype(np.uint8)
    T.check_vs_oracle(ctx, src, sp, rep, rp, hdr, L)


@pytest.mark.parametrize("loss", [0.10, 0.30])
def test_checked_sw_two_repairs_per_step_W255(chk, loss):
    """W 255, two repairs per step: long systems, row-slot compaction, chained logs."""
    T = _sw()
    m, ctx = chk
    nsrc, L, W = 2500, 24, 255
    stride = O.round_up(L, 16)
    src = T.stream(nsrc, L, stride, 255 + int(loss * 100))
    hdr = T.two_per_step(nsrc, W, key0=int(loss * 1000))
    rep = O.sw_encode(src, hdr, L)
    rng = np.random.default_rng(int(loss * 1000) + 1)
    sp = (rng.random(nsrc) >= loss).astype(np.uint8)
    rp = (rng.random(len(hdr)) >= loss).astype(np.uint8)
    assert T.max_system(sp, rp, hdr) > 100
    T.check_vs_oracle(ctx, src, sp, rep, rp, hdr, L)


def test_checked_sw_compaction_with_small_log(chk):
    """sw_log_entries 16: every long system overflows its log chunk and the
    synchronous retries grow it; equal to the oracle, no access outside the log."""
    T = _sw()
    m, _ = chk
    c = m.Context()
    try:
        c.set_tuning("sw_log_entries", 16)
        nsrc, L, W = 1500, 16, 255
        stride = O.round_up(L, 16)
        src = T.stream(nsrc, L, stride, 77)
        hdr = T.two_per_step(nsrc, W, key0=77)
        rep = O.sw_encode(src, hdr, L)
        rng = np.random.default_rng(77)
        sp = (rng.random(nsrc) >= 0.2).astype(np.uint8)
        rp = (rng.random(len(hdr)) >= 0.2).astype(np.uint8)
        T.check_vs_oracle(c, src, sp, rep, rp, hdr, L)
    finally:
        c.close()


def test_checked_sw_checker_fires_when_the_range_is_short(chk):
    """check_shrink=16 hides the last 16 bytes of each of a decode's arrays from
    the combine launches' checker: a syndrome job reading the last source row
    (a source lost near the end) must be reported."""
    T = _sw()
    m, ctx = chk
    nsrc, L, k, W = 400, 64, 4, 16
    stride = O.round_up(L, 16)
    src = T.stream(nsrc, L, stride, 3)
    hdr = T.hdr_array(T.N.sw_schedule(nsrc, k, W, key0=3, dt=15))
    rep = O.sw_encode(src, hdr, L)
    sp = np.ones(nsrc, np.uint8)
    sp[nsrc - 2] = 0
    rp = np.ones(len(hdr), np.uint8)
    ctx.set_tuning("check_shrink", 16)
    try:
        with pytest.raises(m.FecError, match="bounds check"):
            T.gpu_decode(ctx, src, sp, rep, rp, hdr, L)
    finally:
        ctx.set_tuning("check_shrink", 0)
    T.check_vs_oracle(ctx, src, sp, rep, rp, hdr, L)  # and clean again


@pytest.mark.parametrize("k,r,matrix,L", [(248, 8, "cauchy", 300), (120, 8, "rlc", 1200), (150, 5, "cauchy", 64)])
def test_checked_wide_encode_decode(chk, k, r, matrix, L):
    """k + r up to 256: the runtime-mask encode and the two-stage decode."""
    import test_gpu_wide as TW
    m, _ = chk
    c = m.Context()
    try:
        rng = np.random.default_rng(k + r)
        bits = TW._erasures(10, k, r, rng)
        TW._run(c, k, r, matrix, L, 10, bits, m=m)
    finally:
        c.close()


def test_checked_wide_two_stage(chk):
    """The wide two-stage combine decode (bitslice off) on the checked build."""
    import test_gpu_wide as TW
    m, _ = chk
    c = m.Context()
    try:
        c.set_tuning("bitslice", 0)
        bits = TW._erasures(10, 200, 6, np.random.default_rng(5))
        TW._run(c, 200, 6, "cauchy", 500, 10, bits, m=m)
    finally:
        c.close()


@pytest.mark.parametrize("matrix", ["cauchy", "vandermonde"])
def test_checked_gf_decode_many_erasures(chk, matrix):
    """Windows with many erasures (k 32 r 8), mixed lengths, on the checked build."""
    import test_gpu_gfdec_many as TB
    m, _ = chk
    c = m.Context()
    try:
        rng = np.random.default_rng(11)
        bits = TB._erasures(40, 32, 8, rng, lo=4)
        sl = np.where(rng.random(40) < 0.5, 1202, 9002).astype(np.uint32)
        TB._run(c, 32, 8, matrix, 9002, 40, bits, sym_len=sl, m=m)
    finally:
        c.close()
