"""Per-connection wire parity: the repair bytes the sender puts
on the wire, checked against the oracle.

The per-connection objects are the drop-in API (include/fecgpu.h "per-packet
API"): a Connection adds each protected payload with fecgpu_encoder_add_source
and sends fecgpu_encoder_repair's bytes in a REPAIR frame.  Here every repair
of every window is compared byte for byte with np_oracle.encode applied to the
window's Appendix A.3 symbols, framed independently in this file:
  FIXED      symbol = packet (every packet of a window has length L), S = L;
  LENPREFIX  symbol = u16be(len) || payload || zeros, S = 2 + the window's
             longest packet;
  a window closed early (close_window / window timeout) is padded with empty
  (LENPREFIX) or zero (FIXED) sources, and its REPAIR frames carry nsrc.
The same windows then go through frames only — SOURCE_ID + payload and REPAIR
frames, fecgpu_frame_parse, no out-of-band hints — into the decoder, whose
recovered packets are compared with np_oracle.decode of the same framed window.
PARITY UNPINNED against the fec branch (its framing is not mounted,
/root/reference/README.md:7): the oracle restates SURVEY Appendix A.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
import fecgpu  # noqa: E402
import np_oracle as N  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    assert torch.cuda.is_available()
    c = fecgpu.Context()
    yield c
    c.close()


def _oscheme(code):
    if code.scheme == "xor":
        return "xor"
    if code.matrix == "rlc":
        return f"rlc:{code.rlc_key}:{code.rlc_dt}"
    return "gf-vdm" if code.matrix == "vandermonde" else "gf"


def _code(scheme, k, r, framing, matrix):
    """matrix 'rlc:KEY:DT' -> the RFC 8681 RLC rows of repair_key KEY.., density DT."""
    if matrix.startswith("rlc:"):
        _, key, dt = matrix.split(":")
        return fecgpu.Code(scheme, k, r, framing, "rlc", rlc_key=int(key), rlc_dt=int(dt))
    return fecgpu.Code(scheme, k, r, framing, matrix)


def frame_window(code, pkts):
    """Appendix A.3 symbols of one window (real packets first, padding after)."""
    k = code.k
    lp = code.framing == "lenprefix"
    if lp:
        S = 2 + max(len(p) for p in pkts)
    else:
        S = max(1, len(pkts[0]))
    syms = np.zeros((k, S), np.uint8)
    for j, p in enumerate(pkts):
        a = np.frombuffer(p, np.uint8)
        if lp:
            syms[j, 0], syms[j, 1] = len(p) >> 8, len(p) & 0xFF
            syms[j, 2:2 + len(p)] = a
        else:
            syms[j, :len(p)] = a
    return syms, S


def _packets(rng, code, nwin, mtu, short_last):
    """Per-window packet lists; FIXED windows share one length per window."""
    wins = []
    for w in range(nwin):
        n = code.k if (w < nwin - 1 or not short_last) else short_last
        if code.framing == "fixed":
            L = int(rng.integers(1, mtu + 1))
            wins.append([rng.integers(0, 256, L, dtype=np.uint8).tobytes() for _ in range(n)])
        else:
            lens = rng.integers(0, mtu + 1, n)
            lens[rng.random(n) < 0.1] = 0  # empty packets are legal under LENPREFIX
            wins.append([rng.integers(0, 256, int(x), dtype=np.uint8).tobytes() for x in lens])
    return wins


CASES = [
    # (scheme, k, r, framing, matrix, mtu, nwin, short_last, batch)
    ("gf256", 8, 3, "fixed", "cauchy", 1000, 12, 3, 4),
    ("gf256", 16, 4, "lenprefix", "cauchy", 1350, 9, 5, 4),
    ("gf256", 32, 8, "lenprefix", "cauchy", 9000, 5, 2, 2),
    ("gf256", 10, 4, "lenprefix", "vandermonde", 1200, 7, 9, 3),
    ("gf256", 16, 8, "fixed", "vandermonde", 1200, 6, 1, 8),
    ("xor", 4, 1, "lenprefix", "cauchy", 1200, 15, 2, 4),
    ("xor", 8, 2, "fixed", "cauchy", 1200, 10, 5, 16),
    ("xor", 6, 3, "lenprefix", "cauchy", 700, 8, 4, 3),
    ("gf256", 16, 4, "lenprefix", "rlc:0:15", 1350, 9, 5, 4),
    ("gf256", 8, 4, "fixed", "rlc:4660:5", 1000, 12, 3, 4),
]


@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}-k{c[1]}r{c[2]}-{c[3]}-{c[4]}" for c in CASES])
def test_encoder_repairs_match_oracle(ctx, case):
    scheme, k, r, framing, matrix, mtu, nwin, short_last, batch = case
    code = _code(scheme, k, r, framing, matrix)
    rng = np.random.default_rng(k * 100 + r)
    wins = _packets(rng, code, nwin, mtu, short_last)
    enc = fecgpu.Encoder(ctx, code, max_len=mtu, batch=batch)
    for w, pk in enumerate(wins):
        for j, p in enumerate(pk):
            assert enc.add_source(p) == (w, j)
    assert enc.close_window() == nwin - 1  # the short last window
    enc.flush()
    for w, pk in enumerate(wins):
        syms, S = frame_window(code, pk)
        ref = N.encode(_oscheme(code), k, r, syms)
        assert enc.window_sources(w) == len(pk)
        for i in range(r):
            rep = enc.repair(w, i)
            assert rep is not None and len(rep) == S, (w, i)
            assert rep == ref[i].tobytes(), (w, i)
            # the wire payload: REPAIR frame written and parsed back
            n, f = fecgpu.frame_parse(fecgpu.frame_repair(w, k, r, i, rep, nsrc=len(pk)))
            assert (f["win"], f["idx"], f["k"], f["r"], f["nsrc"]) == (w, i, k, r, len(pk))
            assert f["payload"] == ref[i].tobytes()
    enc.close()


@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}-k{c[1]}r{c[2]}-{c[3]}-{c[4]}" for c in CASES])
def test_frames_only_receiver_matches_oracle(ctx, case):
    """Sender -> frames on the wire -> lossy channel -> frame_parse -> decoder.
    The receiver learns nothing out of band: short windows through REPAIR nsrc."""
    scheme, k, r, framing, matrix, mtu, nwin, short_last, batch = case
    code = _code(scheme, k, r, framing, matrix)
    rng = np.random.default_rng(7 * k + r)
    wins = _packets(rng, code, nwin, mtu, short_last)
    enc = fecgpu.Encoder(ctx, code, max_len=mtu, batch=batch)
    wire = []
    for w, pk in enumerate(wins):
        for p in pk:
            ww, j = enc.add_source(p)
            wire.append(fecgpu.frame_source_id(ww, j) + p)
    enc.close_window()
    enc.flush()
    for w, pk in enumerate(wins):
        for i in range(r):
            wire.append(fecgpu.frame_repair(w, k, r, i, enc.repair(w, i), nsrc=enc.window_sources(w)))
    lost = rng.random(len(wire)) < 0.15
    dec = fecgpu.Decoder(ctx, code, max_len=mtu, batch=batch)
    for b, gone in zip(wire, lost):
        if gone:
            continue
        n, f = fecgpu.frame_parse(b)
        if f["type"] == fecgpu.FRAME_SOURCE_ID:
            assert dec.add_source(f["win"], f["idx"], b[n:]) == 0
        else:
            if f["nsrc"] < k:
                assert dec.set_window_sources(f["win"], f["nsrc"]) == 0
            assert dec.add_repair(f["win"], f["idx"], f["payload"]) == 0
    dec.flush()
    # the oracle on the same framed windows and the same loss pattern
    t = 0
    nrec = 0
    for w, pk in enumerate(wins):
        syms, S = frame_window(code, pk)
        ref = N.encode(_oscheme(code), k, r, syms)
        full = np.concatenate([syms, ref])
        pres = 0
        for j in range(len(pk)):
            pres |= (not lost[t + j]) << j
        for j in range(len(pk), k):  # padding: known from nsrc (if any repair arrived)
            pres |= 1 << j
        t += len(pk)
        got_rep = False
        for i in range(r):
            if not lost[len(wire) - nwin * r + w * r + i]:
                pres |= 1 << (k + i)
                got_rep = True
        if not got_rep:  # no REPAIR frame arrived: the receiver cannot know nsrc
            for j in range(len(pk), k):
                pres &= ~(1 << j)
        out, ok_all = N.decode(_oscheme(code), k, r, full, pres)
        for j, p in enumerate(pk):
            q = dec.recovered(w, j)
            if (pres >> j) & 1:
                assert q == p
                continue
            # lost: the oracle recovers it iff the decoder does, with the same bytes
            oracle_ok = ok_all if code.matrix == "rlc" else _recoverable(code, pres, j)
            if oracle_ok:
                exp = bytes(N.deframe(out[j])) if framing == "lenprefix" else out[j][:len(p)].tobytes()
                assert exp == p
                assert q == exp, (w, j)
                nrec += 1
            else:
                assert q is None, (w, j)
        for j in range(len(pk), k):
            assert dec.recovered(w, j) is None  # padding is never a packet
    got = dec.drain_recovered()
    assert len(got) == nrec
    dec.close()
    enc.close()


def _recoverable(code, pres, j):
    k, r = code.k, code.r
    miss = [x for x in range(k) if not (pres >> x) & 1]
    if code.scheme == "xor":
        g = j % r
        mg = [x for x in miss if x % r == g]
        return len(mg) == 1 and bool((pres >> (k + g)) & 1)
    nrep = sum((pres >> (k + i)) & 1 for i in range(r))
    return len(miss) <= nrep


@pytest.mark.parametrize("framing", ["lenprefix", "fixed"])
def test_timeout_window_through_frames_only(ctx, framing):
    """a window closed by the window timeout holds 3 of k = 16 packets;
    its 13 padding slots exceed r = 4.  Through frames alone (REPAIR nsrc = 3), a lost
    packet of that window is recovered; a FIXED receiver gets no zero 'packets'."""
    code = fecgpu.Code("gf256", 16, 4, framing)
    enc = fecgpu.Encoder(ctx, code, max_len=1200, batch=8)
    enc.set_policy(window_timeout_us=100, batch_timeout_us=10)
    enc.tick(0)
    pk = [bytes([(31 * i + 7 * j) & 0xFF for j in range(1000 if framing == "fixed" else 300 + 200 * i)])
          for i in range(3)]
    wire = []
    for p in pk:
        w, j = enc.add_source(p)
        wire.append(fecgpu.frame_source_id(w, j) + p)
    assert enc.tick(100) == 0      # window closed by the timeout, batch not due
    assert enc.tick(110) == 1      # batch launched
    assert enc.window_sources(0) == 3
    syms, S = frame_window(code, pk)
    ref = N.encode("gf", 16, 4, syms)
    for i in range(4):
        rep = enc.repair(0, i)
        assert rep == ref[i].tobytes()
        wire.append(fecgpu.frame_repair(0, 16, 4, i, rep, nsrc=enc.window_sources(0)))
    dec = fecgpu.Decoder(ctx, code, max_len=1200, batch=8)
    for t, b in enumerate(wire):
        if t == 1:
            continue               # packet 1 lost
        n, f = fecgpu.frame_parse(b)
        if f["type"] == fecgpu.FRAME_SOURCE_ID:
            assert dec.add_source(f["win"], f["idx"], b[n:]) == 0
        else:
            assert f["nsrc"] == 3
            assert dec.set_window_sources(f["win"], f["nsrc"]) == 0
            assert dec.add_repair(f["win"], f["idx"], f["payload"]) == 0
    assert dec.flush() == 1
    assert dec.recovered(0, 1) == pk[1]
    assert all(dec.recovered(0, j) is None for j in range(3, 16))
    assert dec.drain_recovered() == [(0, 1)]
    # nsrc conflicts and sources at padding indices are rejected
    assert dec.set_window_sources(0, 4) == fecgpu.ERR_INVALID_ARG
    assert dec.add_source(0, 5, b"x" * (1000 if framing == "fixed" else 5)) == fecgpu.ERR_INVALID_ARG
    dec.close()
    enc.close()


def test_auto_flush_counts_are_not_lost(ctx):
    """recovery counts of an automatic flush completed inside another
    call (a second automatic flush, recovered(), release()) reach the next
    flush()/tick() and the recovered queue."""
    code = fecgpu.Code("xor", 4, 1, "fixed")
    enc = fecgpu.Encoder(ctx, code, max_len=64, batch=1)
    pk = [bytes([9 * n + 1]) * 64 for n in range(4 * 6)]
    for p in pk:
        enc.add_source(p)
    enc.flush()
    dec = fecgpu.Decoder(ctx, code, max_len=64, batch=1)   # automatic flush every 4 symbols
    for w in range(6):
        for i in range(3):                                  # source 3 lost in every window
            assert dec.add_source(w, i, pk[4 * w + i]) == 0
        assert dec.add_repair(w, 0, enc.repair(w, 0)) == 0
    # windows 0..4 were launched by automatic flushes, each completed by the next
    # one; window 5 triggered the last and waits for the explicit flush
    assert dec.flush() == 6
    assert dec.drain_recovered() == [(w, 3) for w in range(6)]
    assert all(dec.recovered(w, 3) == pk[4 * w + 3] for w in range(6))
    assert dec.flush() == 0 and dec.tick(10**6) == 0
    dec.close()
    enc.close()


def test_decoder_window_limit(ctx):
    """a peer spraying window ids cannot make the receiver pin memory
    without bound: past max_windows open windows a symbol returns ERR_LIMIT."""
    code = fecgpu.Code("gf256", 4, 2, "fixed")
    dec = fecgpu.Decoder(ctx, code, max_len=100, batch=4)
    dec.set_max_windows(16)
    for w in range(16):
        assert dec.add_source(1000 * w, 0, b"a" * 100) == 0
    assert dec.add_source(10**9, 0, b"a" * 100) == fecgpu.ERR_LIMIT
    assert dec.add_repair(10**9, 0, b"a" * 100) == fecgpu.ERR_LIMIT
    assert dec.set_window_sources(10**9, 2) == fecgpu.ERR_LIMIT
    assert dec.add_source(0, 1, b"b" * 100) == 0         # open windows still take symbols
    assert dec.release(0) == 0
    assert dec.add_source(10**9, 0, b"a" * 100) == 0     # room again
    dec.close()
