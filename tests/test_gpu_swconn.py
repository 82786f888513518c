"""Per-connection sliding-window objects (fecgpu_sw_encoder_* / fecgpu_sw_decoder_*) and
their frames on the GPU, against the oracle.

Sender: every repair the encoder emits (header with absolute FSS, E bytes) equals
orc_sw_encode over the A.3-framed stream, framed independently here
(LENPREFIX: u16be len || payload || zeros to E; FIXED: payload = symbol), across
buffer compactions.  Receiver: through SW_SOURCE / SW_REPAIR frames only, over a
lossy channel, the final status of every source equals the oracle's global
decode (orc_sw_decode) of the same losses, and every packet returned equals
the original.  PARITY UNPINNED vs the fec branch (its FEC frames are not
mounted; the coefficients follow RFC 8681/8682, pinned in tests/test_rlc_spec.py).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
import fecgpu  # noqa: E402
import oracle as O  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    assert torch.cuda.is_available()
    O.build()
    c = fecgpu.Context()
    yield c
    c.close()


def frame(pkts, E, framing):
    out = np.zeros((len(pkts), O.round_up(E, 16)), np.uint8)
    for i, p in enumerate(pkts):
        a = np.frombuffer(p, np.uint8)
        if framing == "lenprefix":
            out[i, 0], out[i, 1] = len(p) >> 8, len(p) & 0xFF
            out[i, 2:2 + len(p)] = a
        else:
            out[i, :len(p)] = a
    return out


def packets(rng, n, E, framing):
    if framing == "fixed":
        return [rng.integers(0, 256, E, dtype=np.uint8).tobytes() for _ in range(n)]
    lens = rng.integers(0, E - 1, n)
    lens[rng.random(n) < 0.05] = 0
    return [rng.integers(0, 256, int(x), dtype=np.uint8).tobytes() for x in lens]


def hdr_array(h):
    a = np.zeros(len(h), O.SW_REPAIR_DTYPE)
    for t, (fss, nss, key, dt) in enumerate(h):
        a[t]["fss"], a[t]["nss"], a[t]["key"], a[t]["dt"] = fss, nss, key, dt
    return a


CASES = [  # E, W, step, framing, dt, batch, n
    (1202, 32, 8, "lenprefix", 15, 16, 700),
    (100, 16, 4, "fixed", 15, 8, 900),       # several buffer compactions (cap 4 x (16 + 32))
    (48, 10, 3, "lenprefix", 5, 1, 200),
    (9002, 8, 2, "lenprefix", 15, 4, 60),
]


@pytest.mark.parametrize("E,W,step,framing,dt,batch,n", CASES)
def test_sw_encoder_repairs_match_oracle(ctx, E, W, step, framing, dt, batch, n):
    rng = np.random.default_rng(E + W)
    pk = packets(rng, n, E, framing)
    enc = fecgpu.SwEncoder(ctx, fecgpu.sw_params(E, W, step, framing=framing, dt=dt, batch=batch))
    reps = []
    for i, p in enumerate(pk):
        try:
            esi = enc.add_source(p)
        except fecgpu.FecError as ex:   # every launch slot holds unread repairs:
            assert ex.code == fecgpu.ERR_LIMIT   # wait for them, read, retry
            enc.flush()
            while (r := enc.next_repair()) is not None:
                reps.append(r)
            esi = enc.add_source(p)
        assert esi == i
        while (r := enc.next_repair()) is not None:
            reps.append(r)
    enc.flush()
    while (r := enc.next_repair()) is not None:
        reps.append(r)
    assert len(reps) == n // step
    hdr = [h for h, _ in reps]
    for t, (fss, nss, key, d) in enumerate(hdr):
        end = (t + 1) * step
        assert (fss, nss, key, d) == (max(0, end - W), end - max(0, end - W), t & 0xFFFF, dt)
    src = frame(pk, E, framing)
    ref = O.sw_encode(src, hdr_array(hdr), E)
    for t, (_, sym) in enumerate(reps):
        assert sym == ref[t, :E].tobytes(), t
    enc.close()


def test_sw_encoder_limit_until_repairs_are_read(ctx):
    enc = fecgpu.SwEncoder(ctx, fecgpu.sw_params(64, 8, 2, batch=2))
    with pytest.raises(fecgpu.FecError) as ei:
        for _ in range(100):
            enc.add_source(b"x" * 10)
    assert ei.value.code == fecgpu.ERR_LIMIT
    enc.flush()
    got = 0
    while enc.next_repair() is not None:
        got += 1
    assert got == 8          # four slots of two repairs
    enc.add_source(b"y")     # room again
    enc.close()


def test_sw_encoder_survives_failed_launches(ctx):
    """a failed launch must not let the scheduled list grow
    past `batch` (it would overrun the slot's rows).  Launches fail by fault
    injection; the source that scheduled the failed batch is kept, the next
    scheduling call retries the batch first and fails with nothing consumed, and
    once launches work again every repair equals the oracle's."""
    E, W, step, batch, n = 64, 8, 2, 4, 120
    rng = np.random.default_rng(3)
    pk = packets(rng, n, E, "fixed")
    enc = fecgpu.SwEncoder(ctx, fecgpu.sw_params(E, W, step, framing="fixed", batch=batch))
    reps, i, failed = [], 0, 0
    ctx.set_tuning("fault_launches", 5)
    while i < n:
        try:
            assert enc.add_source(pk[i]) == i
            i += 1
        except fecgpu.FecError as e:  # the retried batch failed: nothing consumed
            assert e.code == fecgpu.ERR_DEVICE
            failed += 1
        while (r := enc.next_repair()) is not None:
            reps.append(r)
    enc.flush()
    while (r := enc.next_repair()) is not None:
        reps.append(r)
    assert failed == 4  # the first failure is the consuming call's own launch (not reported)
    assert len(reps) == n // step
    hdr = [h for h, _ in reps]
    assert [h[2] for h in hdr] == list(range(n // step))
    ref = O.sw_encode(frame(pk, E, "fixed"), hdr_array(hdr), E)
    enc.close()
    for t, (_, sym) in enumerate(reps):
        assert sym == ref[t, :E].tobytes(), t


def test_sw_decoder_rejects_overlong_window_before_advancing(ctx):
    """a SW_REPAIR whose nss exceeds the session's window is
    INVALID_ARG and leaves the buffered sources alone."""
    E, W = 32, 8
    dec = fecgpu.SwDecoder(ctx, fecgpu.sw_params(E, W, 2, framing="fixed", span=64))
    for esi in range(10):
        assert dec.add_source(esi, bytes([esi]) * E) == 0
    with pytest.raises(fecgpu.FecError) as ei:
        dec.add_repair((10_000, W + 1, 0, 15), b"z" * E)
    assert ei.value.code == fecgpu.ERR_INVALID_ARG
    assert all(dec.recovered(esi) == bytes([esi]) * E for esi in range(10))
    dec.close()


@pytest.mark.parametrize("E,W,step,framing,dt,batch,n", CASES[:3])
@pytest.mark.parametrize("loss", [0.05, 0.15])
def test_sw_frames_only_receiver_matches_oracle(ctx, E, W, step, framing, dt, batch, n, loss):
    rng = np.random.default_rng(E * 3 + W + int(loss * 100))
    pk = packets(rng, n, E, framing)
    params = fecgpu.sw_params(E, W, step, framing=framing, dt=dt, batch=batch, span=n)
    enc = fecgpu.SwEncoder(ctx, params)
    wire, reps = [], []
    for p in pk:
        esi = enc.add_source(p)
        wire.append(fecgpu.frame_sw_source(esi) + p)
        while (r := enc.next_repair()) is not None:
            reps.append(r)
            wire.append(fecgpu.frame_sw_repair(*r))
    enc.flush()
    while (r := enc.next_repair()) is not None:
        reps.append(r)
        wire.append(fecgpu.frame_sw_repair(*r))
    lost = rng.random(len(wire)) < loss
    dec = fecgpu.SwDecoder(ctx, params)
    sp = np.zeros(n, np.uint8)
    rp = []
    for b, gone in zip(wire, lost):
        m, f = fecgpu.frame_parse(b)
        if f["type"] == fecgpu.FRAME_SW_SOURCE:
            if not gone:
                sp[f["esi"]] = 1
                assert dec.add_source(f["esi"], b[m:]) == 0
        else:
            rp.append(0 if gone else 1)
            if not gone:
                assert dec.add_repair(f["hdr"], f["payload"]) == 0
    dec.flush()
    # oracle: global decode of the same losses
    hdr = hdr_array([h for h, _ in reps])
    src = frame(pk, E, framing)
    rep = np.zeros((len(reps), src.shape[1]), np.uint8)
    for t, (_, sym) in enumerate(reps):
        rep[t, :E] = np.frombuffer(sym, np.uint8)
    od = src.copy()
    od[sp == 0] = 0
    ost, on = O.sw_decode(od, sp, rep, np.array(rp, np.uint8), hdr, E)
    got = dec.drain_recovered()
    assert sorted(got) == [i for i in range(n) if sp[i] == 0 and ost[i] == 0]
    for i, p in enumerate(pk):
        q = dec.recovered(i)
        if sp[i] or ost[i] == 0:
            assert q == p, i
        else:
            assert q is None, i
    dec.close()
    enc.close()


def test_sw_long_stream_small_span(ctx):
    """20,000 packets through a receiver that keeps 256 sources: everything it
    returns is the original, and most losses come back."""
    E, W, step, n = 300, 24, 6, 20000
    rng = np.random.default_rng(9)
    pk = packets(rng, n, E, "lenprefix")
    params = fecgpu.sw_params(E, W, step, batch=32, span=256)
    enc = fecgpu.SwEncoder(ctx, params)
    dec = fecgpu.SwDecoder(ctx, params)
    lost_src = rng.random(n) < 0.03
    nrec = 0
    for i, p in enumerate(pk):
        assert enc.add_source(p) == i
        if not lost_src[i]:
            dec.add_source(i, p)
        while (r := enc.next_repair()) is not None:
            if rng.random() >= 0.03:
                dec.add_repair(*r)
    enc.flush()
    while (r := enc.next_repair()) is not None:
        dec.add_repair(*r)
    dec.flush()
    for esi in dec.drain_recovered():
        assert lost_src[esi] and dec.recovered(esi) in (None, pk[esi])
        nrec += 1
    for i in range(n - 200, n):
        q = dec.recovered(i)
        assert q is None or q == pk[i]
    assert nrec > 0.8 * lost_src.sum()
    enc.close()
    dec.close()
