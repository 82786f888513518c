"""Per-connection encoder/decoder objects (the Connection's per-packet API) on the GPU.

test_loopsim_* is the BASELINE.json config-1 stand-in: a 10 MB
stream in 1200-B packets through the XOR k=4 r=1 sender, a seeded lossy channel
and the receiver; every packet of every recoverable window must come back
byte-identical.  (The reference runs this over quiche client<->server on
loopback; Rust quiche is not available here.)
"""
import os

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


def _stream(nbytes, seed):
    return N.payload(seed, 0, 0, nbytes).tobytes() if nbytes < 1 << 16 else b"".join(
        N.payload(seed, i, 1, min(1 << 16, nbytes - (i << 16))).tobytes()
        for i in range((nbytes + (1 << 16) - 1) >> 16))


def _wire_source(w, i, p, framed):
    """Sender side: the packet as it goes on the wire (SOURCE_ID frame + payload)."""
    return fecgpu.frame_source_id(w, i) + p if framed else (w, i, p)


def _recv_source(wire, framed):
    if not framed:
        return wire
    n, f = fecgpu.frame_parse(wire)
    assert f["type"] == fecgpu.FRAME_SOURCE_ID
    return f["win"], f["idx"], wire[n:]


def _run(ctx, code, data, mtu, loss, seed, batch=256, vary=False, framed=False, m=fecgpu):
    """m: the fecgpu module (a copy bound to another library build may be passed)."""
    rng = np.random.default_rng(seed)
    pkts, pos = [], 0
    while pos < len(data):
        n = mtu if not vary else int(rng.integers(1, mtu + 1))
        pkts.append(data[pos:pos + n])
        pos += n
    enc = m.Encoder(ctx, code, max_len=mtu, batch=batch)
    dec = m.Decoder(ctx, code, max_len=mtu, batch=batch)
    ids = []
    lost_src = rng.random(len(pkts)) < loss
    for p, lost in zip(pkts, lost_src):
        w, i = enc.add_source(p)
        ids.append((w, i))
        wire = _wire_source(w, i, p, framed)
        if not lost:
            rw, ri, rp = _recv_source(wire, framed)
            assert dec.add_source(rw, ri, rp) == 0
    last = enc.close_window() if len(pkts) % code.k else ids[-1][0]
    enc.flush()
    nwin = ids[-1][0] + 1
    assert last == nwin - 1
    rep_lost = rng.random((nwin, code.r)) < loss
    for w in range(nwin):
        nsrc = enc.window_sources(w)  # < k for the short last window
        for i in range(code.r):
            rep = enc.repair(w, i)
            assert rep is not None
            if framed:  # REPAIR frame on the wire, parsed by the receiver
                _, f = fecgpu.frame_parse(fecgpu.frame_repair(w, code.k, code.r, i, rep, nsrc=nsrc))
                assert (f["win"], f["idx"], f["k"], f["r"], f["nsrc"]) == (w, i, code.k, code.r, nsrc)
                rep, nsrc = f["payload"], f["nsrc"]
            if not rep_lost[w, i]:
                # the short last window's padding sources are not losses (REPAIR nsrc)
                if nsrc < code.k:
                    assert dec.set_window_sources(w, nsrc) == 0
                assert dec.add_repair(w, i, rep) == 0
    dec.flush()
    got, missing = [], 0
    for (w, i), p in zip(ids, pkts):
        q = dec.recovered(w, i)
        if q is None:
            missing += 1
        else:
            assert q == p, (w, i)
        got.append(q)
    # expected losses after recovery, from the masks alone
    exp_missing = 0
    for w in range(nwin):
        idx = [t for t, (ww, _) in enumerate(ids) if ww == w]
        rl = list(rep_lost[w])
        # padding counts as received once a REPAIR frame told the receiver nsrc;
        # with every repair lost nothing of the window can be recovered anyway
        lost = [bool(lost_src[t]) for t in idx] + [not any(not x for x in rl)] * (code.k - len(idx))
        if code.scheme == "xor":
            for g in range(code.r):
                mem = [j for j in range(len(idx)) if j % code.r == g]
                nl = sum(lost[j] for j in mem)
                if nl == 1 and not rl[g]:
                    continue
                exp_missing += nl
        else:
            nl = sum(lost[:len(idx)])
            if sum(lost) > code.r - sum(rl):
                exp_missing += nl
    assert missing == exp_missing
    return len(pkts), missing


def test_loopsim_xor_k4r1_10MB(ctx):
    data = _stream(10 * 1024 * 1024, 11)
    code = fecgpu.Code("xor", 4, 1, "lenprefix")
    n, missing = _run(ctx, code, data, 1200, 0.02, 3, framed=True)
    assert n == (len(data) + 1199) // 1200
    assert missing < n * 0.01


def test_conn_gf_variable_lengths(ctx):
    data = _stream(2 * 1024 * 1024, 12)
    code = fecgpu.Code("gf256", 16, 4, "lenprefix")
    n, missing = _run(ctx, code, data, 1350, 0.08, 5, batch=32, vary=True)
    assert missing < n * 0.05


def test_conn_fixed_framing(ctx):
    data = _stream(600 * 1000, 13)
    code = fecgpu.Code("gf256", 8, 3, "fixed")
    _run(ctx, code, data, 1000, 0.1, 7, batch=8)


def test_conn_errors(ctx):
    code = fecgpu.Code("gf256", 4, 2, "fixed")
    enc = fecgpu.Encoder(ctx, code, max_len=100, batch=4)
    with pytest.raises(fecgpu.FecError):
        enc.add_source(b"x" * 101)              # > max_len
    enc.add_source(b"a" * 50)
    with pytest.raises(fecgpu.FecError):
        enc.add_source(b"b" * 49)               # FIXED: lengths must match in a window
    assert enc.repair(0, 0) is None             # not encoded yet
    dec = fecgpu.Decoder(ctx, code, max_len=100, batch=4)
    assert dec.add_source(0, 5, b"z" * 10) == fecgpu.ERR_INVALID_ARG  # idx >= k
    assert dec.recovered(0, 1) is None


CONN_BENCH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts", "conn_bench")


@pytest.mark.parametrize("args", [
    ["xor", "8", "2", "1200", "48", "0.05", "64"],
    ["xor", "4", "1", "1000", "16", "0.03", "16", "0", "64", "0.02"],       # reordered + duplicates
    ["gf256", "16", "4", "1200", "48", "0.08", "128", "1", "33", "0.01"],   # LENPREFIX, reordered
    ["gf256", "32", "8", "9000", "64", "0.12", "16", "1"],                   # mixed lengths, deep loss
    ["gf256", "5", "3", "333", "4", "0.2", "3", "0", "7", "0.05"],           # FIXED, short last window
], ids=["xor-k8r2", "xor-k4r1-reorder-dup", "gf-k16r4-lp-reorder", "gf-k32r8-lp", "gf-k5r3-fixed"])
def test_native_conn_driver(args):
    """scripts/conn_bench (C++, per packet through the C ABI): encoder buffers recycle,
    decoder slots are reused, symbols may arrive reordered and duplicated; every
    delivered packet is byte-identical and exactly the packets the loss pattern
    allows are recovered (exit 3 otherwise)."""
    import json
    import subprocess
    assert os.path.exists(CONN_BENCH), "build first: make -C scripts"
    r = subprocess.run([CONN_BENCH, *args], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["corrupt"] == 0 and res["unrecovered"] == res["expected_unrecovered"]
    assert res["recovered"] + res["unrecovered"] == res["lost"]


UDP_RING = os.path.join(os.path.dirname(CONN_BENCH), "udp_ring")


@pytest.mark.parametrize("args", [
    ["xor", "8", "2", "1200", "200000", "0.03", "256"],
    ["gf256", "16", "4", "1200", "100003", "0.08", "128"],   # short last window
    ["xor", "4", "1", "1000", "10485", "0.02", "16"],        # config-1 shape: 10 MB, XOR k4 r1
], ids=["xor-k8r2", "gf-k16r4-short-last", "xor-k4r1-10MB"])
def test_udp_ring_driver(args):
    """scripts/udp_ring (C++): real UDP loopback sockets -> recvmmsg straight into pinned
    window rows -> GPU encode -> SOURCE_ID / REPAIR frames sent as gather sends from
    the rows -> seeded loss -> recvmmsg -> decoder -> in-order delivery.  Every packet is
    delivered byte-identical or is one the loss pattern cannot recover (exit 3 otherwise)."""
    import json
    import subprocess
    assert os.path.exists(UDP_RING), "build first: make -C scripts"
    r = subprocess.run([UDP_RING, *args], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["corrupt"] == 0 and res["unrecovered"] == res["expected_unrecovered"]
    assert res["delivered"] + res["unrecovered"] == res["packets"]
    assert res["recovered"] + res["unrecovered"] == res["lost"]


@pytest.mark.parametrize("args", [
    ["conn_bench_asan", "gf256", "32", "8", "9000", "16", "0.12", "16", "1"],
    ["conn_bench_asan", "xor", "4", "1", "1000", "8", "0.03", "16", "0", "64", "0.02"],
    ["conn_bench_asan", "gf256", "5", "3", "333", "2", "0.2", "3", "0", "7", "0.05"],
    ["udp_ring_asan", "gf256", "16", "4", "1200", "50003", "0.08", "128"],
    ["many_conn_asan", "gf256", "16", "4", "1200", "60", "5", "0.1", "3"],
    ["many_conn_asan", "xor", "8", "2", "700", "60", "5", "0.05", "2"],
    ["sw_conn_bench_asan", "1202", "32", "8", "6", "0.05", "16"],
    ["sw_conn_bench_asan", "302", "16", "4", "3", "0.1", "4", "128"],
], ids=["conn-gf-k32r8-lp", "conn-xor-reorder-dup", "conn-gf-short-last", "udp-gf-k16r4",
        "many-gf-k16r4", "many-xor-k8r2", "sw-conn-W32", "sw-conn-W16-small-span"])
def test_native_drivers_under_asan(args):
    """The per-connection objects, pools, frames and pinned rings under host
    AddressSanitizer + UBSan (lib/asan/libfecgpu.so: host code instrumented, kernels
    the release ones; GPU ASan is not available on this pool).  Any report aborts."""
    import subprocess
    exe = os.path.join(os.path.dirname(CONN_BENCH), args[0])
    assert os.path.exists(exe), "build first: make -C scripts"
    env = dict(os.environ,
               # quarantine off: ROCm's ASan runtime otherwise recycles one of its device
               # allocator's chunks in the HSA runtime's exit-time finalizer and trips a CHECK
               ASAN_OPTIONS="detect_leaks=0:verify_asan_link_order=0:halt_on_error=1:quarantine_size_mb=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe, *args[1:]], capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]


@pytest.mark.parametrize("nstreams", [4, 1])
def test_many_connections_share_streams(nstreams):
    """A server's worth of connections on one ctx: 400 encoder / decoder pairs (800
    objects) launch on the ctx's pool of `nstreams` streams, interleaved window by
    window; every lost packet comes back from its own connection's decoder."""
    c = fecgpu.Context()
    c.set_tuning("conn_streams", nstreams)
    code = fecgpu.Code("gf256", 4, 2)
    n = 400
    encs = [fecgpu.Encoder(c, code, max_len=64, batch=1) for _ in range(n)]
    decs = [fecgpu.Decoder(c, code, max_len=64, batch=1) for _ in range(n)]
    pk = [[bytes([(i * 7 + j * 13 + t) & 0xFF for t in range(64)]) for j in range(4)] for i in range(n)]
    ids = [[encs[i].add_source(p) for p in pk[i]] for i in range(n)]  # batch=1: launches per window
    for i in range(n):
        w = ids[i][0][0]
        for j in (0, 3):  # sources 1 and 2 lost
            assert decs[i].add_source(w, j, pk[i][j]) == 0
        for t in range(2):
            assert decs[i].add_repair(w, t, encs[i].repair(w, t)) == 0
    for i in range(n):
        decs[i].flush()
        w = ids[i][0][0]
        assert decs[i].recovered(w, 1) == pk[i][1] and decs[i].recovered(w, 2) == pk[i][2], i
    for o in encs + decs:
        o.close()
    c.close()


def test_connection_churn_reuses_pinned_blocks():
    """300 short-lived connections one after another (open, one window each way,
    close): every lost packet is recovered, and with the ctx's pinned-block cache the
    churn costs less than pinning and unpinning fresh memory per connection."""
    import time
    code = fecgpu.Code("gf256", 16, 4)
    pk = [bytes([(j * 31 + t) & 0xFF for t in range(1200)]) for j in range(16)]
    times = {}
    for cache_mb in (1024, 0):
        c = fecgpu.Context()
        c.set_tuning("pinned_cache_mb", cache_mb)
        t0 = time.perf_counter()
        for i in range(300):
            enc = fecgpu.Encoder(c, code, max_len=1200, batch=8)
            dec = fecgpu.Decoder(c, code, max_len=1200, batch=8)
            ids = [enc.add_source(p) for p in pk]
            enc.flush()
            w = ids[0][0]
            for j in range(4, 16):
                assert dec.add_source(w, j, pk[j]) == 0
            for t in range(4):
                assert dec.add_repair(w, t, enc.repair(w, t)) == 0
            dec.flush()
            assert all(dec.recovered(w, j) == pk[j] for j in range(4)), i
            enc.close()
            dec.close()
        times[cache_mb] = time.perf_counter() - t0
        c.close()
    # timings are reported, not asserted (profiles/ holds the measurements)
    print(f"300 connections: {times[1024]:.3f} s with the pinned cache, {times[0]:.3f} s without")


@pytest.mark.parametrize("scheme,framing", [("gf256", "fixed"), ("xor", "fixed"), ("gf256", "lenprefix")])
def test_flush_many_one_launch_for_all_connections(scheme, framing):
    """fecgpu_decoder_flush_many: 200 connections' decoders flushed by one launch
    recover exactly what 200 separate flushes recover, faster."""
    import time
    c = fecgpu.Context()
    k, r, n = 8, 2, 200
    code = fecgpu.Code(scheme, k, r, framing)
    rng = np.random.default_rng(5)

    def setup():
        encs = [fecgpu.Encoder(c, code, max_len=1200, batch=4) for _ in range(n)]
        decs = [fecgpu.Decoder(c, code, max_len=1200, batch=64) for _ in range(n)]
        sent = []
        for i in range(n):
            pk = [rng.integers(0, 256, 1200 if framing == "fixed" else int(rng.integers(1, 1201)),
                               dtype=np.uint8).tobytes() for _ in range(2 * k)]
            ids = [encs[i].add_source(p) for p in pk]
            encs[i].flush()
            lost = {0, 3} if scheme == "gf256" else {0, 1}  # XOR: one per group
            for (w, j), p in zip(ids, pk):
                if j not in lost:
                    assert decs[i].add_source(w, j, p) == 0
            for w in {w for w, _ in ids}:
                for t in range(r):
                    assert decs[i].add_repair(w, t, encs[i].repair(w, t)) == 0
            sent.append((ids, pk, lost))
        return encs, decs, sent

    def check(decs, sent):
        for d, (ids, pk, lost) in zip(decs, sent):
            for (w, j), p in zip(ids, pk):
                assert d.recovered(w, j) == p

    encs, decs, sent = setup()
    t0 = time.perf_counter()
    got_many = fecgpu.decoder_flush_many(decs)
    t_many = time.perf_counter() - t0
    check(decs, sent)
    encs2, decs2, sent2 = setup()
    t0 = time.perf_counter()
    got_each = sum(d.flush() for d in decs2)
    t_each = time.perf_counter() - t0
    check(decs2, sent2)
    assert got_many == got_each == n * 2 * 2
    print(f"{scheme}/{framing}: 200 decoders, one launch {t_many * 1e3:.2f} ms, "
          f"200 launches {t_each * 1e3:.2f} ms")  # reported, not asserted
    with pytest.raises(fecgpu.FecError):  # listed twice
        fecgpu.decoder_flush_many([decs[0], decs[0]])
    other = fecgpu.Decoder(c, fecgpu.Code(scheme, k, r, framing), max_len=600, batch=4)
    with pytest.raises(fecgpu.FecError):  # different max_len
        fecgpu.decoder_flush_many([decs[0], other])
    for o in encs + decs + encs2 + decs2 + [other]:
        o.close()
    c.close()


@pytest.mark.parametrize("scheme,framing", [("gf256", "lenprefix"), ("xor", "fixed")])
def test_encoder_flush_many(scheme, framing):
    """fecgpu_encoder_flush_many: 200 senders' queued windows encoded by one launch
    give the repairs that 200 separate flushes give, faster."""
    import time
    c = fecgpu.Context()
    k, r, n = 8, 2, 200
    code = fecgpu.Code(scheme, k, r, framing)
    rng = np.random.default_rng(9)
    pkts = [[rng.integers(0, 256, 1200 if framing == "fixed" else int(rng.integers(1, 1201)),
                          dtype=np.uint8).tobytes() for _ in range(2 * k)] for _ in range(n)]
    res, t = [], []
    warm = fecgpu.Encoder(c, code, max_len=1200, batch=64)  # the argument block's first pinning
    warm.add_source(pkts[0][0])
    fecgpu.encoder_flush_many([warm])
    warm.close()
    for many in (True, False):
        encs = [fecgpu.Encoder(c, code, max_len=1200, batch=64) for _ in range(n)]
        ids = [[e.add_source(p) for p in pk] for e, pk in zip(encs, pkts)]
        t0 = time.perf_counter()
        if many:
            assert fecgpu.encoder_flush_many(encs) == n * 2
        else:
            assert sum(e.flush() for e in encs) == n * 2
        t.append(time.perf_counter() - t0)
        res.append([[e.repair(w, i) for w in sorted({w for w, _ in ids_e}) for i in range(r)]
                    for e, ids_e in zip(encs, ids)])
        for e in encs:
            e.close()
    assert res[0] == res[1]
    assert all(rep is not None for reps in res[0] for rep in reps)
    print(f"{scheme}/{framing}: 200 encoders, one launch {t[0] * 1e3:.2f} ms, "
          f"200 launches {t[1] * 1e3:.2f} ms")  # reported, not asserted
    c.close()


@pytest.mark.parametrize("args", [["gf256", "16", "4", "1200", "300", "4", "0.1", "3"],
                                  ["xor", "8", "2", "1200", "300", "4", "0.05", "2"],
                                  ["gf256", "32", "8", "9000", "40", "2", "0.12", "2"]],
                         ids=["gf-k16r4", "xor-k8r2", "gf-k32r8-9000"])
def test_native_many_connections(args):
    """scripts/many_conn (C++): hundreds of connections per ctx, senders and receivers
    flushed with the *_flush_many calls, connections closed and reopened each round;
    every lost packet recovered exactly as the loss pattern allows."""
    import json
    import subprocess
    exe = os.path.join(os.path.dirname(CONN_BENCH), "many_conn")
    assert os.path.exists(exe), "build first: make -C scripts"
    r = subprocess.run([exe, *args], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["corrupt"] == 0 and res["unrecovered"] == res["expected_unrecovered"]
    assert res["recovered"] + res["unrecovered"] == res["lost"] > 0


def test_policy_timeouts(ctx):
    """Scheduling policy: on the caller's clock, a window closes
    window_timeout_us after its first packet and a partly filled batch launches
    batch_timeout_us after its first window closed; the receiver flushes
    batch_timeout_us after the first symbol filed since its last flush."""
    code = fecgpu.Code("gf256", 8, 2, "lenprefix")
    enc = fecgpu.Encoder(ctx, code, max_len=1200, batch=64)
    enc.set_policy(window_timeout_us=100, batch_timeout_us=50)
    assert enc.tick(1000) == 0
    pkts = [bytes([i]) * (100 + i) for i in range(3)]
    for p in pkts:
        assert enc.add_source(p)[0] == 0
    assert enc.tick(1099) == 0 and enc.repair(0, 0) is None     # window still open
    assert enc.tick(1100) == 0 and enc.repair(0, 0) is None     # closed, batch not due
    assert enc.tick(1149) == 0
    assert enc.tick(1150) == 1                                   # batch launched
    rep = [enc.repair(0, i) for i in range(2)]
    assert all(r is not None and len(r) == 2 + 102 for r in rep)
    w, i = enc.add_source(b"x" * 10)                             # next window opens at 1150
    assert (w, i) == (1, 0)
    dec = fecgpu.Decoder(ctx, code, max_len=1200, batch=64)
    dec.set_policy(batch_timeout_us=30)
    assert dec.tick(5000) == 0
    assert dec.add_source(0, 1, pkts[1]) == 0
    assert enc.window_sources(0) == 3                            # REPAIR nsrc: 3..7 are padding
    assert dec.set_window_sources(0, 3) == 0
    assert dec.add_repair(0, 0, rep[0]) == 0 and dec.add_repair(0, 1, rep[1]) == 0
    assert dec.tick(5029) == 0 and dec.recovered(0, 0) is None   # flush not due yet
    assert dec.tick(5030) == 2                                   # flushed: sources 0 and 2 back
    assert dec.recovered(0, 0) == pkts[0] and dec.recovered(0, 2) == pkts[2]


def test_async_auto_flush(ctx):
    """The automatic flush (every batch*k filed symbols) launches without waiting:
    a window in flight completes when it is next touched; the window whose symbol
    triggered the flush stays open and is decoded by the next flush."""
    code = fecgpu.Code("xor", 4, 1, "fixed")
    enc = fecgpu.Encoder(ctx, code, max_len=64, batch=2)
    pkts = [bytes([7 * n + 1]) * 64 for n in range(8)]
    for p in pkts:
        enc.add_source(p)
    enc.flush()
    reps = [enc.repair(w, 0) for w in range(2)]
    dec = fecgpu.Decoder(ctx, code, max_len=64, batch=2)     # auto flush every 8 symbols
    for w in range(2):
        for i in range(3):                                  # source 3 of each window is lost
            assert dec.add_source(w, i, pkts[4 * w + i]) == 0
        assert dec.add_repair(w, 0, reps[w]) == 0           # 8th symbol: window 0 launched
    assert dec.recovered(0, 3) == pkts[3]                   # completes the in-flight decode
    assert dec.recovered(1, 3) is None                      # the triggering window waits
    assert dec.add_source(1, 0, pkts[4]) == fecgpu.ERR_DONE  # duplicate, still detected
    assert dec.flush() == 2                                 # window 0 (completed above) + window 1
    assert dec.recovered(1, 3) == pkts[7]
    # a window in flight released before completion, and flush counting pending results
    for w in range(2, 4):
        for i in (0, 2, 3):
            assert dec.add_source(w, i, pkts[i]) == 0
        assert dec.add_repair(w, 0, reps[0]) == 0           # window 2 launched at the 8th
    assert dec.release(2) == 0                              # completes window 2's decode first
    assert dec.flush() == 2                                 # windows 2 and 3
    assert dec.recovered(3, 1) == pkts[1]
    assert dec.drain_recovered() == [(0, 3), (1, 3), (3, 1)]  # released window 2 skipped
