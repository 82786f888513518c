"""Sliding-window RLC (RFC 8681, fecgpu_sw_*) oracles on CPU: the C oracle
(oracle/fec_oracle.c orc_sw_*: identity-augmented Gauss-Jordan) against the
independent numpy restatement (oracle/np_oracle.py sw_*: elimination of the
data rows themselves), on streams with i.i.d. and burst losses.  The
coefficient generator underneath is pinned by RFC 8682's TinyMT32 vectors
(tests/test_rlc_spec.py); stream framing and schedules are build decisions
(parity unpinned vs the fec branch)."""
import numpy as np
import pytest

import oracle as O
import np_oracle as N


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


@pytest.mark.parametrize("nsrc,k,W,dt,L", [(64, 4, 16, 15, 24), (120, 8, 32, 15, 40), (90, 3, 12, 6, 17),
                                           (40, 2, 9, 1, 8)])
def test_sw_encode_c_vs_numpy(nsrc, k, W, dt, L):
    stride = O.round_up(L, 16)
    src = stream(nsrc, L, stride, nsrc)
    h = N.sw_schedule(nsrc, k, W, key0=100, dt=dt)
    rep = O.sw_encode(src, hdr_array(h), L)
    assert np.array_equal(rep[:, :L], N.sw_encode(src[:, :L], h))
    assert not rep[:, L:].any()


LOSS = [("iid", 0.05), ("iid", 0.15), ("iid", 0.3), ("burst", 6), ("burst", 20)]


@pytest.mark.parametrize("loss", LOSS, ids=[f"{a}{b}" for a, b in LOSS])
@pytest.mark.parametrize("k,W,dt", [(4, 16, 15), (8, 32, 15), (4, 12, 3)])
def test_sw_decode_c_vs_numpy(loss, k, W, dt):
    nsrc, L = 160, 20
    stride = O.round_up(L, 16)
    src = stream(nsrc, L, stride, k * W)
    h = N.sw_schedule(nsrc, k, W, key0=7, dt=dt)
    hdr = hdr_array(h)
    rep = O.sw_encode(src, hdr, L)
    rng = np.random.default_rng(W + k)
    if loss[0] == "iid":
        sp = (rng.random(nsrc) >= loss[1]).astype(np.uint8)
        rp = (rng.random(len(h)) >= loss[1]).astype(np.uint8)
    else:
        sp = np.ones(nsrc, np.uint8)
        b = int(rng.integers(0, nsrc - loss[1]))
        sp[b:b + loss[1]] = 0
        rp = np.ones(len(h), np.uint8)
    d = src.copy()
    d[sp == 0] = 0xAB
    st, nrec = O.sw_decode(d, sp, rep, rp, hdr, L)
    ns, nst = N.sw_decode(np.where(sp[:, None] == 1, src[:, :L], 0xAB).astype(np.uint8), sp, rep[:, :L], rp, h)
    assert np.array_equal(st, nst)
    assert nrec == int(((sp == 0) & (st == 0)).sum())
    assert np.array_equal(d[st == 0, :L], src[st == 0, :L])   # recovered == original
    assert np.array_equal(ns[st == 0], src[st == 0, :L])


def _random_case(seed):
    """A random stream, schedule, density and loss pattern (i.i.d., plus a
    burst every fifth case): small enough for the dense oracle."""
    rng = np.random.default_rng(seed)
    nsrc = int(rng.integers(20, 400))
    k = int(rng.integers(1, 9))
    W = int(rng.integers(k, min(255, nsrc) + 1))
    dt = int(rng.choice([15, 15, 7, 3, 0]))
    L = int(rng.integers(1, 40))
    stride = O.round_up(L, 16)
    src = np.zeros((nsrc, stride), np.uint8)
    src[:, :L] = rng.integers(0, 256, (nsrc, L), dtype=np.uint8)
    h = N.sw_schedule(nsrc, k, W, key0=int(rng.integers(0, 60000)), dt=dt)
    loss = float(rng.choice([0.02, 0.1, 0.2, 0.35, 0.5]))
    sp = (rng.random(nsrc) >= loss).astype(np.uint8)
    rp = (rng.random(len(h)) >= loss).astype(np.uint8)
    if seed % 5 == 0:
        b = int(rng.integers(0, nsrc))
        sp[b:b + int(rng.integers(1, 60))] = 0
    return src, h, sp, rp, L


@pytest.mark.parametrize("block", range(4))
def test_sw_decode_banded_equals_dense(block):
    """The banded decode (oracle/fec_sw_banded.c, the GPU long-system
    algorithm) against the dense identity-augmented Gauss-Jordan: equal
    statuses, counts and bytes on 200 random streams (rank-deficient systems
    at low DT and heavy loss included)."""
    for seed in range(block * 50, block * 50 + 50):
        src, h, sp, rp, L = _random_case(seed)
        hdr = hdr_array(h)
        rep = O.sw_encode(src, hdr, L)
        d1 = src.copy()
        d1[sp == 0] = 0xAB
        d2 = d1.copy()
        s1, n1 = O.sw_decode(d1, sp, rep, rp, hdr, L)
        s2, n2 = O.sw_decode_banded(d2, sp, rep, rp, hdr, L)
        assert np.array_equal(s1, s2) and n1 == n2, seed
        assert np.array_equal(d2[s2 == 0, :L], src[s2 == 0, :L]), seed


@pytest.mark.parametrize("W,k,loss,nsrc", [(255, 8, 0.10, 5000), (64, 4, 0.15, 6000), (32, 8, 0.12, 8000)])
def test_sw_decode_banded_long_systems(W, k, loss, nsrc):
    """Streams whose linked systems hold hundreds of unknowns (W 255 at 10 %
    is one system): banded == dense on every status and byte."""
    L, stride = 24, 32
    rng = np.random.default_rng(W * k)
    src = np.zeros((nsrc, stride), np.uint8)
    src[:, :L] = rng.integers(0, 256, (nsrc, L), dtype=np.uint8)
    h = N.sw_schedule(nsrc, k, W, key0=11, dt=15)
    hdr = hdr_array(h)
    rep = O.sw_encode(src, hdr, L)
    sp = (rng.random(nsrc) >= loss).astype(np.uint8)
    rp = (rng.random(len(h)) >= loss).astype(np.uint8)
    d1 = src.copy()
    d1[sp == 0] = 0
    d2 = d1.copy()
    s1, n1 = O.sw_decode(d1, sp, rep, rp, hdr, L)
    s2, n2 = O.sw_decode_banded(d2, sp, rep, rp, hdr, L)
    assert n1 >= 0 and np.array_equal(s1, s2) and n1 == n2
    assert np.array_equal(d2[s2 == 0, :L], src[s2 == 0, :L])
