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
