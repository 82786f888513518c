"""Pin the oracle's codec: C oracle vs the
independent numpy restatement, the committed golden fixtures, every erasure pattern
of small codes, framing and the workload streams.  PARITY UNPINNED vs the reference
fec branch (not mounted)."""
import glob
import os

import numpy as np
import pytest

import np_oracle as N

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def O(oracle_lib):
    return oracle_lib


def sid(O, s):
    return {"xor": O.XOR, "gf": O.GF256, "gf-vdm": O.GF256_VDM}[s]


@pytest.mark.parametrize("scheme", ["xor", "gf", "gf-vdm"])
@pytest.mark.parametrize("wl,L,k,r,era", [(0, 100, 8, 2, 1), (1, 0, 6, 3, 2), (0, 64, 16, 4, 1),
                                           (1, 0, 4, 1, 2), (0, 1, 3, 3, 1), (0, 31, 12, 5, 2)])
def test_c_oracle_matches_numpy(O, scheme, wl, L, k, r, era):
    nwin, seed = 5, 99
    S = O.sym_lens(wl, seed, 3, nwin, k, L)
    stride = O.round_up(int(S.max()), 16)
    wins = O.make_windows(wl, seed, 3, nwin, k, r, L, stride)
    O.encode_batch(sid(O, scheme), k, r, S, wins)
    pres = O.presents(era, seed, 3, nwin, sid(O, scheme), k, r)
    orig = wins.copy()
    O.erase(wins, pres, k, r, fill=0xAB)
    st = O.decode_batch(sid(O, scheme), k, r, S, wins, pres)
    for i in range(nwin):
        w = 3 + i
        pk, Sw, sym = N.window(wl, seed, w, k, L)
        assert Sw == S[i]
        assert np.array_equal(orig[i, :k, :Sw], sym)
        assert np.array_equal(orig[i, k:, :Sw], N.encode(scheme, k, r, sym))
        assert int(pres[i]) == N.present(era, seed, w, scheme, k, r)
        garbage = orig[i, :, :Sw].copy()
        for s in range(k + r):
            if not (int(pres[i]) >> s) & 1:
                garbage[s] = 0xAB
        src, ok = N.decode(scheme, k, r, garbage, int(pres[i]))
        assert ok == (st[i] == 0)
        assert np.array_equal(wins[i, :k, :Sw], src)
        if ok:
            assert np.array_equal(src, sym)


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(HERE, "golden", "*.npz"))),
                         ids=lambda p: os.path.basename(p)[:-4])
def test_c_oracle_reproduces_golden(O, path):
    z = np.load(path)
    scheme_id, k, r, L, era, nwin, w0, seed = (int(x) for x in z["meta"])
    stride = O.round_up(L, 16)
    wins = O.make_windows(0, seed, w0, nwin, k, r, L, stride)
    assert np.array_equal(wins[:, :k, :L], z["src"])
    S = np.full(nwin, L, np.uint32)
    O.encode_batch(scheme_id, k, r, S, wins)
    assert np.array_equal(wins[:, k:, :L], z["repair"])
    pres = O.presents(era, seed, w0, nwin, scheme_id, k, r)
    assert np.array_equal(pres, z["present"])
    O.erase(wins, pres, k, r, fill=0xAB)
    st = O.decode_batch(scheme_id, k, r, S, wins, pres)
    assert np.array_equal(st, z["status"])
    assert np.array_equal(wins[:, :k, :L], z["decoded"])


@pytest.mark.parametrize("scheme,k,r", [("gf", 4, 3), ("gf", 6, 2), ("xor", 6, 3), ("xor", 5, 2),
                                        ("gf", 1, 1), ("xor", 1, 1), ("gf-vdm", 4, 3),
                                        ("gf-vdm", 5, 5), ("gf-vdm", 7, 2), ("gf-vdm", 1, 1)])
def test_every_erasure_pattern(O, scheme, k, r):
    n = k + r
    L = 24
    base = O.make_windows(0, 5, 0, 1, k, r, L, 32)
    O.encode_batch(sid(O, scheme), k, r, np.array([L], np.uint32), base)
    nwin = 1 << n
    wins = np.repeat(base, nwin, axis=0)
    pres = np.arange(nwin, dtype=np.uint64)
    O.erase(wins, pres, k, r, fill=0x5A)
    st = O.decode_batch(sid(O, scheme), k, r, np.full(nwin, L, np.uint32), wins, pres)
    for p in range(nwin):
        miss = [j for j in range(k) if not (p >> j) & 1]
        if scheme != "xor":  # MDS
            reps = sum(1 for i in range(r) if (p >> (k + i)) & 1)
            expect_ok = len(miss) <= reps
        else:
            expect_ok = True
            for g in range(r):
                mg = [j for j in miss if j % r == g]
                if mg and (len(mg) > 1 or not (p >> (k + g)) & 1):
                    expect_ok = False
        assert st[p] == (0 if expect_ok else 1), (p, miss)
        if expect_ok:
            assert np.array_equal(wins[p, :k, :L], base[0, :k, :L])
        elif scheme == "xor":  # recoverable groups are still recovered
            for j in range(k):
                g = j % r
                mg = [x for x in miss if x % r == g]
                if (p >> j) & 1 or (len(mg) == 1 and (p >> (k + g)) & 1):
                    assert np.array_equal(wins[p, j, :L], base[0, j, :L])


def test_lenprefix_framing_and_mixed_mtu(O):
    """a2/a9: u16be len || payload || zero pad; MTU 1200|9000; ~10% shortened to [64, MTU]."""
    seed, k, nwin = 0x5EEDFEC0, 32, 200
    mtus, short, total = set(), 0, 0
    for w in range(nwin):
        pk, S, sym = N.window(1, seed, w, k, 0)
        lens = [len(p) for p in pk]
        assert S == 2 + max(lens)
        mtu = max(lens) if any(l in (1200, 9000) for l in lens) else None
        for j, p in enumerate(pk):
            assert np.array_equal(N.deframe(sym[j]), p)
            assert not sym[j, 2 + len(p):].any()
            total += 1
            if len(p) not in (1200, 9000):
                short += 1
                assert 64 <= len(p) <= 9000
        if mtu:
            mtus.add(mtu)
    assert mtus == {1200, 9000}
    assert 0.07 < short / total < 0.13


def test_erasure_streams(O):
    seed = 0x5EEDFEC0
    # exact, GF: exactly r distinct sources, no repairs
    for w in range(300):
        p = O.lib().orc_present(1, seed, w, O.GF256, 16, 4)
        assert bin(p & 0xFFFF).count("1") == 12 and (p >> 16) == 0xF
    # exact, XOR: one source per group
    for w in range(300):
        p = O.lib().orc_present(1, seed, w, O.XOR, 8, 2)
        miss = [j for j in range(8) if not (p >> j) & 1]
        assert sorted(j % 2 for j in miss) == [0, 1]
    # iid p=0.1 over k+r=40: erasure rate and unrecoverable rate P(Bin(40,.1) > 8) ~ 1.55%
    nwin = 20000
    pres = O.presents(2, seed, 0, nwin, O.GF256, 32, 8)
    erased = sum(40 - bin(int(p)).count("1") for p in pres)
    assert abs(erased / (40 * nwin) - 0.1) < 0.005
    unrec = 0
    for p in pres:
        p = int(p)
        miss = 32 - bin(p & 0xFFFFFFFF).count("1")
        reps = bin(p >> 32).count("1")
        unrec += miss > reps
    # exact tail probability of the decodability event, computed by enumeration
    from math import comb
    q = 0.1
    pr = 0.0
    for ms in range(33):
        for mr in range(9):
            if ms > 8 - mr:
                pr += comb(32, ms) * q**ms * (1 - q)**(32 - ms) * comb(8, mr) * q**mr * (1 - q)**(8 - mr)
    assert abs(unrec / nwin - pr) < 4 * (pr * (1 - pr) / nwin) ** 0.5 + 1e-3


def test_digest_properties(O):
    k, r, L = 4, 2, 100
    wins = O.make_windows(0, 1, 0, 6, k, r, L, 112)
    S = np.full(6, L, np.uint32)
    d = O.batch_digest(k, r, S, wins)
    # order independent across windows when ids move with them
    perm = [3, 1, 5, 0, 2, 4]
    d2 = 0
    for w in perm:
        d2 ^= O.sm64(O.window_digest(k, r, L, wins[w]) + w)
    assert d == d2
    # padding beyond S is ignored, payload bytes are not
    w2 = wins.copy()
    w2[2, 1, L:] = 0xFF
    assert O.batch_digest(k, r, S, w2) == d
    w2[2, 1, L - 1] ^= 1
    assert O.batch_digest(k, r, S, w2) != d
