"""RFC 8681 / RFC 8682 random linear code (FECGPU_MATRIX_RLC) on CPU.

Pins: the TinyMT32 PRNG against the seed-1 output list that RFC 8682 §2.2
publishes (the TinyMT reference's check values for the parameter set mat1
0x8f7011ee, mat2 0xfc78ff1f, tmat 0x3793fdff); the documents are not in this
container, the values are restated from the RFC.  Then RFC 8681 §3.6's
coefficient generator, the C oracle against the independent numpy
restatement, and the product's host-side generator
(fecgpu_code_parity_rows, no device) against both.
"""
import itertools

import numpy as np
import pytest

import fecgpu
import oracle as O
import np_oracle as N

# RFC 8682 §2.2: tinymt32_generate_uint32() after tinymt32_init(seed = 1)
KAT_U32 = [2545341989, 981918433, 3715302833, 2387538352, 3591001365,
           3820442102, 2114400566, 2196103051, 2783359912, 764534509]
# the same outputs through RFC 8681's tinymt32_rand256() (& 0xFF) and rand16() (& 0xF)
KAT_256 = [37, 225, 177, 176, 21, 246, 54, 139, 168, 237]
KAT_16 = [5, 1, 1, 0, 5, 6, 6, 11, 8, 13]


def test_tinymt32_kat_c_oracle():
    out = O.tinymt32(1, 10)
    assert out == KAT_U32
    assert [x & 0xFF for x in out] == KAT_256
    assert [x & 0xF for x in out] == KAT_16


def test_tinymt32_kat_numpy_restatement():
    t = N.TinyMT32(1)
    assert [t.u32() for _ in range(10)] == KAT_U32


def test_tinymt32_restatements_agree_on_many_seeds():
    for seed in [0, 2, 3, 0xFFFF, 0x10000, 0xDEADBEEF, 0xFFFFFFFF]:
        t = N.TinyMT32(seed)
        assert O.tinymt32(seed, 64) == [t.u32() for _ in range(64)]


def test_dense_coefficients_are_rand256_without_zeros():
    """dt = 15: every coefficient is the next nonzero rand256() (RFC 8681 §3.6)."""
    cc = O.rlc_coefs(1, 10, 15)
    assert cc.tolist() == KAT_256       # seed 1's first ten rand256() are all nonzero
    assert (O.rlc_coefs(12345, 500, 15) != 0).all()


@pytest.mark.parametrize("dt", range(16))
def test_rlc_coefs_c_vs_numpy(dt):
    for key in [0, 1, 2, 255, 4660, 65535, 70000]:
        for n in [1, 7, 64]:
            assert np.array_equal(O.rlc_coefs(key, n, dt), N.rlc_coefs(key, n, dt)), (key, n, dt)


def test_repair_key_is_16_bits():
    assert np.array_equal(O.rlc_coefs(70000, 32, 15), O.rlc_coefs(70000 & 0xFFFF, 32, 15))


def test_density_threshold():
    """Coefficient i is nonzero with probability (dt + 1) / 16."""
    for dt in [0, 3, 7, 11]:
        cc = np.concatenate([O.rlc_coefs(key, 256, dt) for key in range(64)])
        frac = np.count_nonzero(cc) / cc.size
        assert abs(frac - (dt + 1) / 16) < 0.03, (dt, frac)


@pytest.mark.parametrize("k,r,key,dt", [(16, 4, 0, 15), (8, 2, 1, 15), (32, 8, 4660, 15),
                                        (10, 6, 4660, 7), (6, 6, 65535, 1), (56, 8, 65530, 0)])
def test_product_parity_rows_match_oracles(k, r, key, dt):
    """The library's host generator (fec_spec.h rlc_coefs) equals both restatements;
    row i wraps its repair_key at 2^16."""
    P = fecgpu.Code("gf256", k, r, matrix="rlc", rlc_key=key, rlc_dt=dt).parity_rows()
    assert np.array_equal(P, O.matrix(O.RLC(key, dt), k, r))
    assert np.array_equal(P, N.generator(f"rlc:{key}:{dt}", k, r)[k:])


def test_other_matrices_parity_rows_match_oracle():
    for k, r in [(16, 4), (5, 5), (32, 8)]:
        assert np.array_equal(fecgpu.Code("gf256", k, r).parity_rows(), O.cauchy(k, r))
        assert np.array_equal(fecgpu.Code("gf256", k, r, matrix="vandermonde").parity_rows(),
                              O.vandermonde(k, r))


@pytest.mark.parametrize("k,r,key,dt", [(4, 3, 9, 15), (4, 4, 3, 2), (5, 3, 77, 0), (3, 5, 1, 4)])
def test_every_erasure_pattern_c_vs_numpy(k, r, key, dt):
    """All 2^(k+r) present masks: recoverable iff the received rows have rank k
    (numpy: elimination over every received row) == the C oracle's greedy
    choice of independent repairs; recovered bytes equal the originals."""
    n, L = k + r, 12
    scheme = O.RLC(key, dt)
    wins = O.make_windows(0, 99, 3, 1, k, r, L, 16)
    S = np.full(1, L, np.uint32)
    O.encode_batch(scheme, k, r, S, wins)
    G = N.generator(f"rlc:{key}:{dt}", k, r)
    assert np.array_equal(wins[0, k:, :L], N.matmul(G[k:], wins[0, :k, :L]))
    nonmds = 0
    for p in range(1 << n):
        d = wins.copy()
        O.erase(d, np.array([p], np.uint64), k, r, fill=0x5A)
        st = O.decode_batch(scheme, k, r, S, d, np.array([p], np.uint64))
        rows = [i for i in range(n) if (p >> i) & 1]
        _, ok = N.decode(f"rlc:{key}:{dt}", k, r, d[0, :, :L], p)
        assert (st[0] == 0) == ok, p
        if ok:
            assert np.array_equal(d[0, :k, :L], wins[0, :k, :L]), p
        miss = sum(1 for j in range(k) if not (p >> j) & 1)
        reps = len(rows) - (k - miss)
        nonmds += int(miss <= reps and not ok)
    if dt < 15:
        assert nonmds > 0   # sparse rows: some masks an MDS code recovers are singular here
