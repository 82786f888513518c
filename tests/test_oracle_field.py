"""Pin the oracle's field: known answers, exhaustive axioms,
and an independent third-party check (sympy.polys.galoistools)."""
import numpy as np
import pytest

import np_oracle as N


@pytest.fixture(scope="module")
def O(oracle_lib):
    return oracle_lib


@pytest.fixture(scope="module")
def table(O):
    t = np.zeros((256, 256), np.uint8)
    for a in range(256):
        for b in range(256):
            t[a, b] = O.gf_mul(a, b)
    return t


def test_known_answers(O):
    # SURVEY.md §4 T0 (ISA-L / Jerasure conventions for 0x11D)
    assert O.lib().orc_gf_exp(8) == 0x1D
    assert O.gf_inv(2) == 0x8E
    assert O.gf_inv(3) == 0xF4
    assert O.gf_mul(0x53, 0xCA) == 0x8F
    assert list(O.cauchy(16, 4)[0, :4]) == [0xD8, 0x72, 0xC0, 0x58]
    # generator 2 has order 255
    assert len({O.lib().orc_gf_exp(i) for i in range(255)}) == 255


def test_table_matches_independent_clmul(table):
    assert np.array_equal(table, N.mul_table())


def test_field_axioms_exhaustive(O, table):
    T = table.astype(np.int64)
    assert np.array_equal(T, T.T)  # commutative
    assert np.all(T[1] == np.arange(256)) and np.all(T[0] == 0)
    a = np.arange(256)
    # distributive over xor: a*(b^c) == a*b ^ a*c for all a, b, c
    for b in range(256):
        lhs = table[:, b][:, None] ^ table  # a*b ^ a*c  -> [a, c]
        rhs = table[a[:, None], (b ^ a)[None, :]]  # a*(b^c)
        assert np.array_equal(lhs, rhs)
    # associative: (a*b)*c == a*(b*c), every a, b, c
    for c in range(256):
        ab_c = table[table, c]               # [a, b] -> (a*b)*c
        a_bc = table[:, table[:, c]]         # [a, b] -> a*(b*c)
        assert np.array_equal(ab_c, a_bc)
    for x in range(1, 256):
        assert O.gf_mul(x, O.gf_inv(x)) == 1


def test_against_sympy_galoistools(O):
    gt = pytest.importorskip("sympy.polys.galoistools")
    from sympy.polys.domains import ZZ
    poly = [ZZ(int(b)) for b in bin(0x11D)[2:]]
    rng = np.random.default_rng(2024)

    def to_poly(x):
        return [ZZ(int(b)) for b in bin(x)[2:]] if x else []

    def from_poly(p):
        v = 0
        for b in p:
            v = (v << 1) | int(b)
        return v

    for a, b in rng.integers(0, 256, (2000, 2)):
        prod = gt.gf_rem(gt.gf_mul(to_poly(int(a)), to_poly(int(b)), 2, ZZ), poly, 2, ZZ)
        assert from_poly(prod) == O.gf_mul(int(a), int(b))


def test_cauchy_is_mds(O):
    """Every square submatrix of the systematic Cauchy rows is invertible (k=8, r=4:
    all 1x1..4x4 minors), so any e <= r erasures are recoverable."""
    import itertools
    k, r = 8, 4
    C = O.cauchy(k, r)
    for e in range(1, r + 1):
        for rows in itertools.combinations(range(r), e):
            for cols in itertools.combinations(range(k), e):
                M = C[np.ix_(rows, cols)].copy()
                # Gaussian elimination over GF(2^8) via numpy tables
                for c in range(e):
                    p = next((i for i in range(c, e) if M[i, c]), None)
                    assert p is not None
                    M[[c, p]] = M[[p, c]]
                    M[c] = N.mul_table()[N.inv(int(M[c, c]))][M[c]]
                    for i in range(e):
                        if i != c and M[i, c]:
                            M[i] ^= N.mul_table()[M[i, c]][M[c]]


def test_vandermonde_kat(oracle_lib):
    """FECGPU_MATRIX_VANDERMONDE pinned by the published known answer of the
    libraries that define it (Backblaze JavaReedSolomon's construction; the 5+5
    one-encode test of klauspost/reedsolomon and of the Rust crate
    reed-solomon-erasure): data {0,1},{4,5},{2,3},{6,7},{8,9} -> parity
    {12,13},{10,11},{14,15},{90,91},{94,95}.  C oracle and numpy restatement."""
    import numpy as np
    import np_oracle as N
    src = np.array([[0, 1], [4, 5], [2, 3], [6, 7], [8, 9]], np.uint8)
    want = [[12, 13], [10, 11], [14, 15], [90, 91], [94, 95]]
    assert N.encode("gf-vdm", 5, 5, src).tolist() == want
    win = np.zeros((1, 10, 16), np.uint8)
    win[0, :5, :2] = src
    oracle_lib.encode_batch(oracle_lib.GF256_VDM, 5, 5, np.array([2], np.uint32), win)
    assert win[0, 5:, :2].tolist() == want
    for k, r in [(5, 5), (8, 2), (16, 4), (32, 8), (56, 8), (3, 7)]:
        assert np.array_equal(N.vandermonde(k, r), oracle_lib.vandermonde(k, r))


@pytest.mark.parametrize("k,r", [(4, 4), (6, 3), (5, 5), (10, 2)])
def test_vandermonde_parity_rows_are_mds(oracle_lib, k, r):
    """Every square submatrix of the parity rows is nonsingular (systematic MDS),
    which is also why the GPU decode plan needs no pivoting for this matrix."""
    import itertools
    import numpy as np
    import np_oracle as N
    P = oracle_lib.vandermonde(k, r)
    for e in range(1, min(k, r) + 1):
        for rows in itertools.combinations(range(r), e):
            for cols in itertools.combinations(range(k), e):
                A = P[np.ix_(rows, cols)]
                N._gj_inverse(A)  # raises StopIteration if singular
