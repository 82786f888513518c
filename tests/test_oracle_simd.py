"""The CPU baseline codec (oracle/fec_cpu_simd.c: AVX2 split-nibble tables, GFNI
affine products, scalar) gives byte-identical repairs, statuses and recovered
sources to the scalar oracle at every level this CPU has — so bench.py's
cpu_baseline times the same work the GPU does."""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def O(oracle_lib):
    yield oracle_lib
    oracle_lib.simd_set_level(-1)


CASES = [  # scheme, k, r, workload, L, erasure
    ("xor", 8, 2, 0, 1200, 1), ("xor", 5, 3, 0, 33, 2), ("xor", 4, 1, 1, 0, 2),
    ("gf", 16, 4, 0, 1200, 1), ("gf", 32, 8, 1, 0, 2), ("gf", 10, 7, 0, 61, 2),
    ("gf", 3, 5, 0, 16, 1), ("gf", 56, 8, 0, 95, 1), ("gf-vdm", 16, 4, 0, 130, 2),
]


@pytest.mark.parametrize("scheme,k,r,wl,L,era", CASES)
def test_simd_levels_match_scalar_oracle(O, scheme, k, r, wl, L, era):
    sid = {"xor": O.XOR, "gf": O.GF256, "gf-vdm": O.GF256_VDM}[scheme]
    nwin = 23
    S = O.sym_lens(wl, 77, 0, nwin, k, L)
    stride = O.round_up(int(S.max()), 16)
    base = O.make_windows(wl, 77, 0, nwin, k, r, L, stride)
    present = O.presents(era, 77, 0, nwin, sid, k, r)
    ref = base.copy()
    O.encode_batch(sid, k, r, S, ref, 2)
    ref_dec = ref.copy()
    O.erase(ref_dec, present, k, r, fill=0xAB)
    ref_st = O.decode_batch(sid, k, r, S, ref_dec, present, 2)
    for level in range(O.simd_detect() + 1):
        O.simd_set_level(level)
        assert O.simd_level() == level
        enc = base.copy()
        O.encode_batch_simd(sid, k, r, S, enc, 3)
        for w in range(nwin):
            assert np.array_equal(enc[w, :, :S[w]], ref[w, :, :S[w]]), (level, w)
        dec = enc.copy()
        O.erase(dec, present, k, r, fill=0xAB)
        st = O.decode_batch_simd(sid, k, r, S, dec, present, 3)
        assert np.array_equal(st, ref_st), level
        for w in range(nwin):
            assert np.array_equal(dec[w, :k, :S[w]], ref_dec[w, :k, :S[w]]), (level, w)
    O.simd_set_level(-1)
