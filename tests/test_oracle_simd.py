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


def _sw_case(O, seed, nsrc, k, W, dt, L, loss):
    import np_oracle as N
    rng = np.random.default_rng(seed)
    stride = O.round_up(L, 16)
    src = np.zeros((nsrc, stride), np.uint8)
    src[:, :L] = rng.integers(0, 256, (nsrc, L), dtype=np.uint8)
    h = N.sw_schedule(nsrc, k, W, key0=seed, dt=dt)
    hdr = np.zeros(len(h), O.SW_REPAIR_DTYPE)
    for t, (fss, nss, key, d) in enumerate(h):
        hdr[t]["fss"], hdr[t]["nss"], hdr[t]["key"], hdr[t]["dt"] = fss, nss, key, d
    sp = (rng.random(nsrc) >= loss).astype(np.uint8)
    rp = (rng.random(len(h)) >= loss).astype(np.uint8)
    return src, hdr, sp, rp


@pytest.mark.parametrize("nsrc,k,W,dt,L,loss", [(3000, 8, 32, 15, 1200, 0.02), (3000, 8, 32, 15, 100, 0.10),
                                                (2000, 4, 64, 15, 33, 0.15), (1500, 1, 255, 15, 40, 0.05),
                                                (1200, 3, 20, 3, 17, 0.2)])
def test_sw_simd_codec_matches_oracle(O, nsrc, k, W, dt, L, loss):
    """The sliding-window CPU baseline (fec_cpu_simd.c orc_sw_*_simd: vectorised,
    threads over repairs / runs of whole linked systems) equals the scalar oracle
    (orc_sw_encode, and the banded decode equal to the dense one) at every SIMD
    level and thread count, long linked systems included."""
    src, hdr, sp, rp = _sw_case(O, nsrc + W, nsrc, k, W, dt, L, loss)
    ref = O.sw_encode(src, hdr, L)
    od = src.copy()
    od[sp == 0] = 0xAB
    ost, on = O.sw_decode_banded(od, sp, ref, rp, hdr, L)
    for level in range(O.simd_detect() + 1):
        O.simd_set_level(level)
        for nth in (1, 5):
            rep = O.sw_encode_simd(src, hdr, L, nth)
            assert np.array_equal(rep[:, :L], ref[:, :L]), (level, nth)
            d = src.copy()
            d[sp == 0] = 0xAB
            st, n = O.sw_decode_simd(d, sp, rep, rp, hdr, L, nth)
            assert np.array_equal(st, ost) and n == on, (level, nth)
            assert np.array_equal(d[:, :L], od[:, :L]), (level, nth)
    O.simd_set_level(-1)


@pytest.mark.parametrize("k,r,scheme,L", [(120, 8, "gf", 300), (248, 8, "gf", 64), (100, 5, "rlc", 97)])
def test_simd_codec_wide_codes_match_numpy_oracle(O, k, r, scheme, L):
    """k + r > 64 (the wide bench lines' CPU baseline): repairs equal the numpy
    restatement's (np_oracle.encode), and the decode over multi-word present masks
    recovers exactly the windows np_oracle.decode does, byte-exact."""
    import np_oracle as N
    key, dt = 9, 15
    sid = O.GF256 if scheme == "gf" else O.RLC(key, dt)
    nps = "gf" if scheme == "gf" else f"rlc:{key}:{dt}"
    nwin, n = 6, k + r
    stride = O.round_up(L, 16)
    rng = np.random.default_rng(k + r)
    wins = np.zeros((nwin, n, stride), np.uint8)
    wins[:, :k, :L] = rng.integers(0, 256, (nwin, k, L), dtype=np.uint8)
    S = np.full(nwin, L, np.uint32)
    enc = wins.copy()
    O.encode_batch_simd(sid, k, r, S, enc, 2)
    for w in range(nwin):
        assert np.array_equal(enc[w, k:, :L], N.encode(nps, k, r, wins[w, :k, :L])), w
    nw = (n + 63) // 64
    pres = np.zeros((nwin, nw), np.uint64)
    bits = np.ones((nwin, n), bool)
    for w in range(nwin):
        e = w % (r + 2)  # 0 .. r + 1 missing sources
        bits[w, rng.choice(k, e, replace=False)] = False
        if w % 3 == 1:
            bits[w, k + rng.integers(0, r)] = False
    for i in range(n):
        pres[:, i // 64] |= bits[:, i].astype(np.uint64) << np.uint64(i % 64)
    dec = enc.copy()
    dec[~bits] = 0xAB
    st = O.decode_batch_simd(sid, k, r, S, dec, pres, 2)
    for w in range(nwin):
        p = 0
        for i in np.flatnonzero(bits[w]):
            p |= 1 << int(i)
        sym = enc[w, :, :L].copy()
        sym[~bits[w]] = 0xAB
        _, ok = N.decode(nps, k, r, sym, p)
        assert st[w] == (0 if ok else 1), w
        if ok:
            assert np.array_equal(dec[w, :k, :L], wins[w, :k, :L]), w
