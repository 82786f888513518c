"""GPU parity of the bit-sliced syndrome GF decode (fec_kernels.hip
gf_decode_bs_gs_kernel): Cauchy k 16 r 4 on uniform rows,
against the numpy oracle (oracle/np_oracle.py decode) and the table decode
(the "bsdec" tuning knob set to 0) on the same inputs.

Windows carry 0..5 missing sources and 0..2 missing repairs (so some are
unrecoverable and some have nothing to do), missing rows poisoned first: the
recovered bytes equal the originals, statuses equal the oracle's, and every
other byte of the buffer (received rows, repairs, unrecoverable windows'
poisoned rows, the padding past S) equals the table decode's output.
PARITY UNPINNED vs the reference fec branch."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import fecgpu  # noqa: E402
import np_oracle as N  # noqa: E402

pytestmark = pytest.mark.gpu

K, R = 16, 4


def _bits(nwin, rng, emax=R + 1):
    bits = np.ones((nwin, K + R), bool)
    for w in range(nwin):
        e = int(rng.integers(0, emax + 1))
        bits[w, rng.choice(K, e, replace=False)] = False
        lr = int(rng.integers(0, 3)) if rng.random() < 0.4 else 0
        if lr:
            bits[w, K + rng.choice(R, lr, replace=False)] = False
    return bits


def _decode(c, code, enc, bits, L, stride):
    nwin = enc.shape[0]
    d = torch.from_numpy(enc.copy()).cuda()
    d[~torch.from_numpy(bits).cuda()] = 0xAB
    pres = np.zeros(nwin, np.uint64)
    for i in range(K + R):
        pres |= bits[:, i].astype(np.uint64) << np.uint64(i)
    st = torch.full((nwin,), 7, dtype=torch.uint8, device="cuda")
    c.decode_batch(code, d, torch.from_numpy(pres.view(np.int64)).cuda(), st, nwin=nwin, stride=stride,
                   sym_len_all=L)
    torch.cuda.synchronize()
    return d.cpu().numpy(), st.cpu().numpy(), pres


@pytest.mark.parametrize("L,stride,nwin", [(1200, 1200, 301), (1000, 1008, 97), (1500, 1520, 203),
                                           (2048, 2048, 64), (1183, 1200, 150), (4000, 4000, 23),
                                           (1200, 1216, 1), (1200, 1200, 12), (1200, 1200, 13)])
def test_bsdec_vs_oracle_and_table_decode(L, stride, nwin):
    rng = np.random.default_rng(L + nwin)
    wins = np.zeros((nwin, K + R, stride), np.uint8)
    wins[:, :K, :L] = rng.integers(0, 256, (nwin, K, L), dtype=np.uint8)
    code = fecgpu.Code("gf256", K, R)
    ref = fecgpu.Context()
    ref.set_tuning("bsdec", 0)
    c = fecgpu.Context()  # bsdec on by default
    try:
        d = torch.from_numpy(wins).cuda()
        ref.encode_batch(code, d, nwin=nwin, stride=stride, sym_len_all=L)
        torch.cuda.synchronize()
        enc = d.cpu().numpy()
        bits = _bits(nwin, rng)
        got, gst, pres = _decode(c, code, enc, bits, L, stride)
        want, wst, _ = _decode(ref, code, enc, bits, L, stride)
        assert np.array_equal(gst, wst), "statuses differ from the table decode"
        for w in range(nwin):
            sym = enc[w, :, :L].copy()
            sym[~bits[w]] = 0xAB
            _, ok = N.decode("gf", K, R, sym, int(pres[w]))
            assert gst[w] == (0 if ok else 1), f"window {w}: status {gst[w]}, oracle ok={ok}"
            if ok:
                assert np.array_equal(got[w, :K, :L], wins[w, :K, :L]), f"window {w}: recovered bytes differ"
        # the whole buffer, padding included (columns past S inside the last
        # 16-B column are recovered as zeros by both; past it nothing is written)
        assert np.array_equal(got, want), "buffer differs from the table decode"
    finally:
        c.close()
        ref.close()


def test_bsdec_every_erasure_pattern_of_one_window_size():
    """All C(16, e) source-erasure sets for e = 4 are too many; take every
    pattern with e <= 2, and 600 random ones with e = 3, 4 (all repairs present
    and with one repair missing), one window each, in one batch."""
    import itertools
    pats = [()]
    pats += [(a,) for a in range(K)]
    pats += list(itertools.combinations(range(K), 2))
    rng = np.random.default_rng(5)
    for e in (3, 4):
        for _ in range(300):
            pats.append(tuple(sorted(rng.choice(K, e, replace=False).tolist())))
    nwin, L = len(pats), 1200
    bits = np.ones((nwin, K + R), bool)
    for w, p in enumerate(pats):
        bits[w, list(p)] = False
        if w % 3 == 1 and len(p) < R:
            bits[w, K + int(rng.integers(0, R))] = False
    wins = np.zeros((nwin, K + R, L), np.uint8)
    wins[:, :K] = rng.integers(0, 256, (nwin, K, L), dtype=np.uint8)
    code = fecgpu.Code("gf256", K, R)
    c = fecgpu.Context()
    try:
        d = torch.from_numpy(wins).cuda()
        c.encode_batch(code, d, nwin=nwin, stride=L, sym_len_all=L)
        torch.cuda.synchronize()
        enc = d.cpu().numpy()
        got, gst, _ = _decode(c, code, enc, bits, L, L)
        assert (gst == 0).all()
        assert np.array_equal(got[:, :K], enc[:, :K]), "recovered sources differ from the encoded ones"
    finally:
        c.close()


def test_bsdec_full_size_iid_erasures():
    """cfg3's geometry at full size (262,144 windows of k 16 r 4 x 1200 B) with
    i.i.d. 10 % erasures over all 20 symbols: windows with 0-4 missing sources,
    missing repairs, and unrecoverable ones (more missing sources than present
    repairs) in one launch of the syndrome decode.  Every recoverable window's
    sources equal the originals, every status equals the one predicted from the
    masks (workloads.Batch.verify), and the table decode reports the same."""
    import dataclasses
    from fecgpu import workloads as WL
    cfg = dataclasses.replace(WL.CONFIGS[3], erasure=WL.ERASURE_IID, name="cfg3-iid10")
    b = WL.Batch.allocate(cfg, cfg.nwin_per_gpu, torch.device("cuda"))
    res = {}
    for knob in (1, 0):
        c = fecgpu.Context()
        c.set_tuning("bsdec", knob)
        try:
            b.synthesize(c, 0)
            b.make_erasures(c, 0)
            res[knob] = b.verify(c, 0)
        finally:
            c.close()
    assert res[1]["ok"] and res[1]["status_matches_expected"], res[1]
    assert res[1]["unrecoverable"] > 0
    assert res[1]["unrecoverable"] == res[0]["unrecoverable"] and res[0]["ok"], res
