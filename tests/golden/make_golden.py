#!/usr/bin/env python3
"""Generate tests/golden/*.npz with the independent numpy restatement (oracle/np_oracle.py).

PARITY UNPINNED: the reference fec branch is not mounted and
holds no golden vectors here, so these fixtures pin the C oracle and the HIP
kernels to an independently written restatement of the same contract
(SURVEY.md Appendix A), not to the reference's own outputs.

Run from the repo root:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import np_oracle as N  # noqa: E402

SEED = 0x601DE5

# (name, scheme, k, r, L, erasure, nwin, w0)
CASES = [
    ("xor_k4r1_L64_exact", "xor", 4, 1, 64, 1, 4, 0),
    ("xor_k8r2_L100_exact", "xor", 8, 2, 100, 1, 4, 17),
    ("xor_k5r3_L17_iid", "xor", 5, 3, 17, 2, 8, 3),
    ("gf_k16r4_L64_exact", "gf", 16, 4, 64, 1, 4, 0),
    ("gf_k4r2_L1_exact", "gf", 4, 2, 1, 1, 4, 5),
    ("gf_k10r7_L33_iid", "gf", 10, 7, 33, 2, 8, 100),
    ("gf_k32r8_L48_iid", "gf", 32, 8, 48, 2, 4, 1 << 20),
    ("gf_k56r8_L16_exact", "gf", 56, 8, 16, 1, 2, 9),
    # systematic Vandermonde rows (FECGPU_MATRIX_VANDERMONDE), scheme id 2
    ("vdm_k5r5_L24_iid", "gf-vdm", 5, 5, 24, 2, 8, 40),
    ("vdm_k16r4_L64_exact", "gf-vdm", 16, 4, 64, 1, 4, 7),
    ("vdm_k32r8_L40_iid", "gf-vdm", 32, 8, 40, 2, 4, 1 << 21),
    # RFC 8681 random linear code rows (FECGPU_MATRIX_RLC): "rlc:KEY:DT",
    # scheme id 3 | DT << 4 | KEY << 8 (the C oracle's ORC_RLC)
    ("rlc_k16r4_L64_exact_dt15", "rlc:1:15", 16, 4, 64, 1, 4, 3),
    ("rlc_k10r6_L33_iid_dt7", "rlc:4660:7", 10, 6, 33, 2, 16, 50),
    ("rlc_k6r6_L20_iid_dt1", "rlc:65535:1", 6, 6, 20, 2, 24, 7),
]


def make(name, scheme, k, r, L, erasure, nwin, w0):
    src = np.zeros((nwin, k, L), np.uint8)
    rep = np.zeros((nwin, r, L), np.uint8)
    pres = np.zeros(nwin, np.uint64)
    status = np.zeros(nwin, np.uint8)
    dec = np.zeros((nwin, k, L), np.uint8)
    for i in range(nwin):
        w = w0 + i
        _, S, sym = N.window(0, SEED, w, k, L)
        assert S == L
        src[i] = sym
        rep[i] = N.encode(scheme, k, r, sym)
        p = N.present(erasure, SEED, w, scheme, k, r)
        pres[i] = p
        full = np.concatenate([sym, rep[i]])
        garbage = full.copy()
        for s in range(k + r):
            if not (p >> s) & 1:
                garbage[s] = 0xAB
        out, ok = N.decode(scheme, k, r, garbage, p)
        status[i] = 0 if ok else 1
        dec[i] = out
    np.savez_compressed(os.path.join(HERE, name + ".npz"), src=src, repair=rep, present=pres,
                        status=status, decoded=dec,
                        meta=np.array([N.scheme_id(scheme), k, r, L, erasure, nwin, w0, SEED],
                                      np.int64))


if __name__ == "__main__":
    # optional names: regenerate only those fixtures (others keep their bytes)
    want = set(sys.argv[1:])
    for c in CASES:
        if want and c[0] not in want:
            continue
        make(*c)
        print("wrote", c[0])
