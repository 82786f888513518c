"""GF(2^8) block codes with k + r > 64 (up to 256):
the host side (no GPU).  The library's parity rows for wide codes equal the
numpy restatement's (oracle/np_oracle.py: Cauchy inv((k+i)^j), systematic
Vandermonde, RFC 8681 RLC rows), and the limits of every entry point.
PARITY UNPINNED vs the reference fec branch."""
import ctypes

import numpy as np
import pytest

import fecgpu
import np_oracle as N


@pytest.mark.parametrize("k,r,matrix", [(60, 8, "cauchy"), (120, 4, "cauchy"), (248, 8, "cauchy"),
                                        (90, 6, "vandermonde"), (150, 8, "rlc")])
def test_wide_parity_rows_vs_numpy(k, r, matrix):
    code = fecgpu.Code("gf256", k, r, matrix=matrix, rlc_key=77, rlc_dt=15)
    assert code.check() == 0
    scheme = {"cauchy": "gf", "vandermonde": "gf-vdm", "rlc": "rlc:77:15"}[matrix]
    assert np.array_equal(code.parity_rows(), N.generator(scheme, k, r)[k:])


def test_wide_limits():
    L = fecgpu.lib()
    assert fecgpu.Code("gf256", 248, 8).check() == 0
    assert fecgpu.Code("gf256", 249, 8).check() == fecgpu.ERR_UNSUPPORTED
    assert fecgpu.Code("gf256", 200, 9).check() == fecgpu.ERR_UNSUPPORTED
    assert fecgpu.Code("xor", 64, 4).check() == fecgpu.ERR_UNSUPPORTED
    # the Cauchy construction's points k + i ^ j stay below 256: every row nonzero
    rows = fecgpu.Code("gf256", 248, 8).parity_rows()
    assert rows.shape == (8, 248) and (rows != 0).all()
    # entry points without a GPU context refuse before touching the device
    code = fecgpu.Code("gf256", 100, 4).c
    buf = (ctypes.c_uint8 * 64)()
    assert L.fecgpu_encode_batch(None, ctypes.byref(code), buf, None, None, 10, 64, 1, 0, None) \
        == fecgpu.ERR_INVALID_ARG
