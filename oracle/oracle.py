"""ctypes wrapper over oracle/_build/liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, always as the checker, never as the measured or shipped path.
PARITY UNPINNED: see fec_oracle.h for what pins the oracle.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

XOR, GF256, GF256_VDM = 0, 1, 2     # GF256: Cauchy rows; GF256_VDM: systematic Vandermonde


def RLC(key0: int, dt: int) -> int:
    """Scheme id of the RFC 8681 random linear code rows (fec_oracle.h ORC_RLC):
    parity row i from repair_key key0 + i at density threshold dt."""
    return 3 | (dt << 4) | (key0 << 8)


def scheme_kind(scheme: int) -> int:
    return scheme & 0xF
FIXED_WL, MIXED_WL = 0, 1            # workloads
ERA_NONE, ERA_EXACT, ERA_IID = 0, 1, 2
OK, UNRECOVERABLE = 0, 1


def build() -> str:
    """Compile the oracle with its Makefile (gcc only)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u8, u32, u64, i32 = ctypes.c_uint8, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
        vp = ctypes.c_void_p
        sig = {
            "orc_gf_mul": (u8, [u8, u8]),
            "orc_gf_inv": (u8, [u8]),
            "orc_gf_exp": (u8, [i32]),
            "orc_gf_log": (i32, [u8]),
            "orc_cauchy": (None, [i32, i32, vp]),
            "orc_vandermonde": (None, [i32, i32, vp]),
            "orc_matrix": (None, [i32, i32, i32, vp]),
            "orc_tinymt32": (None, [u32, i32, vp]),
            "orc_rlc_coefs": (i32, [u32, i32, i32, vp]),
            "orc_sw_encode": (None, [vp, u64, u32, u32, vp, u64, vp]),
            "orc_sw_decode": (ctypes.c_int64, [vp, vp, u64, vp, vp, vp, u64, u32, u32, vp]),
            "orc_sw_decode_banded": (ctypes.c_int64, [vp, vp, u64, vp, vp, vp, u64, u32, u32, vp]),
            "orc_sm64": (u64, [u64]),
            "orc_pkt_len": (u32, [i32, u64, u64, i32, i32, u32]),
            "orc_sym_len": (u32, [i32, u64, u64, i32, u32]),
            "orc_fill_window": (None, [i32, u64, u64, i32, i32, u32, u32, vp]),
            "orc_present": (u64, [i32, u64, u64, i32, i32, i32]),
            "orc_encode": (None, [i32, i32, i32, u32, u32, vp]),
            "orc_decode": (i32, [i32, i32, i32, u32, u32, u64, vp]),
            "orc_window_digest": (u64, [i32, i32, u32, u32, vp]),
            "orc_encode_batch": (None, [i32, i32, i32, vp, u32, u64, vp, i32]),
            "orc_decode_batch": (None, [i32, i32, i32, vp, u32, u64, vp, vp, vp, i32]),
            "orc_make_batch": (u64, [i32, u64, u64, u64, i32, i32, i32, i32, u32, u32, vp, vp, vp,
                                     i32]),
            "orc_simd_detect": (i32, []),
            "orc_simd_level": (i32, []),
            "orc_simd_set_level": (None, [i32]),
            "orc_encode_batch_simd": (None, [i32, i32, i32, vp, u32, u64, vp, i32]),
            "orc_decode_batch_simd": (None, [i32, i32, i32, vp, u32, u64, vp, vp, vp, i32]),
            "orc_decode_batch_simd_w": (None, [i32, i32, i32, vp, u32, u64, i32, vp, vp, vp, i32]),
            "orc_sw_encode_simd": (None, [vp, u64, u32, u32, vp, u64, vp, i32]),
            "orc_sw_decode_simd": (ctypes.c_int64, [vp, vp, u64, vp, vp, vp, u64, u32, u32, vp, i32]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _p(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.c_void_p)


def gf_mul(a: int, b: int) -> int:
    return lib().orc_gf_mul(a, b)


def gf_inv(a: int) -> int:
    return lib().orc_gf_inv(a)


def cauchy(k: int, r: int) -> np.ndarray:
    C = np.zeros((r, k), np.uint8)
    lib().orc_cauchy(k, r, _p(C))
    return C


def vandermonde(k: int, r: int) -> np.ndarray:
    """Parity rows of the systematic Vandermonde generator (Backblaze construction)."""
    P = np.zeros((r, k), np.uint8)
    lib().orc_vandermonde(k, r, _p(P))
    return P


def matrix(scheme: int, k: int, r: int) -> np.ndarray:
    """Parity rows [r, k] of a GF scheme id."""
    P = np.zeros((r, k), np.uint8)
    lib().orc_matrix(scheme, k, r, _p(P))
    return P


def tinymt32(seed: int, n: int) -> list:
    """RFC 8682 TinyMT32 outputs 1..n after tinymt32_init(seed)."""
    out = np.zeros(n, np.uint32)
    lib().orc_tinymt32(seed, n, _p(out))
    return [int(x) for x in out]


def rlc_coefs(key: int, n: int, dt: int) -> np.ndarray:
    """RFC 8681 §3.6 coding coefficients (m = 8)."""
    cc = np.zeros(n, np.uint8)
    assert lib().orc_rlc_coefs(key, n, dt, _p(cc)) == 0
    return cc


SW_REPAIR_DTYPE = [("fss", "<u8"), ("nss", "<u2"), ("key", "<u2"), ("dt", "u1"), ("reserved", "u1", (3,))]


def sw_encode(src: np.ndarray, hdr: np.ndarray, S: int) -> np.ndarray:
    """Sliding-window RLC repairs [nrep, stride] of src [nsrc, stride] (headers SW_REPAIR_DTYPE)."""
    nsrc, stride = src.shape
    rep = np.zeros((len(hdr), stride), np.uint8)
    src = np.ascontiguousarray(src)
    lib().orc_sw_encode(_p(src), nsrc, S, stride, _p(hdr), len(hdr), _p(rep))
    return rep


def sw_decode(src: np.ndarray, src_present: np.ndarray, rep: np.ndarray, rep_present: np.ndarray,
              hdr: np.ndarray, S: int):
    """In place on src; -> (status per source, number recovered)."""
    nsrc, stride = src.shape
    st = np.zeros(nsrc, np.uint8)
    n = lib().orc_sw_decode(_p(src), _p(src_present), nsrc, _p(rep), _p(rep_present), _p(hdr),
                            len(hdr), S, stride, _p(st))
    return st, int(n)


def sw_decode_banded(src: np.ndarray, src_present: np.ndarray, rep: np.ndarray, rep_present: np.ndarray,
                     hdr: np.ndarray, S: int):
    """Same contract and results as sw_decode, by banded elimination (no size
    limit; oracle/fec_sw_banded.c).  In place on src; -> (status, #recovered)."""
    nsrc, stride = src.shape
    st = np.zeros(nsrc, np.uint8)
    n = lib().orc_sw_decode_banded(_p(src), _p(src_present), nsrc, _p(rep), _p(rep_present), _p(hdr),
                                   len(hdr), S, stride, _p(st))
    return st, int(n)


def sw_encode_simd(src: np.ndarray, hdr: np.ndarray, S: int, nthreads: int = 1) -> np.ndarray:
    """sw_encode on the CPU baseline codec (fec_cpu_simd.c; same outputs)."""
    nsrc, stride = src.shape
    rep = np.zeros((len(hdr), stride), np.uint8)
    src = np.ascontiguousarray(src)
    lib().orc_sw_encode_simd(_p(src), nsrc, S, stride, _p(hdr), len(hdr), _p(rep), nthreads)
    return rep


def sw_decode_simd(src: np.ndarray, src_present: np.ndarray, rep: np.ndarray, rep_present: np.ndarray,
                   hdr: np.ndarray, S: int, nthreads: int = 1):
    """sw_decode on the CPU baseline codec (headers in fss order).  In place;
    -> (status, #recovered)."""
    nsrc, stride = src.shape
    st = np.zeros(nsrc, np.uint8)
    n = lib().orc_sw_decode_simd(_p(src), _p(src_present), nsrc, _p(rep), _p(rep_present), _p(hdr),
                                 len(hdr), S, stride, _p(st), nthreads)
    return st, int(n)


def sm64(x: int) -> int:
    return lib().orc_sm64(x & 0xFFFFFFFFFFFFFFFF)


def round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def sym_lens(workload: int, seed: int, w0: int, nwin: int, k: int, L: int) -> np.ndarray:
    f = lib().orc_sym_len
    return np.array([f(workload, seed, w0 + w, k, L) for w in range(nwin)], np.uint32)


def make_windows(workload: int, seed: int, w0: int, nwin: int, k: int, r: int, L: int,
                 stride: int) -> np.ndarray:
    """[nwin, k+r, stride] u8 with sources filled, repairs zero (A.3/A.4)."""
    wins = np.zeros((nwin, k + r, stride), np.uint8)
    f = lib().orc_fill_window
    for w in range(nwin):
        f(workload, seed, w0 + w, k, r, L, stride, _p(wins[w]))
    return wins


def make_batch(workload: int, seed: int, w0: int, nwin: int, scheme: int, erasure: int, k: int,
               r: int, L: int, stride: int, nthreads: int = 1):
    """-> (wins [nwin, k+r, stride], S [nwin], present [nwin], source-packet bytes)."""
    wins = np.zeros((nwin, k + r, stride), np.uint8)
    S = np.zeros(nwin, np.uint32)
    pres = np.zeros(nwin, np.uint64)
    src = lib().orc_make_batch(workload, seed, w0, nwin, scheme, erasure, k, r, L, stride,
                               _p(wins), _p(S), _p(pres), nthreads)
    return wins, S, pres, int(src)


def presents(erasure: int, seed: int, w0: int, nwin: int, scheme: int, k: int, r: int) -> np.ndarray:
    f = lib().orc_present
    return np.array([f(erasure, seed, w0 + w, scheme, k, r) for w in range(nwin)], np.uint64)


def encode_batch(scheme: int, k: int, r: int, S: np.ndarray, wins: np.ndarray, nthreads: int = 1):
    nwin, _, stride = wins.shape
    S = np.ascontiguousarray(S, np.uint32)
    lib().orc_encode_batch(scheme, k, r, _p(S), stride, nwin, _p(wins), nthreads)


def decode_batch(scheme: int, k: int, r: int, S: np.ndarray, wins: np.ndarray,
                 present: np.ndarray, nthreads: int = 1) -> np.ndarray:
    nwin, _, stride = wins.shape
    S = np.ascontiguousarray(S, np.uint32)
    present = np.ascontiguousarray(present, np.uint64)
    status = np.zeros(nwin, np.uint8)
    lib().orc_decode_batch(scheme, k, r, _p(S), stride, nwin, _p(present), _p(status), _p(wins),
                           nthreads)
    return status


def erase(wins: np.ndarray, present: np.ndarray, k: int, r: int, fill: int = 0) -> None:
    """Overwrite every symbol whose present bit is clear (proves decode never reads it)."""
    for w in range(wins.shape[0]):
        p = int(present[w])
        for i in range(k + r):
            if not (p >> i) & 1:
                wins[w, i, :] = fill


def window_digest(k: int, r: int, S: int, win: np.ndarray) -> int:
    return lib().orc_window_digest(k, r, S, win.shape[-1], _p(np.ascontiguousarray(win)))


SIMD_NAMES = {0: "scalar", 1: "AVX2 vpshufb nibble tables", 2: "AVX2+GFNI vgf2p8affineqb"}


def simd_detect() -> int:
    """CPU baseline codec level this CPU supports (fec_cpu_simd.c)."""
    return lib().orc_simd_detect()


def simd_level() -> int:
    return lib().orc_simd_level()


def simd_set_level(level: int) -> None:
    lib().orc_simd_set_level(level)


def encode_batch_simd(scheme: int, k: int, r: int, S: np.ndarray, wins: np.ndarray, nthreads: int = 1):
    nwin, _, stride = wins.shape
    S = np.ascontiguousarray(S, np.uint32)
    lib().orc_encode_batch_simd(scheme, k, r, _p(S), stride, nwin, _p(wins), nthreads)


def decode_batch_simd(scheme: int, k: int, r: int, S: np.ndarray, wins: np.ndarray,
                      present: np.ndarray, nthreads: int = 1) -> np.ndarray:
    """present: [nwin] u64, or [nwin, ceil((k + r) / 64)] u64 words (k + r > 64)."""
    nwin, _, stride = wins.shape
    S = np.ascontiguousarray(S, np.uint32)
    present = np.ascontiguousarray(present, np.uint64)
    status = np.zeros(nwin, np.uint8)
    if present.ndim == 2:
        lib().orc_decode_batch_simd_w(scheme, k, r, _p(S), stride, nwin, present.shape[1], _p(present),
                                      _p(status), _p(wins), nthreads)
    else:
        lib().orc_decode_batch_simd(scheme, k, r, _p(S), stride, nwin, _p(present), _p(status),
                                    _p(wins), nthreads)
    return status


def batch_digest(k: int, r: int, S: np.ndarray, wins: np.ndarray, w0: int = 0) -> int:
    """XOR over windows of sm64(window_digest + global window id)."""
    d = 0
    for w in range(wins.shape[0]):
        d ^= sm64(window_digest(k, r, int(S[w]), wins[w]) + w0 + w)
    return d
