"""fecgpu — Python host layer over the MI355X FEC engine's C ABI (include/fecgpu.h).

The product path is libfecgpu.so (gfx950 HIP kernels + C++ runtime), loaded
in-tree from quic-fec-eps_amd/lib/.  There is no CPU fallback: if the library
is missing, importing this package raises; if no GPU is present, every compute
call raises FecError(FECGPU_ERR_DEVICE).

Reference interface mirrored: the fec branch's FEC encoder/decoder/frame API
(BASELINE.json north_star; branch not mounted, /root/reference/README.md:7),
restated as batch calls:
  encode_batch  — repair generation for many windows
  decode_batch  — erasure recovery in place
plus on-device workload synthesis, erasure streams and run digests used by
bench.py and the parity tests.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FECGPU_LIB") or os.path.join(os.path.dirname(_HERE), "lib",
                                                        "libfecgpu.so")

# enums of include/fecgpu.h
ERR_DONE, ERR_BUFFER_TOO_SHORT, ERR_INVALID_ARG = -1, -2, -3
ERR_UNSUPPORTED, ERR_DEVICE, ERR_UNRECOVERABLE, ERR_LIMIT = -4, -5, -6, -7
SCHEME_XOR, SCHEME_GF256 = 0, 1
MATRIX_CAUCHY, MATRIX_VANDERMONDE, MATRIX_RLC = 0, 1, 2
_MATRIX_IDS = {"cauchy": MATRIX_CAUCHY, "vandermonde": MATRIX_VANDERMONDE, "rlc": MATRIX_RLC}
FRAMING_FIXED, FRAMING_LENPREFIX = 0, 1
STATUS_OK, STATUS_UNRECOVERABLE = 0, 1
F_HOST_PTRS, F_SYNC = 1, 2
SW_ERR_HEADER, SW_ERR_CAPACITY, SW_ERR_INTERNAL = 1, 2, 4  # fecgpu_sw_decode_errors flags
MAX_K, MAX_R = 64, 8
WORKLOAD_FIXED, WORKLOAD_MIXED = 0, 1
ERASURE_NONE, ERASURE_EXACT, ERASURE_IID = 0, 1, 2

# every symbol include/fecgpu.h declares (tests check the library exports them)
EXPORTS = (
    "fecgpu_abi_version", "fecgpu_strerror", "fecgpu_last_error", "fecgpu_code_check",
    "fecgpu_code_parity_rows",
    "fecgpu_ctx_new", "fecgpu_ctx_free", "fecgpu_ctx_set_tuning",
    "fecgpu_host_alloc", "fecgpu_host_free",
    "fecgpu_encode_batch", "fecgpu_encode_split", "fecgpu_decode_batch",
    "fecgpu_synth_batch", "fecgpu_erasure_batch", "fecgpu_digest_batch",
    "fecgpu_encoder_new", "fecgpu_encoder_free", "fecgpu_encoder_add_source",
    "fecgpu_encoder_close_window", "fecgpu_encoder_flush", "fecgpu_encoder_repair",
    "fecgpu_encoder_release",
    "fecgpu_decoder_new", "fecgpu_decoder_free", "fecgpu_decoder_add_source",
    "fecgpu_decoder_add_repair", "fecgpu_decoder_flush", "fecgpu_decoder_flush_many",
    "fecgpu_encoder_flush_many",
    "fecgpu_decoder_recovered", "fecgpu_decoder_next_recovered",
    "fecgpu_decoder_release", "fecgpu_encoder_window_sources",
    "fecgpu_decoder_set_window_sources", "fecgpu_decoder_set_max_windows",
    "fecgpu_encoder_set_policy", "fecgpu_encoder_tick", "fecgpu_decoder_set_policy",
    "fecgpu_decoder_tick",
    "fecgpu_frame_source_id_len", "fecgpu_frame_write_source_id", "fecgpu_frame_repair_len",
    "fecgpu_frame_write_repair", "fecgpu_frame_write_repair_header", "fecgpu_frame_parse",
    "fecgpu_sw_encode", "fecgpu_sw_decode", "fecgpu_sw_decode_device", "fecgpu_sw_decode_errors",
    "fecgpu_frame_write_sw_source", "fecgpu_frame_write_sw_repair",
    "fecgpu_sw_encoder_new", "fecgpu_sw_encoder_free", "fecgpu_sw_encoder_add_source",
    "fecgpu_sw_encoder_flush", "fecgpu_sw_encoder_next_repair",
    "fecgpu_sw_decoder_new", "fecgpu_sw_decoder_free", "fecgpu_sw_decoder_add_source",
    "fecgpu_sw_decoder_add_repair", "fecgpu_sw_decoder_flush", "fecgpu_sw_decoder_recovered",
    "fecgpu_sw_decoder_next_recovered",
)
FRAME_SW_SOURCE, FRAME_SW_REPAIR = 0xFEC2, 0xFEC3
SW_MAX_WINDOW = 255
# fecgpu_sw_repair as a numpy dtype (16 bytes, the C layout)
SW_REPAIR_DTYPE = [("fss", "<u8"), ("nss", "<u2"), ("key", "<u2"), ("dt", "u1"), ("reserved", "u1", (3,))]
FRAME_SOURCE_ID, FRAME_REPAIR = 0xFEC0, 0xFEC4


class FecError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        msg = f"{what}: {_lib().fecgpu_strerror(code).decode()} ({code})"
        detail = _lib().fecgpu_last_error().decode()
        if code == ERR_DEVICE and detail:
            msg += f" [{detail}]"
        super().__init__(msg)


class fecgpu_code(ctypes.Structure):
    _fields_ = [
        ("scheme", ctypes.c_uint32),
        ("matrix", ctypes.c_uint32),
        ("framing", ctypes.c_uint32),
        ("k", ctypes.c_uint16),
        ("r", ctypes.c_uint16),
        ("poly", ctypes.c_uint32),
        ("rlc_key", ctypes.c_uint16),
        ("rlc_dt", ctypes.c_uint8),
        ("reserved", ctypes.c_uint8),
    ]


class fecgpu_frame(ctypes.Structure):
    _fields_ = [
        ("type", ctypes.c_uint64),
        ("win", ctypes.c_uint64),
        ("k", ctypes.c_uint16),
        ("r", ctypes.c_uint16),
        ("idx", ctypes.c_uint16),
        ("payload", ctypes.c_void_p),
        ("payload_len", ctypes.c_size_t),
        ("nsrc", ctypes.c_uint16),
        ("key", ctypes.c_uint16),
        ("dt", ctypes.c_uint8),
    ]


class fecgpu_sw_repair(ctypes.Structure):
    _fields_ = [("fss", ctypes.c_uint64), ("nss", ctypes.c_uint16), ("key", ctypes.c_uint16),
                ("dt", ctypes.c_uint8), ("reserved", ctypes.c_uint8 * 3)]


class fecgpu_sw_params(ctypes.Structure):
    _fields_ = [("framing", ctypes.c_uint32), ("symbol_size", ctypes.c_uint32), ("window", ctypes.c_uint16),
                ("step", ctypes.c_uint16), ("dt", ctypes.c_uint8), ("reserved", ctypes.c_uint8 * 3),
                ("batch", ctypes.c_uint32), ("span", ctypes.c_uint32)]


_L = None


class _Policy(ctypes.Structure):
    """fecgpu_policy (include/fecgpu.h)."""
    _fields_ = [("window_timeout_us", ctypes.c_uint64), ("batch_timeout_us", ctypes.c_uint64)]


def _lib():
    global _L
    if _L is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"libfecgpu.so not built at {LIB_PATH}: run `make -C quic-fec-eps_amd` "
                "or __graft_entry__.build() (no CPU fallback exists)")
        # One HIP runtime per process: torch's wheel bundles its own
        # libamdhip64 (NEEDED as "libamdhip64.so", SONAME libamdhip64.so.7).
        # Loading torch first makes libfecgpu's libamdhip64.so.7 dependency
        # resolve to that same runtime; loading libfecgpu first would pull in
        # /opt/rocm's copy and torch would then load a second one.
        try:
            import torch  # noqa: F401
        except ImportError:  # pragma: no cover - non-torch hosts use /opt/rocm's runtime
            pass
        L = ctypes.CDLL(LIB_PATH)
        vp, u32, u64, i32, sz = (ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int,
                                 ctypes.c_ssize_t)
        cp = vp  # const fecgpu_code * (byref of any fecgpu_code layout)
        sigs = {
            "fecgpu_abi_version": (i32, []),
            "fecgpu_strerror": (ctypes.c_char_p, [sz]),
            "fecgpu_last_error": (ctypes.c_char_p, []),
            "fecgpu_code_check": (sz, [cp]),
            "fecgpu_code_parity_rows": (sz, [cp, vp, ctypes.c_size_t]),
            "fecgpu_ctx_new": (sz, [vp, i32, ctypes.POINTER(vp)]),
            "fecgpu_ctx_free": (None, [vp]),
            "fecgpu_ctx_set_tuning": (sz, [vp, ctypes.c_char_p, ctypes.c_int64]),
            "fecgpu_host_alloc": (sz, [ctypes.c_size_t, ctypes.POINTER(vp)]),
            "fecgpu_host_free": (None, [vp]),
            "fecgpu_encode_batch": (sz, [vp, cp, vp, vp, vp, u32, u32, u64, u32, vp]),
            "fecgpu_encode_split": (sz, [vp, cp, vp, vp, vp, u32, u32, u64, u32, vp]),
            "fecgpu_decode_batch": (sz, [vp, cp, vp, vp, vp, u32, u32, u64, vp, vp, u32, vp]),
            "fecgpu_synth_batch": (sz, [vp, cp, i32, u64, u64, vp, vp, u32, u32, u64, vp]),
            "fecgpu_erasure_batch": (sz, [vp, cp, i32, u64, u64, vp, u64, vp]),
            "fecgpu_digest_batch": (sz, [vp, cp, vp, vp, u32, u32, u64, u64, vp, vp]),
            "fecgpu_encoder_new": (sz, [vp, cp, u32, u32, ctypes.POINTER(vp)]),
            "fecgpu_encoder_free": (None, [vp]),
            "fecgpu_encoder_add_source": (sz, [vp, vp, ctypes.c_size_t,
                                               ctypes.POINTER(ctypes.c_uint64),
                                               ctypes.POINTER(ctypes.c_uint16)]),
            "fecgpu_encoder_close_window": (sz, [vp]),
            "fecgpu_encoder_flush": (sz, [vp]),
            "fecgpu_encoder_repair": (sz, [vp, u64, ctypes.c_uint16, vp, ctypes.c_size_t]),
            "fecgpu_encoder_release": (sz, [vp, u64]),
            "fecgpu_decoder_new": (sz, [vp, cp, u32, u32, ctypes.POINTER(vp)]),
            "fecgpu_decoder_free": (None, [vp]),
            "fecgpu_decoder_add_source": (sz, [vp, u64, ctypes.c_uint16, vp, ctypes.c_size_t]),
            "fecgpu_decoder_add_repair": (sz, [vp, u64, ctypes.c_uint16, vp, ctypes.c_size_t]),
            "fecgpu_decoder_flush": (sz, [vp]),
            "fecgpu_decoder_flush_many": (sz, [ctypes.POINTER(vp), ctypes.c_size_t]),
            "fecgpu_encoder_flush_many": (sz, [ctypes.POINTER(vp), ctypes.c_size_t]),
            "fecgpu_decoder_recovered": (sz, [vp, u64, ctypes.c_uint16, vp, ctypes.c_size_t]),
            "fecgpu_decoder_release": (sz, [vp, u64]),
            "fecgpu_decoder_next_recovered": (sz, [vp, ctypes.POINTER(ctypes.c_uint64),
                                                   ctypes.POINTER(ctypes.c_uint16)]),
            "fecgpu_encoder_window_sources": (sz, [vp, u64]),
            "fecgpu_decoder_set_window_sources": (sz, [vp, u64, ctypes.c_uint16]),
            "fecgpu_decoder_set_max_windows": (sz, [vp, u64]),
            "fecgpu_encoder_set_policy": (sz, [vp, ctypes.POINTER(_Policy)]),
            "fecgpu_encoder_tick": (sz, [vp, u64]),
            "fecgpu_decoder_set_policy": (sz, [vp, ctypes.POINTER(_Policy)]),
            "fecgpu_decoder_tick": (sz, [vp, u64]),
            "fecgpu_frame_source_id_len": (sz, [u64, ctypes.c_uint16]),
            "fecgpu_frame_write_source_id": (sz, [vp, ctypes.c_size_t, u64, ctypes.c_uint16]),
            "fecgpu_frame_repair_len": (sz, [u64, ctypes.c_uint16, ctypes.c_uint16, ctypes.c_uint16,
                                             ctypes.c_uint16, ctypes.c_size_t]),
            "fecgpu_frame_write_repair": (sz, [vp, ctypes.c_size_t, u64, ctypes.c_uint16,
                                               ctypes.c_uint16, ctypes.c_uint16, ctypes.c_uint16, vp,
                                               ctypes.c_size_t]),
            "fecgpu_frame_write_repair_header": (sz, [vp, ctypes.c_size_t, u64, ctypes.c_uint16,
                                                      ctypes.c_uint16, ctypes.c_uint16, ctypes.c_uint16,
                                                      ctypes.c_size_t]),
            "fecgpu_frame_parse": (sz, [vp, ctypes.c_size_t, ctypes.POINTER(fecgpu_frame)]),
            "fecgpu_sw_encode": (sz, [vp, vp, u64, vp, vp, u64, u32, u32, u32, u32, vp]),
            "fecgpu_sw_decode": (sz, [vp, vp, vp, u64, vp, vp, vp, u64, u32, u32, vp, u32, vp]),
            "fecgpu_sw_decode_device": (sz, [vp, vp, vp, u64, vp, vp, vp, u64, u32, u32, vp, u32, vp]),
            "fecgpu_sw_decode_errors": (sz, [vp, ctypes.POINTER(ctypes.c_uint32)]),
            "fecgpu_frame_write_sw_source": (sz, [vp, ctypes.c_size_t, u64]),
            "fecgpu_frame_write_sw_repair": (sz, [vp, ctypes.c_size_t, ctypes.POINTER(fecgpu_sw_repair), vp,
                                                  ctypes.c_size_t]),
            "fecgpu_sw_encoder_new": (sz, [vp, ctypes.POINTER(fecgpu_sw_params), ctypes.POINTER(vp)]),
            "fecgpu_sw_encoder_free": (None, [vp]),
            "fecgpu_sw_encoder_add_source": (sz, [vp, vp, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint64)]),
            "fecgpu_sw_encoder_flush": (sz, [vp]),
            "fecgpu_sw_encoder_next_repair": (sz, [vp, ctypes.POINTER(fecgpu_sw_repair), vp, ctypes.c_size_t]),
            "fecgpu_sw_decoder_new": (sz, [vp, ctypes.POINTER(fecgpu_sw_params), ctypes.POINTER(vp)]),
            "fecgpu_sw_decoder_free": (None, [vp]),
            "fecgpu_sw_decoder_add_source": (sz, [vp, u64, vp, ctypes.c_size_t]),
            "fecgpu_sw_decoder_add_repair": (sz, [vp, ctypes.POINTER(fecgpu_sw_repair), vp, ctypes.c_size_t]),
            "fecgpu_sw_decoder_flush": (sz, [vp]),
            "fecgpu_sw_decoder_recovered": (sz, [vp, u64, vp, ctypes.c_size_t]),
            "fecgpu_sw_decoder_next_recovered": (sz, [vp, ctypes.POINTER(ctypes.c_uint64)]),
        }
        for name, (res, args) in sigs.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _L = L
    return _L


def lib():
    """The loaded ctypes library (raises ImportError if not built)."""
    return _lib()


_lib()  # fail loudly at import when the native library is missing


@dataclass(frozen=True)
class Code:
    """fecgpu_code: scheme 'xor' | 'gf256', k sources, r repairs per window;
    GF matrix 'cauchy' (default) | 'vandermonde' | 'rlc' (RFC 8681 random
    linear code: parity row i from repair_key rlc_key + i, density rlc_dt)."""
    scheme: str
    k: int
    r: int
    framing: str = "fixed"
    matrix: str = "cauchy"
    rlc_key: int = 0
    rlc_dt: int = 15

    @property
    def c(self) -> fecgpu_code:
        return fecgpu_code(SCHEME_XOR if self.scheme == "xor" else SCHEME_GF256,
                           _MATRIX_IDS[self.matrix],
                           FRAMING_FIXED if self.framing == "fixed" else FRAMING_LENPREFIX,
                           self.k, self.r, 0x11D, self.rlc_key, self.rlc_dt, 0)

    @property
    def scheme_id(self) -> int:
        return SCHEME_XOR if self.scheme == "xor" else SCHEME_GF256

    def check(self) -> int:
        return _lib().fecgpu_code_check(ctypes.byref(self.c))

    def parity_rows(self):
        """[r, k] u8 parity rows of the code (host only, fecgpu_code_parity_rows)."""
        import numpy as np
        out = np.zeros((self.r, self.k), np.uint8)
        _check(_lib().fecgpu_code_parity_rows(ctypes.byref(self.c), out.ctypes.data, out.size),
               "fecgpu_code_parity_rows")
        return out


def _check(rc: int, what: str) -> int:
    if rc < 0:
        raise FecError(rc, what)
    return rc


def _ptr(t) -> int | None:
    if t is None:
        return None
    if isinstance(t, int):
        return t
    if hasattr(t, "data_ptr"):
        return t.data_ptr()
    if hasattr(t, "ctypes"):  # numpy
        return t.ctypes.data
    raise TypeError(type(t))


def _stream(stream) -> int | None:
    if stream is None:
        try:
            import torch
            if torch.cuda.is_available():
                return torch.cuda.current_stream().cuda_stream
        except Exception:  # pragma: no cover
            pass
        return None
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


class Context:
    """fecgpu_ctx over the given devices (default: the current device)."""

    def __init__(self, devices=None):
        self._h = ctypes.c_void_p()
        if devices:
            arr = (ctypes.c_int * len(devices))(*devices)
            rc = _lib().fecgpu_ctx_new(ctypes.cast(arr, ctypes.c_void_p), len(devices),
                                       ctypes.byref(self._h))
        else:
            rc = _lib().fecgpu_ctx_new(None, 0, ctypes.byref(self._h))
        _check(rc, "fecgpu_ctx_new")
        # per-connection objects made from this ctx: the C ABI requires them freed
        # before the ctx, so close() frees whatever is still open first
        import weakref
        self._children = weakref.WeakSet()

    @property
    def handle(self):
        return self._h

    def set_tuning(self, key: str, value: int) -> None:
        _check(_lib().fecgpu_ctx_set_tuning(self._h, key.encode(), value), "fecgpu_ctx_set_tuning")

    def close(self):
        if self._h:
            for child in list(self._children):
                child.close()
            _lib().fecgpu_ctx_free(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------ batch ---
    def encode_batch(self, code: Code, win, *, nwin: int, stride: int, sym_len=None,
                     sym_len_all: int = 0, win_off=None, flags: int = 0, stream=None) -> int:
        return _check(_lib().fecgpu_encode_batch(
            self._h, ctypes.byref(code.c), _ptr(win), _ptr(win_off), _ptr(sym_len),
            sym_len_all, stride, nwin, flags, _stream(stream) if not flags & F_HOST_PTRS else None),
            "fecgpu_encode_batch")

    def encode_split(self, code: Code, src, repair, *, nwin: int, stride: int, sym_len=None,
                     sym_len_all: int = 0, flags: int = 0, stream=None) -> int:
        """Sources src[w][k][stride] -> repairs repair[w][r][stride] (device memory)."""
        return _check(_lib().fecgpu_encode_split(
            self._h, ctypes.byref(code.c), _ptr(src), _ptr(repair), _ptr(sym_len), sym_len_all,
            stride, nwin, flags, _stream(stream)), "fecgpu_encode_split")

    def decode_batch(self, code: Code, win, present, status, *, nwin: int, stride: int,
                     sym_len=None, sym_len_all: int = 0, win_off=None, flags: int = 0,
                     stream=None) -> int:
        return _check(_lib().fecgpu_decode_batch(
            self._h, ctypes.byref(code.c), _ptr(win), _ptr(win_off), _ptr(sym_len),
            sym_len_all, stride, nwin, _ptr(present), _ptr(status), flags,
            _stream(stream) if not flags & F_HOST_PTRS else None), "fecgpu_decode_batch")

    def sw_encode(self, src, rep, hdr, *, nsrc: int, nrep: int, sym_len: int, stride: int,
                  max_window: int = 0, flags: int = 0, stream=None) -> int:
        """Sliding-window RLC repairs (fecgpu_sw_encode): rep[t] from hdr[t]'s window of src."""
        return _check(_lib().fecgpu_sw_encode(
            self._h, _ptr(src), nsrc, _ptr(rep), _ptr(hdr), nrep, max_window, sym_len, stride, flags,
            _stream(stream) if not flags & F_HOST_PTRS else None), "fecgpu_sw_encode")

    def sw_decode(self, src, src_present, rep, rep_present, hdr, src_status, *, nsrc: int, nrep: int,
                  sym_len: int, stride: int, flags: int = 0, stream=None) -> int:
        """Sliding-window RLC recovery in place (fecgpu_sw_decode); src_present, rep_present,
        hdr and src_status are host (numpy) arrays.  Returns the number recovered."""
        return _check(_lib().fecgpu_sw_decode(
            self._h, _ptr(src), _ptr(src_present), nsrc, _ptr(rep), _ptr(rep_present), _ptr(hdr),
            nrep, sym_len, stride, _ptr(src_status), flags,
            _stream(stream) if not flags & F_HOST_PTRS else None), "fecgpu_sw_decode")

    def sw_decode_device(self, src, src_present, rep, rep_present, hdr, src_status, *, nsrc: int,
                         nrep: int, sym_len: int, stride: int, flags: int = 0, stream=None) -> int:
        """fecgpu_sw_decode_device: the same decode with the bookkeeping (flags, headers,
        statuses) in device memory too.  Asynchronous (returns 0) unless flags has F_SYNC,
        which returns the number recovered."""
        return _check(_lib().fecgpu_sw_decode_device(
            self._h, _ptr(src), _ptr(src_present), nsrc, _ptr(rep), _ptr(rep_present), _ptr(hdr),
            nrep, sym_len, stride, _ptr(src_status), flags, _stream(stream)), "fecgpu_sw_decode_device")

    def sw_decode_errors(self) -> int:
        """fecgpu_sw_decode_errors: the SW_ERR_* flags raised by asynchronous
        sw_decode_device calls on the current device since the last query (waits for
        them; clears the flags)."""
        f = ctypes.c_uint32(0)
        _check(_lib().fecgpu_sw_decode_errors(self._h, ctypes.byref(f)), "fecgpu_sw_decode_errors")
        return int(f.value)

    def synth_batch(self, code: Code, workload: int, seed: int, w0: int, win, sym_len, *,
                    L: int, stride: int, nwin: int, stream=None) -> int:
        return _check(_lib().fecgpu_synth_batch(
            self._h, ctypes.byref(code.c), workload, seed, w0, _ptr(win), _ptr(sym_len), L,
            stride, nwin, _stream(stream)), "fecgpu_synth_batch")

    def erasure_batch(self, code: Code, erasure: int, seed: int, w0: int, present, *, nwin: int,
                      stream=None) -> int:
        return _check(_lib().fecgpu_erasure_batch(
            self._h, ctypes.byref(code.c), erasure, seed, w0, _ptr(present), nwin,
            _stream(stream)), "fecgpu_erasure_batch")

    def digest_batch(self, code: Code, win, digest, *, nwin: int, stride: int, w0: int = 0,
                     sym_len=None, sym_len_all: int = 0, stream=None) -> int:
        return _check(_lib().fecgpu_digest_batch(
            self._h, ctypes.byref(code.c), _ptr(win), _ptr(sym_len), sym_len_all, stride, w0,
            nwin, _ptr(digest), _stream(stream)), "fecgpu_digest_batch")


class PinnedBuffer:
    """Page-locked host memory (fecgpu_host_alloc) viewed as a numpy uint8 array."""

    def __init__(self, nbytes: int):
        import numpy as np
        self._p = ctypes.c_void_p()
        _check(_lib().fecgpu_host_alloc(nbytes, ctypes.byref(self._p)), "fecgpu_host_alloc")
        buf = (ctypes.c_uint8 * nbytes).from_address(self._p.value)
        self.array = np.frombuffer(buf, dtype=np.uint8)
        self.nbytes = nbytes

    def close(self):
        if self._p:
            self.array = None
            _lib().fecgpu_host_free(self._p)
            self._p = ctypes.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class Encoder:
    """Per-connection sender (fecgpu_encoder_*): append packets, read repairs."""

    def __init__(self, ctx: Context, code: Code, max_len: int, batch: int = 64):
        self._ctx = ctx  # keep the ctx alive
        ctx._children.add(self)
        self.code = code
        self._h = ctypes.c_void_p()
        _check(_lib().fecgpu_encoder_new(ctx.handle, ctypes.byref(code.c), max_len, batch,
                                         ctypes.byref(self._h)), "fecgpu_encoder_new")

    def add_source(self, pkt: bytes) -> tuple[int, int]:
        w, i = ctypes.c_uint64(), ctypes.c_uint16()
        _check(_lib().fecgpu_encoder_add_source(self._h, pkt, len(pkt), ctypes.byref(w),
                                                ctypes.byref(i)), "fecgpu_encoder_add_source")
        return w.value, i.value

    def close_window(self) -> int:
        return _check(_lib().fecgpu_encoder_close_window(self._h), "fecgpu_encoder_close_window")

    def flush(self) -> int:
        return _check(_lib().fecgpu_encoder_flush(self._h), "fecgpu_encoder_flush")

    def repair(self, win: int, i: int, cap: int = 65538) -> bytes | None:
        buf = ctypes.create_string_buffer(cap)
        n = _lib().fecgpu_encoder_repair(self._h, win, i, buf, cap)
        if n == ERR_DONE:
            return None
        return buf.raw[:_check(n, "fecgpu_encoder_repair")]

    def release(self, win: int) -> int:
        return _lib().fecgpu_encoder_release(self._h, win)

    def window_sources(self, win: int) -> int | None:
        """Real sources of closed window `win` (the REPAIR frame's nsrc), None if unknown."""
        n = _lib().fecgpu_encoder_window_sources(self._h, win)
        return None if n == ERR_DONE else _check(n, "fecgpu_encoder_window_sources")

    def set_policy(self, window_timeout_us: int = 0, batch_timeout_us: int = 0) -> None:
        p = _Policy(window_timeout_us, batch_timeout_us)
        _check(_lib().fecgpu_encoder_set_policy(self._h, ctypes.byref(p)), "fecgpu_encoder_set_policy")

    def tick(self, now_us: int) -> int:
        """Windows launched by the policy at `now_us`."""
        return _check(_lib().fecgpu_encoder_tick(self._h, now_us), "fecgpu_encoder_tick")

    def close(self):
        if self._h:
            _lib().fecgpu_encoder_free(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class Decoder:
    """Per-connection receiver (fecgpu_decoder_*): file packets, read recovered ones."""

    def __init__(self, ctx: Context, code: Code, max_len: int, batch: int = 64):
        self._ctx = ctx
        ctx._children.add(self)
        self.code = code
        self._h = ctypes.c_void_p()
        _check(_lib().fecgpu_decoder_new(ctx.handle, ctypes.byref(code.c), max_len, batch,
                                         ctypes.byref(self._h)), "fecgpu_decoder_new")

    def add_source(self, win: int, idx: int, pkt: bytes) -> int:
        return _lib().fecgpu_decoder_add_source(self._h, win, idx, pkt, len(pkt))

    def add_repair(self, win: int, idx: int, sym: bytes) -> int:
        return _lib().fecgpu_decoder_add_repair(self._h, win, idx, sym, len(sym))

    def flush(self) -> int:
        return _check(_lib().fecgpu_decoder_flush(self._h), "fecgpu_decoder_flush")

    def recovered(self, win: int, idx: int, cap: int = 65536) -> bytes | None:
        buf = ctypes.create_string_buffer(cap)
        n = _lib().fecgpu_decoder_recovered(self._h, win, idx, buf, cap)
        if n == ERR_DONE:
            return None
        return buf.raw[:_check(n, "fecgpu_decoder_recovered")]

    def release(self, win: int) -> int:
        return _lib().fecgpu_decoder_release(self._h, win)

    def set_window_sources(self, win: int, nsrc: int) -> int:
        """A REPAIR frame's nsrc: sources nsrc..k-1 of `win` are padding, not losses."""
        return _lib().fecgpu_decoder_set_window_sources(self._h, win, nsrc)

    def set_max_windows(self, n: int) -> None:
        _check(_lib().fecgpu_decoder_set_max_windows(self._h, n), "fecgpu_decoder_set_max_windows")

    def next_recovered(self) -> tuple[int, int] | None:
        """(win, idx) of the oldest recovered packet not yet returned, or None."""
        w, i = ctypes.c_uint64(), ctypes.c_uint16()
        rc = _lib().fecgpu_decoder_next_recovered(self._h, ctypes.byref(w), ctypes.byref(i))
        if rc == ERR_DONE:
            return None
        _check(rc, "fecgpu_decoder_next_recovered")
        return w.value, i.value

    def drain_recovered(self) -> list[tuple[int, int]]:
        out = []
        while (x := self.next_recovered()) is not None:
            out.append(x)
        return out

    def set_policy(self, window_timeout_us: int = 0, batch_timeout_us: int = 0) -> None:
        p = _Policy(window_timeout_us, batch_timeout_us)
        _check(_lib().fecgpu_decoder_set_policy(self._h, ctypes.byref(p)), "fecgpu_decoder_set_policy")

    def tick(self, now_us: int) -> int:
        """Sources recovered by a policy flush at `now_us`."""
        return _check(_lib().fecgpu_decoder_tick(self._h, now_us), "fecgpu_decoder_tick")

    def close(self):
        if self._h:
            _lib().fecgpu_decoder_free(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


def sw_params(symbol_size: int, window: int, step: int, *, framing: str = "lenprefix", dt: int = 15,
              batch: int = 16, span: int = 0) -> fecgpu_sw_params:
    return fecgpu_sw_params(FRAMING_FIXED if framing == "fixed" else FRAMING_LENPREFIX, symbol_size, window,
                            step, dt, (ctypes.c_uint8 * 3)(), batch, span)


class SwEncoder:
    """Per-connection sliding-window sender (fecgpu_sw_encoder_*)."""

    def __init__(self, ctx: Context, params: fecgpu_sw_params):
        self._ctx = ctx
        ctx._children.add(self)
        self.params = params
        self._h = ctypes.c_void_p()
        _check(_lib().fecgpu_sw_encoder_new(ctx.handle, ctypes.byref(params), ctypes.byref(self._h)),
               "fecgpu_sw_encoder_new")

    def add_source(self, pkt: bytes) -> int:
        """-> the packet's ESI; raises FecError(ERR_LIMIT) while repairs wait to be read."""
        esi = ctypes.c_uint64()
        _check(_lib().fecgpu_sw_encoder_add_source(self._h, pkt, len(pkt), ctypes.byref(esi)),
               "fecgpu_sw_encoder_add_source")
        return esi.value

    def flush(self) -> int:
        return _check(_lib().fecgpu_sw_encoder_flush(self._h), "fecgpu_sw_encoder_flush")

    def next_repair(self):
        """-> ((fss, nss, key, dt), symbol bytes) or None."""
        h = fecgpu_sw_repair()
        buf = ctypes.create_string_buffer(self.params.symbol_size)
        n = _lib().fecgpu_sw_encoder_next_repair(self._h, ctypes.byref(h), buf, self.params.symbol_size)
        if n == ERR_DONE:
            return None
        _check(n, "fecgpu_sw_encoder_next_repair")
        return (h.fss, h.nss, h.key, h.dt), buf.raw[:n]

    def close(self):
        if self._h:
            _lib().fecgpu_sw_encoder_free(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class SwDecoder:
    """Per-connection sliding-window receiver (fecgpu_sw_decoder_*)."""

    def __init__(self, ctx: Context, params: fecgpu_sw_params):
        self._ctx = ctx
        ctx._children.add(self)
        self.params = params
        self._h = ctypes.c_void_p()
        _check(_lib().fecgpu_sw_decoder_new(ctx.handle, ctypes.byref(params), ctypes.byref(self._h)),
               "fecgpu_sw_decoder_new")

    def add_source(self, esi: int, pkt: bytes) -> int:
        return _lib().fecgpu_sw_decoder_add_source(self._h, esi, pkt, len(pkt))

    def add_repair(self, hdr, sym: bytes) -> int:
        fss, nss, key, dt = hdr
        h = fecgpu_sw_repair(fss, nss, key, dt)
        return _check(_lib().fecgpu_sw_decoder_add_repair(self._h, ctypes.byref(h), sym, len(sym)),
                      "fecgpu_sw_decoder_add_repair")

    def flush(self) -> int:
        return _check(_lib().fecgpu_sw_decoder_flush(self._h), "fecgpu_sw_decoder_flush")

    def recovered(self, esi: int) -> bytes | None:
        cap = self.params.symbol_size
        buf = ctypes.create_string_buffer(cap)
        n = _lib().fecgpu_sw_decoder_recovered(self._h, esi, buf, cap)
        if n == ERR_DONE:
            return None
        n = _check(n, "fecgpu_sw_decoder_recovered")
        return buf.raw[:n]

    def drain_recovered(self) -> list[int]:
        out, esi = [], ctypes.c_uint64()
        while _lib().fecgpu_sw_decoder_next_recovered(self._h, ctypes.byref(esi)) == 0:
            out.append(esi.value)
        return out

    def close(self):
        if self._h:
            _lib().fecgpu_sw_decoder_free(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


def frame_sw_source(esi: int) -> bytes:
    buf = ctypes.create_string_buffer(16)
    n = _check(_lib().fecgpu_frame_write_sw_source(buf, 16, esi), "fecgpu_frame_write_sw_source")
    return buf.raw[:n]


def frame_sw_repair(hdr, sym: bytes) -> bytes:
    fss, nss, key, dt = hdr
    h = fecgpu_sw_repair(fss, nss, key, dt)
    cap = len(sym) + 48
    buf = ctypes.create_string_buffer(cap)
    n = _check(_lib().fecgpu_frame_write_sw_repair(buf, cap, ctypes.byref(h), sym, len(sym)),
               "fecgpu_frame_write_sw_repair")
    return buf.raw[:n]


def encoder_flush_many(encs) -> int:
    """fecgpu_encoder_flush_many: encode every queued window of several encoders
    (same ctx, code, max_len) in one launch; returns the windows encoded."""
    arr = (ctypes.c_void_p * len(encs))(*[e._h.value for e in encs])
    return _check(_lib().fecgpu_encoder_flush_many(arr, len(encs)), "fecgpu_encoder_flush_many")


def decoder_flush_many(decs) -> int:
    """fecgpu_decoder_flush_many: flush several decoders (same ctx, code, max_len)
    in one launch; returns the sources recovered over all of them."""
    arr = (ctypes.c_void_p * len(decs))(*[d._h.value for d in decs])
    return _check(_lib().fecgpu_decoder_flush_many(arr, len(decs)), "fecgpu_decoder_flush_many")


def frame_source_id(win: int, idx: int) -> bytes:
    """SOURCE_ID frame bytes (fecgpu_frame_write_source_id)."""
    n = _check(_lib().fecgpu_frame_source_id_len(win, idx), "fecgpu_frame_source_id_len")
    buf = ctypes.create_string_buffer(n)
    m = _check(_lib().fecgpu_frame_write_source_id(buf, n, win, idx), "fecgpu_frame_write_source_id")
    return buf.raw[:m]


def frame_repair(win: int, k: int, r: int, idx: int, sym: bytes, nsrc: int | None = None) -> bytes:
    """REPAIR frame bytes (fecgpu_frame_write_repair); nsrc = the window's real
    sources (default k: a full window)."""
    ns = k if nsrc is None else nsrc
    n = _check(_lib().fecgpu_frame_repair_len(win, k, r, ns, idx, len(sym)), "fecgpu_frame_repair_len")
    buf = ctypes.create_string_buffer(n)
    m = _check(_lib().fecgpu_frame_write_repair(buf, n, win, k, r, ns, idx, sym, len(sym)),
               "fecgpu_frame_write_repair")
    return buf.raw[:m]


def frame_repair_header(win: int, k: int, r: int, idx: int, sym_len: int,
                        nsrc: int | None = None) -> bytes:
    """REPAIR frame header without the symbol bytes (fecgpu_frame_write_repair_header):
    header + symbol == frame_repair(...), so the symbol can be sent from its own buffer."""
    buf = ctypes.create_string_buffer(40)
    m = _check(_lib().fecgpu_frame_write_repair_header(buf, 40, win, k, r, k if nsrc is None else nsrc,
                                                       idx, sym_len),
               "fecgpu_frame_write_repair_header")
    return buf.raw[:m]


def frame_parse(data: bytes):
    """-> (consumed, dict) or raises FecError (fecgpu_frame_parse)."""
    f = fecgpu_frame()
    buf = ctypes.create_string_buffer(bytes(data), len(data))
    n = _check(_lib().fecgpu_frame_parse(buf, len(data), ctypes.byref(f)), "fecgpu_frame_parse")
    out = {"type": f.type, "win": f.win, "idx": f.idx}
    if f.type == FRAME_REPAIR:
        off = f.payload - ctypes.addressof(buf)
        out.update(k=f.k, r=f.r, nsrc=f.nsrc, payload=bytes(data[off:off + f.payload_len]))
    elif f.type == FRAME_SW_SOURCE:
        out.update(esi=f.win)
    elif f.type == FRAME_SW_REPAIR:
        off = f.payload - ctypes.addressof(buf)
        out.update(hdr=(f.win, f.nsrc, f.key, f.dt), payload=bytes(data[off:off + f.payload_len]))
    return n, out


def round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m
