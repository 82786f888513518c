"""Benchmark workloads of BASELINE.json configs 2-4 on device memory.

Everything here runs on the GPU through libfecgpu (synthesis, erasure masks,
encode, decode); torch only provides device memory, streams and the
post-run bookkeeping (byte counts, verification against a saved copy).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from . import (ERASURE_EXACT, ERASURE_IID, STATUS_OK, WORKLOAD_FIXED, WORKLOAD_MIXED, Code,
               Context, round_up)

SEED = 0x5EEDFEC0


@dataclass(frozen=True)
class Config:
    name: str
    scheme: str
    k: int
    r: int
    workload: int          # 0 fixed L, 1 mixed MTU (LENPREFIX)
    L: int
    nwin_per_gpu: int
    erasure: int
    erasure_desc: str
    host: bool = False     # windows live in pinned host memory (config 5: PCIe inclusive)
    matrix: str = "cauchy"  # GF parity rows: cauchy | vandermonde | rlc (bench.py --matrix)
    rlc_key: int = 0
    rlc_dt: int = 15
    window: int = 0        # scheme "sw": a repair after every k sources over the last `window`
    loss: float = 0.0      # scheme "sw": i.i.d. loss of sources and repairs

    @property
    def code(self) -> Code:
        return Code(self.scheme, self.k, self.r,
                    "fixed" if self.workload == WORKLOAD_FIXED else "lenprefix", self.matrix,
                    self.rlc_key, self.rlc_dt)

    @property
    def mds(self) -> bool:
        """Any e <= r erasures recoverable (every matrix but the random linear code)."""
        return self.scheme == "xor" or self.matrix != "rlc"

    @property
    def stride(self) -> int:
        return round_up(self.L if self.workload == WORKLOAD_FIXED else 9002, 16)


CONFIGS = {
    2: Config("cfg2-xor-k8r2-1200B-64k", "xor", 8, 2, WORKLOAD_FIXED, 1200, 65536, ERASURE_EXACT,
              "one source per XOR group (e=r=2)"),
    3: Config("cfg3-gf256-k16r4-1200B-256k", "gf256", 16, 4, WORKLOAD_FIXED, 1200, 262144,
              ERASURE_EXACT, "exactly r=4 sources per window"),
    4: Config("cfg4-gf256-k32r8-mixedMTU-1M/8", "gf256", 32, 8, WORKLOAD_MIXED, 0, 131072,
              ERASURE_IID, "i.i.d. p=0.1 over all k+r symbols"),
    5: Config("cfg5-stream-xor-k8r2-1200B-pinned-host", "xor", 8, 2, WORKLOAD_FIXED, 1200, 65536,
              ERASURE_EXACT, "one source per XOR group (e=r=2)", host=True),
    6: Config("cfg5gf-stream-gf256-k8r2-1200B-pinned-host", "gf256", 8, 2, WORKLOAD_FIXED, 1200,
              65536, ERASURE_EXACT, "exactly r=2 sources per window", host=True),
    # sliding-window RLC (RFC 8681, fecgpu_sw_*): 65,536 repairs per GPU, one every
    # k = 8 sources over the last 32, over 524,288 sources x 1200 B (one stream per rank)
    7: Config("cfg7-sw-rlc-W32-step8-1200B-512k", "sw", 8, 1, WORKLOAD_FIXED, 1200, 65536, ERASURE_IID,
              "i.i.d. p=0.02 over sources and repairs", matrix="rlc", window=32, loss=0.02),
}


def _bits(x: torch.Tensor, n: int) -> torch.Tensor:
    """[nwin] int64 masks -> [nwin, n] bool (bit i)."""
    sh = torch.arange(n, device=x.device, dtype=torch.int64)
    return ((x.unsqueeze(1) >> sh) & 1).bool()


@dataclass
class Batch:
    cfg: Config
    nwin: int
    win: torch.Tensor        # [nwin * (k+r) * stride] u8
    sym_len: torch.Tensor    # [nwin] int32 (u32)
    present: torch.Tensor    # [nwin] int64 (u64)
    status: torch.Tensor     # [nwin] u8

    @staticmethod
    def allocate(cfg: Config, nwin: int, dev) -> "Batch":
        n = cfg.k + cfg.r
        win = torch.zeros(nwin * n * cfg.stride, dtype=torch.uint8, device=dev)
        sym_len = torch.full((nwin,), cfg.L, dtype=torch.int32, device=dev)
        present = torch.zeros(nwin, dtype=torch.int64, device=dev)
        status = torch.zeros(nwin, dtype=torch.uint8, device=dev)
        return Batch(cfg, nwin, win, sym_len, present, status)

    @property
    def view(self) -> torch.Tensor:
        return self.win.view(self.nwin, self.cfg.k + self.cfg.r, self.cfg.stride)

    def _len_args(self):
        if self.cfg.workload == WORKLOAD_FIXED:
            return dict(sym_len=None, sym_len_all=self.cfg.L)
        return dict(sym_len=self.sym_len, sym_len_all=0)

    def synthesize(self, ctx: Context, w0: int) -> None:
        c = self.cfg
        ctx.synth_batch(c.code, c.workload, SEED, w0, self.win,
                        self.sym_len if c.workload == WORKLOAD_MIXED else None,
                        L=c.L, stride=c.stride, nwin=self.nwin)

    def make_erasures(self, ctx: Context, w0: int) -> None:
        c = self.cfg
        ctx.erasure_batch(c.code, c.erasure, SEED, w0, self.present, nwin=self.nwin)

    def encode(self, ctx: Context) -> None:
        c = self.cfg
        ctx.encode_batch(c.code, self.win, nwin=self.nwin, stride=c.stride, **self._len_args())

    def decode(self, ctx: Context) -> None:
        c = self.cfg
        ctx.decode_batch(c.code, self.win, self.present, self.status, nwin=self.nwin,
                         stride=c.stride, **self._len_args())

    # ---------------------------------------------------------- accounting ---
    def source_bytes(self) -> int:
        """Sum of packet lengths (no prefix, no padding)."""
        c = self.cfg
        if c.workload == WORKLOAD_FIXED:
            return self.nwin * c.k * c.L
        hdr = self.view[:, :c.k, :2].to(torch.int64)
        return int((hdr[..., 0] * 256 + hdr[..., 1]).sum().item())

    def expected_outputs(self):
        """Per window: sources the decoder recovers, symbols it reads, unrecoverable flag."""
        c = self.cfg
        pres = _bits(self.present, c.k + c.r)
        miss = ~pres[:, :c.k]
        if c.scheme == "xor":
            ne = torch.zeros(self.nwin, dtype=torch.int64, device=self.win.device)
            reads = torch.zeros_like(ne)
            bad = torch.zeros(self.nwin, dtype=torch.bool, device=self.win.device)
            for g in range(c.r):
                members = list(range(g, c.k, c.r))
                nm = miss[:, members].sum(1)
                rec = (nm == 1) & pres[:, c.k + g]
                ne += rec.long()
                reads += rec.long() * len(members)
                bad |= (nm >= 1) & ~rec
            return ne, reads, bad
        e = miss.sum(1)
        reps = pres[:, c.k:].sum(1)
        ok = (e <= reps) & (e > 0)
        ne = torch.where(ok, e, torch.zeros_like(e))
        reads = torch.where(ok, torch.full_like(e, c.k), torch.zeros_like(e))
        return ne, reads, e > reps

    def algorithmic_bytes(self) -> dict:
        """HBM bytes each kernel must move: encode (k+r)*S, decode (reads+writes)*S."""
        c = self.cfg
        S = self.sym_len.to(torch.int64)
        ne, reads, _ = self.expected_outputs()
        enc = int(((c.k + c.r) * S).sum().item())
        dec = int(((reads + ne) * S).sum().item())
        return {"encode": enc, "decode": dec}

    # --------------------------------------------------------- verification ---
    def digest(self, ctx: Context, w0: int) -> int:
        """Run digest of the encoded windows: sources and
        repairs, order- and shard-invariant (XOR over global window ids)."""
        c = self.cfg
        self.encode(ctx)
        d = torch.zeros(1, dtype=torch.int64, device=self.win.device)
        ctx.digest_batch(c.code, self.win, d, nwin=self.nwin, stride=c.stride, w0=w0,
                         **self._len_args())
        torch.cuda.synchronize()
        return int(d.item()) & (2**64 - 1)

    def verify(self, ctx: Context, w0: int, chunk: int = 8192) -> dict:
        """Poison every erased symbol, decode once, and compare each window's
        sources with a copy taken before poisoning (all on device)."""
        c = self.cfg
        self.encode(ctx)
        v = self.view
        saved = v[:, :c.k].clone()
        pres = _bits(self.present, c.k + c.r)
        for s in range(0, self.nwin, chunk):
            blk = v[s:s + chunk]
            blk[~pres[s:s + chunk]] = 0xAB
        self.decode(ctx)
        torch.cuda.synchronize()
        _, _, bad_expect = self.expected_outputs()
        ok_status = self.status == STATUS_OK
        mismatched = 0
        pos = torch.arange(c.stride, device=v.device, dtype=torch.int32)
        for s in range(0, self.nwin, chunk):
            # only the emitted bytes [0, S_w) of each symbol are part of the contract
            pad = pos[None, None, :] >= self.sym_len[s:s + chunk, None, None]
            eq = ((v[s:s + chunk, :c.k] == saved[s:s + chunk]) | pad).flatten(1).all(1)
            mismatched += int((ok_status[s:s + chunk] & ~eq).sum().item())
        unrec = int((~ok_status).sum().item())
        if c.mds:
            status_agree = bool(((~ok_status) == bad_expect).all().item())
            rank_deficient = 0
        else:  # RLC: every window an MDS code loses is lost, plus the rank-deficient ones
            status_agree = bool((~ok_status | ~bad_expect).all().item())
            rank_deficient = int((~ok_status & ~bad_expect).sum().item())
        del saved
        # restore the erased symbols so the buffer is reusable
        self.synthesize(ctx, w0)
        out = {"ok": mismatched == 0 and status_agree, "windows": self.nwin,
               "mismatched_ok_windows": mismatched, "unrecoverable": unrec,
               "status_matches_expected": status_agree}
        if not c.mds:
            out["rank_deficient"] = rank_deficient
        return out


@dataclass
class HostBatch:
    """Config 5: the windows live in pinned host memory and every call crosses
    PCIe through the library's chunked H2D / kernel / D2H pipeline
    (FECGPU_F_HOST_PTRS).  Same packets and erasures as the device batches."""
    cfg: Config
    nwin: int
    buf: object              # fecgpu.PinnedBuffer
    present: "np.ndarray"
    status: "np.ndarray"

    @staticmethod
    def allocate(cfg: Config, nwin: int, dev) -> "HostBatch":
        import numpy as np
        from . import PinnedBuffer
        buf = PinnedBuffer(nwin * (cfg.k + cfg.r) * cfg.stride)
        return HostBatch(cfg, nwin, buf, np.zeros(nwin, np.uint64), np.zeros(nwin, np.uint8))

    @property
    def view(self):
        return self.buf.array.reshape(self.nwin, self.cfg.k + self.cfg.r, self.cfg.stride)

    def synthesize(self, ctx: Context, w0: int, dev=None) -> None:
        d = Batch.allocate(self.cfg, self.nwin, dev or torch.device("cuda"))
        d.synthesize(ctx, w0)
        d.make_erasures(ctx, w0)
        self.buf.array[:] = d.win.cpu().numpy()
        self.present[:] = d.present.cpu().numpy().view("uint64")
        del d

    def make_erasures(self, ctx: Context, w0: int) -> None:
        pass  # drawn in synthesize()

    def encode(self, ctx: Context) -> None:
        from . import F_HOST_PTRS
        ctx.encode_batch(self.cfg.code, self.buf.array, nwin=self.nwin, stride=self.cfg.stride,
                         sym_len_all=self.cfg.L, flags=F_HOST_PTRS)

    def decode(self, ctx: Context) -> None:
        from . import F_HOST_PTRS
        ctx.decode_batch(self.cfg.code, self.buf.array, self.present, self.status, nwin=self.nwin,
                         stride=self.cfg.stride, sym_len_all=self.cfg.L, flags=F_HOST_PTRS)

    def source_bytes(self) -> int:
        return self.nwin * self.cfg.k * self.cfg.L

    def algorithmic_bytes(self) -> dict:
        """PCIe bytes each call must move: encode sends k source rows and returns
        r repair rows; decode needs the k present rows that solve the window
        (received sources + as many repairs as erasures) plus the mask, and
        returns the e recovered rows plus status.  (The pipeline sends whole
        windows, k + r rows, on the way in.)"""
        import numpy as np
        c, n = self.cfg, self.nwin
        kmask = np.uint64((1 << c.k) - 1)
        miss = (~self.present) & kmask
        e = int(sum(int(((miss >> np.uint64(j)) & np.uint64(1)).sum()) for j in range(c.k)))
        return {"encode": n * (c.k + c.r) * c.stride,
                "decode": n * (c.k * c.stride + 8 + 1) + e * c.stride}

    def pcie_bytes(self) -> dict:
        """Bytes per call in each PCIe direction (the link is full duplex, 63 GB/s
        each way): encode copies the k source rows up (2-D copy) and the r repair
        rows down; the zero-copy decode reads its k solving rows and the mask
        over the link and writes the e recovered rows and the status back."""
        import numpy as np
        c, n = self.cfg, self.nwin
        kmask = np.uint64((1 << c.k) - 1)
        miss = (~self.present) & kmask
        e = int(sum(int(((miss >> np.uint64(j)) & np.uint64(1)).sum()) for j in range(c.k)))
        return {"encode": {"h2d": n * c.k * c.stride, "d2h": n * c.r * c.stride},
                "decode": {"h2d": n * (c.k * c.stride + 8), "d2h": e * c.stride + n}}

    def verify(self, ctx: Context, w0: int) -> dict:
        import numpy as np
        c = self.cfg
        self.encode(ctx)
        v = self.view
        saved = v[:, :c.k].copy()
        for i in range(c.k + c.r):
            erased = ((self.present >> np.uint64(i)) & np.uint64(1)) == 0
            v[erased, i] = 0xAB
        self.decode(ctx)
        ok = self.status == STATUS_OK
        eq = (v[:, :c.k, :c.L] == saved[:, :, :c.L]).reshape(self.nwin, -1).all(1)
        mism = int((ok & ~eq).sum())
        v[:, :c.k] = saved
        return {"ok": mism == 0 and bool(ok.all()), "windows": self.nwin,
                "mismatched_ok_windows": mism, "unrecoverable": int((~ok).sum())}


@dataclass
class SwBatch:
    """Config 7: one sliding-window RLC stream per rank (RFC 8681 with m = 8):
    nsrc = nwin * k sources of L bytes resident in HBM, nwin repairs, a repair
    after every k sources over the last `window` (repair_key = its index, DT 15).
    One step = fecgpu_sw_encode of every repair, then the decode at the config's
    loss rate.  The receiver's bookkeeping (arrival flags, headers, statuses) is
    kept on the device and the decode is planned there too
    (fecgpu_sw_decode_device, asynchronous like the encode); `host_meta` uses
    fecgpu_sw_decode instead (flags and headers copied up, statuses down, one
    synchronous call)."""
    cfg: Config
    nsrc: int
    nrep: int
    src: torch.Tensor        # [nsrc, stride] u8
    rep: torch.Tensor        # [nrep, stride] u8
    hdr: "np.ndarray"        # SW_REPAIR_DTYPE [nrep]
    d_hdr: torch.Tensor      # the headers on the device
    sp: "np.ndarray"         # source arrived flags
    rp: "np.ndarray"         # repair arrived flags
    st: "np.ndarray"         # per-source status of the last decode
    d_sp: torch.Tensor = None  # the flags and statuses on the device
    d_rp: torch.Tensor = None
    d_st: torch.Tensor = None
    host_meta: bool = False

    @staticmethod
    def allocate(cfg: Config, nwin: int, dev) -> "SwBatch":
        import numpy as np
        from . import SW_REPAIR_DTYPE
        nsrc, stride = nwin * cfg.k, cfg.stride
        hdr = np.zeros(nwin, SW_REPAIR_DTYPE)
        end = (np.arange(nwin, dtype=np.int64) + 1) * cfg.k
        fss = np.maximum(0, end - cfg.window)
        hdr["fss"], hdr["nss"], hdr["key"], hdr["dt"] = fss, end - fss, np.arange(nwin) & 0xFFFF, 15
        return SwBatch(cfg, nsrc, nwin, torch.zeros((nsrc, stride), dtype=torch.uint8, device=dev),
                       torch.zeros((nwin, stride), dtype=torch.uint8, device=dev), hdr,
                       torch.from_numpy(hdr.view(np.uint8).copy()).to(dev),
                       np.ones(nsrc, np.uint8), np.ones(nwin, np.uint8), np.zeros(nsrc, np.uint8))

    def synthesize(self, ctx: Context, w0: int) -> None:
        g = torch.Generator(device=self.src.device).manual_seed(SEED ^ w0)
        self.src[:, :self.cfg.L] = torch.randint(0, 256, (self.nsrc, self.cfg.L), dtype=torch.uint8,
                                                 device=self.src.device, generator=g)

    def make_erasures(self, ctx: Context, w0: int) -> None:
        import numpy as np
        rng = np.random.default_rng(SEED + w0)
        self.sp[:] = rng.random(self.nsrc) >= self.cfg.loss
        self.rp[:] = rng.random(self.nrep) >= self.cfg.loss
        dev = self.src.device
        self.d_sp = torch.from_numpy(self.sp).to(dev)
        self.d_rp = torch.from_numpy(self.rp).to(dev)
        self.d_st = torch.zeros(self.nsrc, dtype=torch.uint8, device=dev)

    def encode(self, ctx: Context) -> None:
        c = self.cfg
        ctx.sw_encode(self.src, self.rep, self.d_hdr, nsrc=self.nsrc, nrep=self.nrep, sym_len=c.L,
                      stride=c.stride, max_window=c.window)

    def decode(self, ctx: Context, sync: bool = False) -> int:
        """Asynchronous (returns 0) unless `sync` or host_meta: then the number recovered,
        with self.st holding the statuses."""
        from . import F_SYNC
        c = self.cfg
        if self.host_meta:
            return ctx.sw_decode(self.src, self.sp, self.rep, self.rp, self.hdr, self.st, nsrc=self.nsrc,
                                 nrep=self.nrep, sym_len=c.L, stride=c.stride)
        n = ctx.sw_decode_device(self.src, self.d_sp, self.rep, self.d_rp, self.d_hdr, self.d_st,
                                 nsrc=self.nsrc, nrep=self.nrep, sym_len=c.L, stride=c.stride,
                                 flags=F_SYNC if sync else 0)
        if sync:
            self.st[:] = self.d_st.cpu().numpy()
        return n

    def source_bytes(self) -> int:
        return self.nsrc * self.cfg.L

    def algorithmic_bytes(self) -> dict:
        """encode: every source read once and every repair written, (nsrc + nrep) * L
        (a source sits in window / k windows; the re-reads are the kernel's, not the
        algorithm's).  decode: per recovered source one equation, i.e. its repair's
        window read (window + 1 rows: the sources and the repair) and the source
        written, (window + 2) * L each."""
        c = self.cfg
        lost = int((self.sp == 0).sum())
        return {"encode": (self.nsrc + self.nrep) * c.L, "decode": lost * (c.window + 2) * c.L}

    def digest(self, ctx: Context, w0: int) -> int:
        """Checksum of the repairs (sum of their 8-byte words mod 2^64)."""
        self.encode(ctx)
        torch.cuda.synchronize()
        return int(self.rep[:, :self.cfg.stride // 8 * 8].contiguous().view(torch.int64).sum().item()) & (2**64 - 1)

    def verify(self, ctx: Context, w0: int) -> dict:
        """Poison the lost sources, decode once, compare every source reported
        recovered with the copy taken before; then restore the stream."""
        import numpy as np
        c = self.cfg
        self.encode(ctx)
        saved = self.src.clone()
        lost = torch.from_numpy(self.sp == 0).to(self.src.device)
        self.src[lost] = 0xAB
        n = self.decode(ctx, sync=True)
        torch.cuda.synchronize()
        ok = torch.from_numpy(self.st == STATUS_OK).to(self.src.device)
        mism = int((ok & ~(self.src[:, :c.L] == saved[:, :c.L]).all(1)).sum().item())
        nlost = int(lost.sum().item())
        unrec = int((self.st != STATUS_OK).sum())
        self.src.copy_(saved)
        return {"ok": mism == 0 and n + unrec == nlost, "sources": self.nsrc, "lost": nlost, "recovered": n,
                "unrecovered": unrec, "mismatched_recovered": mism}


@dataclass
class WideBatch:
    """GF(2^8) block codes with k + r > 64 (fec_wide.hip; bench.py --k/--r):
    nwin windows of k + r symbols of L bytes in HBM, sources seeded random bytes
    (torch generator on the device), exactly r sources erased per window (the
    decode's worst case: e = r), present masks of ceil((k + r) / 64) words."""
    cfg: Config
    nwin: int
    win: torch.Tensor        # [nwin, k + r, stride] u8
    present: torch.Tensor    # [nwin, words] int64 (u64)
    status: torch.Tensor     # [nwin] u8
    erased: torch.Tensor     # [nwin, k + r] bool

    @staticmethod
    def allocate(cfg: Config, nwin: int, dev) -> "WideBatch":
        n = cfg.k + cfg.r
        words = (n + 63) // 64
        return WideBatch(cfg, nwin, torch.zeros((nwin, n, cfg.stride), dtype=torch.uint8, device=dev),
                         torch.zeros((nwin, words), dtype=torch.int64, device=dev),
                         torch.zeros(nwin, dtype=torch.uint8, device=dev),
                         torch.zeros((nwin, n), dtype=torch.bool, device=dev))

    def synthesize(self, ctx: Context, w0: int) -> None:
        c = self.cfg
        g = torch.Generator(device=self.win.device).manual_seed(SEED ^ w0)
        self.win[:, :c.k, :c.L] = torch.randint(0, 256, (self.nwin, c.k, c.L), dtype=torch.uint8,
                                                device=self.win.device, generator=g)

    def make_erasures(self, ctx: Context, w0: int) -> None:
        c = self.cfg
        g = torch.Generator(device=self.win.device).manual_seed(SEED + 1 + w0)
        key = torch.rand((self.nwin, c.k), device=self.win.device, generator=g)
        miss = key.argsort(dim=1)[:, :c.r]  # r distinct sources per window
        self.erased.zero_()
        self.erased.scatter_(1, miss, True)
        n = c.k + c.r
        pres = ~self.erased
        words = self.present.shape[1]
        self.present.zero_()
        sh = torch.arange(64, device=self.win.device, dtype=torch.int64)
        for wd in range(words):
            bits = pres[:, wd * 64:min(n, wd * 64 + 64)].to(torch.int64)
            self.present[:, wd] = (bits << sh[:bits.shape[1]]).sum(1)

    def encode(self, ctx: Context) -> None:
        c = self.cfg
        ctx.encode_batch(c.code, self.win, nwin=self.nwin, stride=c.stride, sym_len_all=c.L)

    def decode(self, ctx: Context) -> None:
        c = self.cfg
        ctx.decode_batch(c.code, self.win, self.present, self.status, nwin=self.nwin, stride=c.stride,
                         sym_len_all=c.L)

    def source_bytes(self) -> int:
        return self.nwin * self.cfg.k * self.cfg.L

    def algorithmic_bytes(self) -> dict:
        """encode (k + r) * L per window; decode: k rows read (k - r received
        sources and the r repairs) and r written, (k + r) * L."""
        c = self.cfg
        return {"encode": self.nwin * (c.k + c.r) * c.L, "decode": self.nwin * (c.k + c.r) * c.L}

    def digest(self, ctx: Context, w0: int) -> int:
        """Checksum of the encoded windows (sum of their 8-byte words mod 2^64)."""
        self.encode(ctx)
        torch.cuda.synchronize()
        return int(self.win.view(torch.int64).sum().item()) & (2**64 - 1)

    def verify(self, ctx: Context, w0: int, chunk: int = 2048) -> dict:
        c = self.cfg
        self.encode(ctx)
        saved = self.win[:, :c.k].clone()
        self.win[self.erased] = 0xAB
        self.decode(ctx)
        torch.cuda.synchronize()
        ok = self.status == STATUS_OK
        mism = 0
        for s0 in range(0, self.nwin, chunk):
            eq = (self.win[s0:s0 + chunk, :c.k, :c.L] == saved[s0:s0 + chunk, :, :c.L]).flatten(1).all(1)
            mism += int((ok[s0:s0 + chunk] & ~eq).sum().item())
        unrec = int((~ok).sum().item())
        self.win[:, :c.k] = saved
        del saved
        # every window has exactly r erasures: an MDS code recovers all of them
        return {"ok": mism == 0 and (unrec == 0 or not c.mds), "windows": self.nwin,
                "mismatched_ok_windows": mism, "unrecoverable": unrec}
