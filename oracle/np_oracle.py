"""Independent numpy restatement of the coding contract — TEST INFRASTRUCTURE ONLY.

Written separately from fec_oracle.c (different derivations on purpose):
  * field multiply by carry-less shift-and-add with reduction by 0x11D
    (no log/exp tables), inverse by exhaustive search;
  * encode as a vectorised matrix product through a 256x256 product table;
  * decode by solving the full (k+r) x k generator system restricted to the
    received rows with Gauss-Jordan on the augmented byte matrix.
Used to cross-check the C oracle and to generate tests/golden/ fixtures
(tests/golden/make_golden.py).  PARITY UNPINNED: the
reference fec branch is not mounted (/root/reference/README.md:7 is a URL).
Contract clauses: SURVEY.md Appendix A.1-A.6, DESIGN.md §Workloads.
"""
from __future__ import annotations

import numpy as np

M64 = (1 << 64) - 1
POLY = 0x11D


def clmul_mod(a: int, b: int) -> int:
    """A.1: a*b in GF(2^8)/0x11D by shift-and-add."""
    p = 0
    for _ in range(8):
        if b & 1:
            p ^= a
        b >>= 1
        a <<= 1
        if a & 0x100:
            a ^= POLY
    return p


_MUL = np.array([[clmul_mod(a, b) for b in range(256)] for a in range(256)], np.uint8)
_INV = np.zeros(256, np.uint8)
for _a in range(1, 256):
    _INV[_a] = int(np.nonzero(_MUL[_a] == 1)[0][0])


def mul_table() -> np.ndarray:
    return _MUL


def inv(a: int) -> int:
    return int(_INV[a])


def cauchy(k: int, r: int) -> np.ndarray:
    """A.2: C[i][j] = inv((k+i) ^ j)."""
    return np.array([[_INV[(k + i) ^ j] for j in range(k)] for i in range(r)], np.uint8)


def _gj_inverse(A: np.ndarray) -> np.ndarray:
    """Gauss-Jordan inverse over GF(2^8) (row pivoting) through the product table."""
    n = A.shape[0]
    M = np.concatenate([A.astype(np.uint8), np.eye(n, dtype=np.uint8)], axis=1)
    for c in range(n):
        piv = next(i for i in range(c, n) if M[i, c])
        M[[c, piv]] = M[[piv, c]]
        M[c] = _MUL[_INV[M[c, c]]][M[c]]
        for i in range(n):
            if i != c and M[i, c]:
                M[i] ^= _MUL[M[i, c]][M[c]]
    return M[:, n:].copy()


def vandermonde(k: int, r: int) -> np.ndarray:
    """Systematic Vandermonde parity rows: V[i][j] = i^j (i < k+r, powers by
    repeated table multiplication, 0^0 = 1) times inv(V[:k]); rows k.. (the
    Backblaze JavaReedSolomon / klauspost / reed-solomon-erasure matrix)."""
    V = np.zeros((k + r, k), np.uint8)
    for i in range(k + r):
        x = 1
        for j in range(k):
            V[i, j] = x
            x = int(_MUL[x][i])
    return matmul(V[k:], _gj_inverse(V[:k]))


class TinyMT32:
    """RFC 8682 TinyMT32 (mat1 0x8f7011ee, mat2 0xfc78ff1f, tmat 0x3793fdff),
    restated in Python from the RFC's description: 127-bit state of four
    words, 8 pre-loop steps after seeding, tempered output."""
    MAT1, MAT2, TMAT = 0x8F7011EE, 0xFC78FF1F, 0x3793FDFF

    def __init__(self, seed: int):
        st = [seed & 0xFFFFFFFF, self.MAT1, self.MAT2, self.TMAT]
        for i in range(1, 8):
            prev = st[(i - 1) & 3]
            st[i & 3] ^= (i + 1812433253 * (prev ^ (prev >> 30))) & 0xFFFFFFFF
        if (st[0] & 0x7FFFFFFF) == 0 and st[1] == st[2] == st[3] == 0:
            st = [ord(c) for c in "TINY"]
        self.st = st
        for _ in range(8):
            self._next()

    def _next(self):
        s0, s1, s2, s3 = self.st
        x = (s0 & 0x7FFFFFFF) ^ s1 ^ s2
        x = (x ^ (x << 1)) & 0xFFFFFFFF
        y = s3 ^ (s3 >> 1) ^ x
        n1, n2 = s2, (x ^ (y << 10)) & 0xFFFFFFFF
        if y & 1:
            n1 ^= self.MAT1
            n2 ^= self.MAT2
        self.st = [s1, n1, n2, y]

    def u32(self) -> int:
        self._next()
        s0, _, s2, s3 = self.st
        t1 = (s0 + (s2 >> 8)) & 0xFFFFFFFF
        return (s3 ^ t1 ^ (self.TMAT if t1 & 1 else 0)) & 0xFFFFFFFF


def rlc_coefs(key: int, n: int, dt: int) -> np.ndarray:
    """RFC 8681 §3.6 generate_coding_coefficients(repair_key, n, dt, m = 8)."""
    assert 0 <= dt <= 15
    t = TinyMT32(key & 0xFFFF)
    cc = np.zeros(n, np.uint8)
    for i in range(n):
        if dt == 15 or (t.u32() & 0xF) <= dt:
            c = 0
            while c == 0:
                c = t.u32() & 0xFF
            cc[i] = c
    return cc


def parse_rlc(scheme: str):
    """"rlc:KEY:DT" -> (key, dt), else None."""
    if not scheme.startswith("rlc:"):
        return None
    _, key, dt = scheme.split(":")
    return int(key), int(dt)


def scheme_id(scheme: str) -> int:
    """The C oracle's scheme integer (fec_oracle.h, ORC_RLC for RLC)."""
    rl = parse_rlc(scheme)
    if rl:
        return 3 | (rl[1] << 4) | (rl[0] << 8)
    return {"xor": 0, "gf": 1, "gf-vdm": 2}[scheme]


def generator(scheme: str, k: int, r: int) -> np.ndarray:
    """Systematic (k+r) x k generator: identity on top, repair rows below.
    scheme: "xor", "gf" (Cauchy rows), "gf-vdm" (systematic Vandermonde) or
    "rlc:KEY:DT" (RFC 8681 coefficients, row i from repair_key KEY + i)."""
    G = np.zeros((k + r, k), np.uint8)
    G[:k] = np.eye(k, dtype=np.uint8)
    rl = parse_rlc(scheme)
    if scheme == "xor":
        for g in range(r):
            G[k + g, g::r] = 1
    elif rl:
        for i in range(r):
            G[k + i] = rlc_coefs(rl[0] + i, k, rl[1])
    elif scheme == "gf-vdm":
        G[k:] = vandermonde(k, r)
    else:
        G[k:] = cauchy(k, r)
    return G


def matmul(A: np.ndarray, X: np.ndarray) -> np.ndarray:
    """GF(2^8) product A (m x n) times X (n x L)."""
    out = np.zeros((A.shape[0], X.shape[1]), np.uint8)
    for i in range(A.shape[0]):
        acc = np.zeros(X.shape[1], np.uint8)
        for j in range(A.shape[1]):
            if A[i, j]:
                acc ^= _MUL[A[i, j]][X[j]]
        out[i] = acc
    return out


def encode(scheme: str, k: int, r: int, src: np.ndarray) -> np.ndarray:
    """src [k, L] -> repairs [r, L]."""
    return matmul(generator(scheme, k, r)[k:], src)


def decode(scheme: str, k: int, r: int, sym: np.ndarray, present: int):
    """sym [k+r, L] with garbage in erased rows -> (sources [k, L], ok).

    GF: solve G[rows] x = sym[rows] over k unknowns by Gauss-Jordan on the
    augmented matrix, using received sources plus the first e received repairs.
    XOR: per group (A.2), one missing member and its repair present.
    """
    L = sym.shape[1]
    src = sym[:k].copy()
    missing = [j for j in range(k) if not (present >> j) & 1]
    if not missing:
        return src, True
    if scheme == "xor":
        ok = True
        for g in range(r):
            grp = list(range(g, k, r))
            miss = [j for j in grp if j in missing]
            if not miss:
                continue
            if len(miss) > 1 or not (present >> (k + g)) & 1:
                ok = False
                continue
            acc = sym[k + g].copy()
            for j in grp:
                if j != miss[0]:
                    acc ^= sym[j]
            src[miss[0]] = acc
        return src, ok
    reps = [k + i for i in range(r) if (present >> (k + i)) & 1]
    if len(reps) < len(missing):
        return src, False
    if parse_rlc(scheme):
        return _solve_all_rows(generator(scheme, k, r), sym, present, k, r)
    rows = [j for j in range(k) if (present >> j) & 1] + reps[: len(missing)]
    G = generator(scheme, k, r)
    A = np.concatenate([G[rows], sym[rows]], axis=1).astype(np.uint8)  # k x (k+L)
    n = k
    for c in range(n):
        piv = next(i for i in range(c, n) if A[i, c])
        A[[c, piv]] = A[[piv, c]]
        A[c] = _MUL[_INV[A[c, c]]][A[c]]
        for i in range(n):
            if i != c and A[i, c]:
                A[i] ^= _MUL[A[i, c]][A[c]]
    return A[:, k:k + L].copy(), True


def _solve_all_rows(G: np.ndarray, sym: np.ndarray, present: int, k: int, r: int):
    """Random linear code (not MDS): Gaussian elimination of EVERY received row
    of the generator (sources and repairs) against the k unknowns; recoverable
    iff that system has rank k.  Row-echelon with pivot search over all rows,
    then back substitution."""
    L = sym.shape[1]
    rows = [i for i in range(k + r) if (present >> i) & 1]
    A = np.concatenate([G[rows], sym[rows]], axis=1).astype(np.uint8)
    m, piv_rows = A.shape[0], []
    for c in range(k):
        piv = next((i for i in range(len(piv_rows), m) if A[i, c]), None)
        if piv is None:
            return sym[:k].copy(), False
        t = len(piv_rows)
        A[[t, piv]] = A[[piv, t]]
        A[t] = _MUL[_INV[A[t, c]]][A[t]]
        for i in range(m):
            if i != t and A[i, c]:
                A[i] ^= _MUL[A[i, c]][A[t]]
        piv_rows.append(t)
    return A[:k, k:k + L].copy(), True


# ------------------------------------------------------------ workloads ---
TAG_PAY = 0x5041594C4F414400
TAG_MTU = 0x4D54550000000000
TAG_LEN = 0x4C454E0000000000
TAG_ERA = 0x4552415345000000
P10 = 429496730


def sm64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M64
    return x ^ (x >> 31)


def sm64_np(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64) + np.uint64(0x9E3779B97F4A7C15)
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def pkt_len(workload: int, seed: int, w: int, j: int, L: int) -> int:
    if workload == 0:
        return L
    mtu = 9000 if sm64((sm64(seed ^ TAG_MTU) + w) & M64) & 1 else 1200
    h = sm64((sm64(seed ^ TAG_LEN) + ((w << 8) | j)) & M64)
    if (h & 0xFFFFFFFF) < P10:
        return 64 + (h >> 32) % (mtu - 63)
    return mtu


def payload(seed: int, w: int, j: int, n: int) -> np.ndarray:
    spay = sm64(seed ^ TAG_PAY)
    words = np.arange((n + 7) // 8, dtype=np.uint64) + np.uint64(((w << 24) | (j << 16)) & M64)
    with np.errstate(over="ignore"):
        hw = sm64_np(words + np.uint64(spay))
    return hw.view(np.uint8)[:n].copy()  # little-endian host


def window(workload: int, seed: int, w: int, k: int, L: int):
    """-> (list of k packets, S, symbols [k, S])"""
    pkts = [payload(seed, w, j, pkt_len(workload, seed, w, j, L)) for j in range(k)]
    if workload == 0:
        S = L
        return pkts, S, np.stack(pkts)
    S = 2 + max(len(p) for p in pkts)
    sym = np.zeros((k, S), np.uint8)
    for j, p in enumerate(pkts):
        sym[j, 0], sym[j, 1] = len(p) >> 8, len(p) & 0xFF
        sym[j, 2:2 + len(p)] = p
    return pkts, S, sym


def present(erasure: int, seed: int, w: int, scheme: str, k: int, r: int) -> int:
    allm = (1 << (k + r)) - 1
    sera = sm64(seed ^ TAG_ERA)
    if erasure == 0:
        return allm
    p = allm
    if erasure == 2:
        for i in range(k + r):
            if (sm64((sera + ((w << 8) | i)) & M64) & 0xFFFFFFFF) < P10:
                p &= ~(1 << i)
        return p
    if scheme != "xor":
        perm = list(range(k))
        for t in range(min(r, k)):
            u = t + sm64((sera + ((w << 8) | t)) & M64) % (k - t)
            perm[t], perm[u] = perm[u], perm[t]
            p &= ~(1 << perm[t])
        return p
    for g in range(r):
        n = (k - g + r - 1) // r
        if n <= 0:
            continue
        idx = sm64((sera + ((w << 8) | g)) & M64) % n
        p &= ~(1 << (g + idx * r))
    return p


def deframe(sym: np.ndarray) -> np.ndarray:
    """a9: LENPREFIX symbol -> packet payload."""
    n = (int(sym[0]) << 8) | int(sym[1])
    return sym[2:2 + n]


# ------------------------------------------------- sliding-window RLC ---
def sw_encode(src: np.ndarray, hdr) -> np.ndarray:
    """RFC 8681 sliding-window repairs: rep[t] = sum_j cc_t[j] * src[fss_t + j]
    (hdr: iterable of (fss, nss, key, dt)); src [nsrc, L]."""
    reps = []
    for fss, nss, key, dt in hdr:
        cc = rlc_coefs(key, nss, dt)
        reps.append(matmul(cc[None, :], src[fss:fss + nss])[0])
    return np.array(reps, np.uint8).reshape(len(reps), src.shape[1])


def sw_decode(src: np.ndarray, src_present, rep: np.ndarray, rep_present, hdr):
    """Recover what the received repairs determine, by elimination of the data
    itself: rows [A | s] with s = rep + known-source terms (A: coefficients of
    the lost sources), reduced to row echelon form with pivot search; a lost
    source is determined iff its pivot row is zero on every free column.
    -> (sources [nsrc, L], status per source: 0 present/recovered, 1 lost)."""
    src = src.copy()
    nsrc, L = src.shape
    lost = [i for i in range(nsrc) if not src_present[i]]
    col = {s: c for c, s in enumerate(lost)}
    status = np.array([0 if src_present[i] else 1 for i in range(nsrc)], np.uint8)
    e = len(lost)
    rows = []
    for t, (fss, nss, key, dt) in enumerate(hdr):
        if not rep_present[t] or not any((fss + j) in col for j in range(nss)):
            continue
        cc = rlc_coefs(key, nss, dt)
        a = np.zeros(e, np.uint8)
        s = rep[t].copy()
        for j in range(nss):
            i = fss + j
            if i in col:
                a[col[i]] = cc[j]
            elif cc[j]:
                s ^= _MUL[cc[j]][src[i]]
        rows.append(np.concatenate([a, s]))
    if not rows or e == 0:
        return src, status
    M = np.array(rows, np.uint8)
    pivots, r = {}, 0
    for c in range(e):
        piv = next((i for i in range(r, len(M)) if M[i, c]), None)
        if piv is None:
            continue
        M[[r, piv]] = M[[piv, r]]
        M[r] = _MUL[_INV[M[r, c]]][M[r]]
        for i in range(len(M)):
            if i != r and M[i, c]:
                M[i] ^= _MUL[M[i, c]][M[r]]
        pivots[c] = r
        r += 1
    free = [c for c in range(e) if c not in pivots]
    for c, pr in pivots.items():
        if all(M[pr, f] == 0 for f in free):
            src[lost[c]] = M[pr, e:]
            status[lost[c]] = 0
    return src, status


def sw_schedule(nsrc: int, k: int, W: int, key0: int = 0, dt: int = 15):
    """A repair after every k sources over the last W (RFC 8681 sliding window):
    repair t covers [max(0, (t+1)k - W), (t+1)k), repair_key key0 + t."""
    hdr = []
    for t in range(nsrc // k):
        end = (t + 1) * k
        fss = max(0, end - W)
        hdr.append((fss, end - fss, (key0 + t) & 0xFFFF, dt))
    return hdr
