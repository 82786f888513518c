"""The GF decode plan's closed form (csrc/fec_kernels.hip plan_gf) restated in
pure Python and checked against an explicit Gauss-Jordan inverse of the Cauchy
submatrix (D = A^-1 folded over the received
sources).  CPU only: this pins the algebra the kernel relies on; the GPU
parity tests pin the kernel itself.

    A_u = sum_t log(x_t ^ m_u) - sum_{v != u} log(m_u ^ m_v)
    K_q = sum_v log(z_q ^ m_v) - sum_{t: x_t != z_q} log(x_t ^ z_q)
    log D[u][q] = A_u + K_q - log(z_q ^ m_u)   (mod 255)
"""
import random

EXP = [0] * 512
LOG = [0] * 256
_x = 1
for _i in range(255):
    EXP[_i] = _x
    LOG[_x] = _i
    _x <<= 1
    if _x & 0x100:
        _x ^= 0x11D
for _i in range(255, 512):
    EXP[_i] = EXP[_i - 255]


def _mul(a, b):
    return 0 if a == 0 or b == 0 else EXP[LOG[a] + LOG[b]]


def _inv(a):
    return EXP[255 - LOG[a]]


def _decode_matrix_gj(k, r, pres):
    m = [j for j in range(k) if not (pres >> j) & 1]
    e = len(m)
    xs = [k + i for i in range(r) if (pres >> (k + i)) & 1][:e]
    rows = [[_inv(xs[t] ^ m[u]) for u in range(e)] + [int(t == w) for w in range(e)] for t in range(e)]
    for c in range(e):
        p = next(i for i in range(c, e) if rows[i][c])
        rows[c], rows[p] = rows[p], rows[c]
        ip = _inv(rows[c][c])
        rows[c] = [_mul(v, ip) for v in rows[c]]
        for i in range(e):
            if i != c and rows[i][c]:
                f = rows[i][c]
                rows[i] = [a ^ _mul(f, b) for a, b in zip(rows[i], rows[c])]
    ainv = [row[e:] for row in rows]
    z = [j for j in range(k) if (pres >> j) & 1] + xs
    d = [[0] * k for _ in range(e)]
    for u in range(e):
        for q, zq in enumerate(z):
            if q < k - e:
                s = 0
                for t in range(e):
                    s ^= _mul(ainv[u][t], _inv(xs[t] ^ zq))
                d[u][q] = s
            else:
                d[u][q] = ainv[u][q - (k - e)]
    return d, m, xs, z


def _decode_matrix_closed(k, m, xs, z):
    e = len(m)
    a = [sum(LOG[xs[t] ^ m[u]] for t in range(e)) - sum(LOG[m[u] ^ m[v]] for v in range(e) if v != u)
         for u in range(e)]
    kq = [sum(LOG[zq ^ mv] for mv in m) - sum(LOG[xt ^ zq] for xt in xs if xt != zq) for zq in z]
    # the kernel adds 255*4*kMaxR before the modulo to keep the sum positive
    return [[EXP[(a[u] + kq[q] - LOG[z[q] ^ m[u]] + 255 * 32) % 255] for q in range(k)] for u in range(e)]


def test_closed_form_matches_gauss_jordan():
    rng = random.Random(1)
    for _ in range(1500):
        k = rng.randint(1, 56)
        r = rng.randint(1, min(8, 64 - k))
        e = rng.randint(1, min(r, k))
        miss = set(rng.sample(range(k), e))
        reps = rng.sample(range(r), rng.randint(e, r))
        pres = sum(1 << j for j in range(k) if j not in miss) | sum(1 << (k + i) for i in reps)
        d, m, xs, z = _decode_matrix_gj(k, r, pres)
        assert _decode_matrix_closed(k, m, xs, z) == d, (k, r, hex(pres))


def test_closed_form_extremes():
    # k + r = 64 with every repair used, and single-erasure windows
    for k, r, miss in [(56, 8, range(48, 56)), (56, 8, range(8)), (1, 1, [0]), (63, 1, [62])]:
        pres = sum(1 << j for j in range(k) if j not in miss) | (((1 << r) - 1) << k)
        d, m, xs, z = _decode_matrix_gj(k, r, pres)
        assert _decode_matrix_closed(k, m, xs, z) == d
