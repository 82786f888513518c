// fec_spec.h — the coding contract shared by host runtime and gfx950 kernels.
//
// A.1 field GF(2^8)/0x11D generator 2, A.2 systematic
// Cauchy rows C[i][j] = inv((k+i) ^ j) / XOR groups j mod r, A.3 framing,
// A.5 splitmix64 streams.  Workload and digest definitions: DESIGN.md.
// The reference fec branch is not mounted (/root/reference/README.md:7),
// so these are build-owned choices (parity unpinned).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define FEC_HD __host__ __device__ __forceinline__
#else
#define FEC_HD inline
#endif

namespace fecgpu {

// ---------------------------------------------------------------- A.1 ----
struct GfTables {
    uint8_t exp[512];
    uint8_t log[256];
};

constexpr GfTables make_gf_tables() {
    GfTables t{};
    unsigned x = 1;
    for (int i = 0; i < 255; i++) {
        t.exp[i] = (uint8_t)x;
        t.log[x] = (uint8_t)i;
        x <<= 1;
        if (x & 0x100) x ^= 0x11D;
    }
    for (int i = 255; i < 512; i++) t.exp[i] = t.exp[i - 255];
    t.log[0] = 0;  // never used: callers test for zero first
    return t;
}

// ---------------------------------------------------------------- A.2 ----
// Parity rows P[i][j] (i < R, j < K) of the systematic generator, computed at
// compile time for the bit-sliced kernels (same construction as the host's
// host_parity_rows): matrix 0 = Cauchy inv((K+i) ^ j); matrix 1 = systematic
// Vandermonde, rows K.. of V * inv(V[0..K)) with V[i][j] = i^j.
template <int K, int R, int M>
struct ParityRows {
    uint8_t p[R][K];
    static constexpr uint8_t mul(const GfTables &t, uint8_t a, uint8_t b) {
        return (a && b) ? t.exp[t.log[a] + t.log[b]] : 0;
    }
    static constexpr uint8_t pw(const GfTables &t, uint8_t a, int n) {
        return n == 0 ? 1 : a == 0 ? 0 : t.exp[(t.log[a] * n) % 255];
    }
    constexpr ParityRows() : p{} {
        const GfTables t = make_gf_tables();
        if (M == 0) {
            for (int i = 0; i < R; i++)
                for (int j = 0; j < K; j++) p[i][j] = t.exp[255 - t.log[(uint8_t)((K + i) ^ j)]];
            return;
        }
        uint8_t a[K][2 * K] = {};  // [V_top | I] -> [I | inv(V_top)]
        for (int i = 0; i < K; i++)
            for (int j = 0; j < 2 * K; j++) a[i][j] = j < K ? pw(t, (uint8_t)i, j) : (uint8_t)(j - K == i);
        for (int c = 0; c < K; c++) {
            int piv = c;
            while (!a[piv][c]) piv++;
            for (int j = 0; j < 2 * K; j++) {
                const uint8_t x = a[piv][j];
                a[piv][j] = a[c][j];
                a[c][j] = x;
            }
            const uint8_t iv = t.exp[255 - t.log[a[c][c]]];
            for (int j = 0; j < 2 * K; j++) a[c][j] = mul(t, a[c][j], iv);
            for (int i = 0; i < K; i++) {
                const uint8_t f = a[i][c];
                if (i == c || !f) continue;
                for (int j = 0; j < 2 * K; j++) a[i][j] ^= mul(t, f, a[c][j]);
            }
        }
        for (int i = 0; i < R; i++)
            for (int j = 0; j < K; j++) {
                uint8_t v = 0;
                for (int q = 0; q < K; q++) v ^= mul(t, pw(t, (uint8_t)(K + i), q), a[q][K + j]);
                p[i][j] = v;
            }
    }
};

// ------------------------------------------------- A.2 random linear codes --
// RFC 8682 TinyMT32 (parameter set mat1 0x8f7011ee, mat2 0xfc78ff1f, tmat
// 0x3793fdff) and RFC 8681 §3.6 generate_coding_coefficients(): the PRNG and
// coefficient generator of the Sliding Window RLC FEC schemes, whose field
// for m = 8 is GF(2^8)/0x11D as A.1.  Pinned by RFC 8682's seed-1 outputs
// (tests/test_rlc_spec.py).  Used by FECGPU_MATRIX_RLC (block form: parity row
// i = coefficients of repair_key rlc_key + i over the k sources) and by the
// sliding-window encoder (one repair_key per repair symbol).
struct Tinymt32 {
    uint32_t s[4];
};

constexpr uint32_t kTmtMat1 = 0x8f7011eeu, kTmtMat2 = 0xfc78ff1fu, kTmtTmat = 0x3793fdffu;

FEC_HD void tinymt32_next(Tinymt32 &t) {
    uint32_t y = t.s[3];
    uint32_t x = (t.s[0] & 0x7fffffffu) ^ t.s[1] ^ t.s[2];
    x ^= x << 1;
    y ^= (y >> 1) ^ x;
    t.s[0] = t.s[1];
    t.s[1] = t.s[2];
    t.s[2] = x ^ (y << 10);
    t.s[3] = y;
    const uint32_t m = 0u - (y & 1u);
    t.s[1] ^= m & kTmtMat1;
    t.s[2] ^= m & kTmtMat2;
}

FEC_HD uint32_t tinymt32_u32(Tinymt32 &t) {
    tinymt32_next(t);
    uint32_t t0 = t.s[3];
    const uint32_t t1 = t.s[0] + (t.s[2] >> 8);
    t0 ^= t1;
    if (t1 & 1u) t0 ^= kTmtTmat;
    return t0;
}

FEC_HD void tinymt32_init(Tinymt32 &t, uint32_t seed) {
    t.s[0] = seed;
    t.s[1] = kTmtMat1;
    t.s[2] = kTmtMat2;
    t.s[3] = kTmtTmat;
    for (uint32_t i = 1; i < 8; i++)
        t.s[i & 3] ^= i + 1812433253u * (t.s[(i - 1) & 3] ^ (t.s[(i - 1) & 3] >> 30));
    if ((t.s[0] & 0x7fffffffu) == 0 && t.s[1] == 0 && t.s[2] == 0 && t.s[3] == 0) {
        t.s[0] = 'T';
        t.s[1] = 'I';
        t.s[2] = 'N';
        t.s[3] = 'Y';
    }
    for (int i = 0; i < 8; i++) tinymt32_next(t);
}

// RFC 8681 §3.6 for m = 8: cc[0..n) of repair_key `key` at density threshold
// dt (0..15; 15 = every coefficient nonzero, else each is nonzero with
// probability (dt + 1) / 16).  Returns false for dt > 15.
FEC_HD bool rlc_coefs(uint32_t key, int n, uint32_t dt, uint8_t *cc) {
    if (dt > 15) return false;
    Tinymt32 t;
    tinymt32_init(t, key & 0xFFFFu);
    for (int i = 0; i < n; i++) {
        uint32_t c = 0;
        if (dt == 15 || (tinymt32_u32(t) & 0xFu) <= dt) {
            do {
                c = tinymt32_u32(t) & 0xFFu;
            } while (c == 0);
        }
        cc[i] = (uint8_t)c;
    }
    return true;
}

// rlc_coefs read from the dense coefficient table (256 bytes per repair key:
// every key's dt-15 sequence, fec_internal.h kRlcRow) when it holds the row, else
// drawn; table words 8 at a time (independent loads, all in bounds: n <= 255)
FEC_HD void rlc_coefs_tab(const uint8_t *tab, uint32_t key, int n, uint32_t dt, uint8_t *cc) {
    if (!tab || dt != 15) {
        (void)rlc_coefs(key, n, dt, cc);
        return;
    }
    const uint32_t *row = reinterpret_cast<const uint32_t *>(tab + (size_t)(key & 0xFFFFu) * 256u);
    for (int q0 = 0; q0 * 4 < n; q0 += 8) {
        uint32_t w[8];
        for (int k = 0; k < 8; k++) w[k] = row[q0 + k];
        for (int k = 0; k < 8; k++)
            for (int b = 0; b < 4; b++) {
                const int j = (q0 + k) * 4 + b;
                if (j < n) cc[j] = (uint8_t)(w[k] >> (8 * b));
            }
    }
}

// multiply by x (=2) in GF(2^8)/0x11D, one byte in the low 8 bits
FEC_HD uint32_t gf_xtime(uint32_t a) { return ((a << 1) ^ ((a & 0x80u) ? 0x1Du : 0u)) & 0xFFu; }

// Product table of one coefficient c for the byte-permute multiply
// (DESIGN.md §GF multiply):  a data byte x = x[2:0] | x[5:3]<<3 | x[7:6]<<6
// gives  c*x = TA[x & 7] ^ TB[(x >> 3) & 7] ^ TC[x >> 6].
// TA/TB are 8-entry byte tables (lo dword = entries 0..3, hi = 4..7),
// TC a 4-entry table, so each lookup is one v_perm_b32.
struct CoefTab {
    uint32_t a_lo, a_hi, b_lo, b_hi;
    uint32_t c;
};

FEC_HD CoefTab make_coef_tab(uint32_t c) {
    uint32_t p[8];
    p[0] = c & 0xFFu;
    for (int b = 1; b < 8; b++) p[b] = gf_xtime(p[b - 1]);
    CoefTab t;
    // entries v = 0..3 of a 3-bit table over basis (q0, q1, q2): 0, q0, q1, q0^q1
    t.a_lo = (p[0] << 8) ^ (p[1] << 16) ^ ((p[0] ^ p[1]) << 24);
    t.a_hi = t.a_lo ^ (p[2] * 0x01010101u);
    t.b_lo = (p[3] << 8) ^ (p[4] << 16) ^ ((p[3] ^ p[4]) << 24);
    t.b_hi = t.b_lo ^ (p[5] * 0x01010101u);
    t.c = (p[6] << 8) ^ (p[7] << 16) ^ ((p[6] ^ p[7]) << 24);
    return t;
}

// ---------------------------------------------------------------- A.5 ----
FEC_HD uint64_t sm64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

constexpr uint64_t TAG_PAY = 0x5041594C4F414400ull;
constexpr uint64_t TAG_MTU = 0x4D54550000000000ull;
constexpr uint64_t TAG_LEN = 0x4C454E0000000000ull;
constexpr uint64_t TAG_ERA = 0x4552415345000000ull;
constexpr uint32_t P10 = 429496730u;  // 0.1 * 2^32

// packet length of source j of window w
FEC_HD uint32_t pkt_len(int workload, uint64_t smtu, uint64_t slen, uint64_t w, int j, uint32_t L) {
    if (workload == 0) return L;
    uint32_t mtu = (sm64(smtu + w) & 1) ? 9000u : 1200u;
    uint64_t h = sm64(slen + ((w << 8) | (uint64_t)j));
    if ((uint32_t)h < P10) return 64u + (uint32_t)((h >> 32) % (uint64_t)(mtu - 63u));
    return mtu;
}

}  // namespace fecgpu
