// fec_kernels.hip — gfx950 kernels of the FEC hot path.
//
// Work decomposition.  A workgroup of 256 threads owns
// `wpb` consecutive windows.  Their 16-byte symbol columns are flattened into
// one slot range (prefix sum of per-window column counts in LDS), so a wave
// streams columns of one or two windows and no lane idles on a short window.
// A lane owns one 16-byte column and walks the window's k input symbols with
// coalesced 16-B loads (consecutive lanes = consecutive columns of one symbol
// row), accumulating up to r outputs in registers, then stores them.
//
// GF(2^8) multiply (DESIGN.md §GF multiply): a coefficient c becomes three
// byte tables (3+3+2 bits of the data byte) and each lookup is one
// v_perm_b32 on four packed bytes, so c*x for 4 bytes costs 3 v_perm + 3
// v_xor, and the bit-field split of the data (5 VALU per dword) is shared by
// every output.  Tables are wave-uniform (encode) or per window (decode) and
// read from LDS as broadcasts.
#include "fec_internal.h"

namespace fecgpu {

__constant__ GfTables c_gf = make_gf_tables();

// ------------------------------------------------------------ helpers ---
__device__ __forceinline__ uint4 ld16(const uint8_t *p) {
    return *reinterpret_cast<const uint4 *>(p);
}
__device__ __forceinline__ void st16(uint8_t *p, uint4 v) { *reinterpret_cast<uint4 *>(p) = v; }
__device__ __forceinline__ uint4 xor4(uint4 a, uint4 b) {
    return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w);
}

struct Split {
    uint32_t a[4], b[4], c[4];
};

__device__ __forceinline__ Split split(uint4 v) {
    Split s;
    const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; i++) {
        s.a[i] = d[i] & 0x07070707u;
        s.b[i] = (d[i] >> 3) & 0x07070707u;
        s.c[i] = (d[i] >> 6) & 0x03030303u;
    }
    return s;
}

__device__ __forceinline__ uint32_t gmul4(const Split &s, int i, uint4 ab, uint32_t tc) {
    return __builtin_amdgcn_perm(ab.y, ab.x, s.a[i]) ^ __builtin_amdgcn_perm(ab.w, ab.z, s.b[i]) ^
           __builtin_amdgcn_perm(tc, tc, s.c[i]);
}

__device__ __forceinline__ void gmac(uint4 &acc, const Split &s, uint4 ab, uint32_t tc) {
    acc.x ^= gmul4(s, 0, ab, tc);
    acc.y ^= gmul4(s, 1, ab, tc);
    acc.z ^= gmul4(s, 2, ab, tc);
    acc.w ^= gmul4(s, 3, ab, tc);
}

__device__ __forceinline__ void win_geom(const BatchArgs &a, uint64_t w, uint64_t &base,
                                         uint32_t &stride, uint32_t &S) {
    S = a.sym_len ? a.sym_len[w] : a.S_all;
    if (a.win_off) {
        base = reinterpret_cast<uint64_t>(a.win) + a.win_off[w];
        stride = (S + 15u) & ~15u;
    } else {
        base = reinterpret_cast<uint64_t>(a.win) + w * (uint64_t)(a.k + a.r) * a.stride;
        stride = a.stride;
    }
}

// Inclusive scan of ncol over the block's windows by wave 0 (nb <= 64).
__device__ __forceinline__ void block_prefix(uint32_t *pfx, uint32_t v, int lane) {
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    pfx[lane + 1] = x;
    if (lane == 0) pfx[0] = 0;
}

#define WAVE_SYNC()                                                  \
    do {                                                             \
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");      \
        __builtin_amdgcn_wave_barrier();                             \
    } while (0)

// ============================================================ encode ===
// XOR (a4): R_g = xor of S_j, j = g mod r.  STEP loads in flight per lane.
template <int R>
__global__ __launch_bounds__(kBlock) void xor_encode_kernel(BatchArgs a) {
    __shared__ uint32_t s_pfx[kMaxWpb + 1];
    __shared__ uint64_t s_base[kMaxWpb];
    __shared__ uint32_t s_stride[kMaxWpb];
    constexpr int STEP = R >= 4 ? R : R * ((4 + R - 1) / R);
    const int tid = threadIdx.x, k = a.k;
    const uint64_t w0 = (uint64_t)blockIdx.x * a.wpb;
    const int nb = (int)min((uint64_t)a.wpb, a.nwin - w0);
    if (tid < 64) {
        uint32_t ncol = 0;
        if (tid < nb) {
            uint64_t base; uint32_t stride, S;
            win_geom(a, w0 + tid, base, stride, S);
            s_base[tid] = base;
            s_stride[tid] = stride;
            ncol = (S + 15u) >> 4;
        }
        block_prefix(s_pfx, ncol, tid);
    }
    __syncthreads();
    const uint32_t total = s_pfx[nb];
    int wl = 0;
    for (uint32_t s = tid; s < total; s += kBlock) {
        while (s >= s_pfx[wl + 1]) wl++;
        const uint32_t col = s - s_pfx[wl];
        uint8_t *base = reinterpret_cast<uint8_t *>(s_base[wl]) + col * 16u;
        const uint32_t stride = s_stride[wl];
        uint4 acc[R];
#pragma unroll
        for (int g = 0; g < R; g++) acc[g] = make_uint4(0, 0, 0, 0);
        for (int j0 = 0; j0 < k; j0 += STEP) {
            uint4 v[STEP];
#pragma unroll
            for (int t = 0; t < STEP; t++)
                v[t] = (j0 + t < k) ? ld16(base + (size_t)(j0 + t) * stride) : make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int t = 0; t < STEP; t++) acc[t % R] = xor4(acc[t % R], v[t]);
        }
#pragma unroll
        for (int g = 0; g < R; g++) st16(base + (size_t)(k + g) * stride, acc[g]);
    }
}

// GF(2^8) (a5): R_i = sum_j C[i][j] * S_j with kernel-uniform tables in LDS.
template <int R>
__global__ __launch_bounds__(kBlock) void gf_encode_kernel(BatchArgs a) {
    extern __shared__ uint4 dyn[];
    __shared__ uint32_t s_pfx[kMaxWpb + 1];
    __shared__ uint64_t s_base[kMaxWpb];
    __shared__ uint32_t s_stride[kMaxWpb];
    constexpr int U = 4;
    const int tid = threadIdx.x, k = a.k;
    uint4 *tab = dyn;
    uint32_t *tc = reinterpret_cast<uint32_t *>(dyn + k * R);
    for (int i = tid; i < k * R; i += kBlock) {
        tab[i] = a.enc_ab[i];
        tc[i] = a.enc_c[i];
    }
    const uint64_t w0 = (uint64_t)blockIdx.x * a.wpb;
    const int nb = (int)min((uint64_t)a.wpb, a.nwin - w0);
    if (tid < 64) {
        uint32_t ncol = 0;
        if (tid < nb) {
            uint64_t base; uint32_t stride, S;
            win_geom(a, w0 + tid, base, stride, S);
            s_base[tid] = base;
            s_stride[tid] = stride;
            ncol = (S + 15u) >> 4;
        }
        block_prefix(s_pfx, ncol, tid);
    }
    __syncthreads();
    const uint32_t total = s_pfx[nb];
    int wl = 0;
    for (uint32_t s = tid; s < total; s += kBlock) {
        while (s >= s_pfx[wl + 1]) wl++;
        const uint32_t col = s - s_pfx[wl];
        uint8_t *base = reinterpret_cast<uint8_t *>(s_base[wl]) + col * 16u;
        const uint32_t stride = s_stride[wl];
        uint4 acc[R];
#pragma unroll
        for (int m = 0; m < R; m++) acc[m] = make_uint4(0, 0, 0, 0);
        for (int j0 = 0; j0 < k; j0 += U) {
            uint4 v[U];
#pragma unroll
            for (int t = 0; t < U; t++)
                v[t] = (j0 + t < k) ? ld16(base + (size_t)(j0 + t) * stride) : make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int t = 0; t < U; t++) {
                if (j0 + t < k) {
                    const Split sp = split(v[t]);
                    const int row = (j0 + t) * R;
#pragma unroll
                    for (int m = 0; m < R; m++) gmac(acc[m], sp, tab[row + m], tc[row + m]);
                }
            }
        }
#pragma unroll
        for (int m = 0; m < R; m++) st16(base + (size_t)(k + m) * stride, acc[m]);
    }
}

// ============================================================ decode ===
// Window plan (a6) for XOR by one wave: every group with exactly one missing
// source and its repair present becomes an output (group g, missing m).
__device__ void plan_xor(const BatchArgs &a, uint64_t w, int lane, uint8_t *outg, uint8_t *outm,
                         uint8_t &ne_out) {
    const int k = a.k, r = a.r;
    const uint64_t kmask = (k >= 64) ? ~0ull : ((1ull << k) - 1);
    const uint64_t pres = a.present[w];
    const uint64_t miss = ~pres & kmask;
    bool rec = false, bad = false;
    uint64_t gm = 0;
    if (lane < r) {
        gm = a.gmask[lane];
        const int nm = __popcll(miss & gm);
        const bool rp = (pres >> (k + lane)) & 1;
        rec = (nm == 1) && rp;
        bad = (nm >= 1) && !rec;
    }
    const uint64_t recm = __ballot(rec);
    const uint64_t badm = __ballot(bad);
    if (rec) {
        const int u = __popcll(recm & ((1ull << lane) - 1));
        outg[u] = (uint8_t)lane;
        outm[u] = (uint8_t)(__ffsll((unsigned long long)(miss & gm)) - 1);
    }
    if (lane == 0) {
        ne_out = (uint8_t)__popcll(recm);
        a.status[w] = badm ? 1 : 0;
    }
}

template <int R>
__global__ __launch_bounds__(kBlock) void xor_decode_kernel(BatchArgs a) {
    __shared__ uint32_t s_pfx[kMaxWpb + 1];
    __shared__ uint64_t s_base[kMaxWpb];
    __shared__ uint32_t s_stride[kMaxWpb];
    __shared__ uint32_t s_ncol[kMaxWpb];
    __shared__ uint8_t s_ne[kMaxWpb];
    __shared__ uint8_t s_outg[kMaxWpb][kMaxR];
    __shared__ uint8_t s_outm[kMaxWpb][kMaxR];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, k = a.k, r = a.r;
    const uint64_t w0 = (uint64_t)blockIdx.x * a.wpb;
    const int nb = (int)min((uint64_t)a.wpb, a.nwin - w0);
    for (int wl = wave; wl < nb; wl += kBlock / 64) {
        plan_xor(a, w0 + wl, lane, s_outg[wl], s_outm[wl], s_ne[wl]);
        if (lane == 0) {
            uint64_t base; uint32_t stride, S;
            win_geom(a, w0 + wl, base, stride, S);
            s_base[wl] = base;
            s_stride[wl] = stride;
            s_ncol[wl] = (S + 15u) >> 4;
        }
    }
    __syncthreads();
    if (tid < 64) block_prefix(s_pfx, (tid < nb && s_ne[tid]) ? s_ncol[tid] : 0u, tid);
    __syncthreads();
    const uint32_t total = s_pfx[nb];
    int wl = 0;
    for (uint32_t s = tid; s < total; s += kBlock) {
        while (s >= s_pfx[wl + 1]) wl++;
        const uint32_t col = s - s_pfx[wl];
        uint8_t *base = reinterpret_cast<uint8_t *>(s_base[wl]) + col * 16u;
        const uint32_t stride = s_stride[wl];
        const int ne = s_ne[wl];
        for (int u = 0; u < ne; u++) {
            const int g = s_outg[wl][u], m = s_outm[wl][u];
            uint4 acc = ld16(base + (size_t)(k + g) * stride);
            for (int j0 = g; j0 < k; j0 += 4 * r) {
                uint4 v[4];
#pragma unroll
                for (int t = 0; t < 4; t++) {
                    const int j = j0 + t * r;
                    v[t] = (j < k && j != m) ? ld16(base + (size_t)j * stride) : make_uint4(0, 0, 0, 0);
                }
#pragma unroll
                for (int t = 0; t < 4; t++) acc = xor4(acc, v[t]);
            }
            st16(base + (size_t)m * stride, acc);
        }
    }
}

// GF plan (a6/a7) by one wave: choose the first e present repairs, invert the
// e x e Cauchy submatrix by Gauss-Jordan (lane = (row, col) of [A | I],
// exchanges by cross-lane shuffles), fold the inverse into one decode matrix
// D (e x k inputs: received sources then chosen repairs) and write D's
// byte-permute tables into the window's LDS region.
__device__ __forceinline__ uint32_t gf_mul_lds(const uint8_t *ex, const uint8_t *lg, uint32_t x,
                                               uint32_t y) {
    return (x && y) ? ex[lg[x] + lg[y]] : 0u;
}
__device__ __forceinline__ uint32_t gf_inv_lds(const uint8_t *ex, const uint8_t *lg, uint32_t x) {
    return ex[255 - lg[x]];
}

template <int R>
__device__ void plan_gf(const BatchArgs &a, uint64_t w, int lane, uint8_t *region,
                        const uint8_t *ex, const uint8_t *lg, uint8_t &ne_out) {
    const int k = a.k, r = a.r;
    uint4 *tab = reinterpret_cast<uint4 *>(region);
    uint32_t *tc = reinterpret_cast<uint32_t *>(region + k * R * 16);
    uint8_t *insym = region + k * R * 20;
    uint8_t *outsym = insym + 64;
    const uint64_t kmask = (k >= 64) ? ~0ull : ((1ull << k) - 1);
    const uint64_t pres = a.present[w];
    const uint64_t miss = ~pres & kmask;
    const uint64_t rep = (pres >> k) & ((1ull << r) - 1);
    const int e = __popcll(miss);
    if (e == 0 || __popcll(rep) < e || e > R) {
        if (lane == 0) {
            ne_out = 0;
            a.status[w] = (e == 0) ? 0 : 1;
        }
        return;
    }
    // u-th missing source / t-th present repair for lane u, t < e
    uint64_t mm = miss, rr = rep;
    for (int i = 0; i < lane && i < e; i++) { mm &= mm - 1; rr &= rr - 1; }
    const int my_m = (int)__ffsll((unsigned long long)mm) - 1;  // valid for lane < e
    const int my_sel = (int)__ffsll((unsigned long long)rr) - 1;
    // input list: received sources ascending, then the e chosen repairs
    if (lane < k && ((pres >> lane) & 1)) insym[__popcll(pres & kmask & ((1ull << lane) - 1))] = (uint8_t)lane;
    if (lane < e) {
        insym[k - e + lane] = (uint8_t)(k + my_sel);
        outsym[lane] = (uint8_t)my_m;
    }
    // [A | I], A[t][u] = inv((k + sel_t) ^ m_u); lane = t*8 + u
    const int t = lane >> 3, u = lane & 7;
    const int sel_t = __shfl(my_sel, t & 7, 64);
    const int m_u = __shfl(my_m, u, 64);
    const bool valid = (t < e) && (u < e);
    uint32_t xl = valid ? gf_inv_lds(ex, lg, (uint32_t)((k + sel_t) ^ m_u)) : 0u;
    uint32_t xr = (valid && t == u) ? 1u : 0u;
    bool singular = false;
    for (int c = 0; c < e; c++) {
        const uint32_t piv = __shfl(xl, c * 8 + c, 64);
        if (piv == 0) { singular = true; break; }  // never for Cauchy (leading minors are Cauchy)
        const uint32_t ip = gf_inv_lds(ex, lg, piv);
        if (t == c) {
            xl = gf_mul_lds(ex, lg, xl, ip);
            xr = gf_mul_lds(ex, lg, xr, ip);
        }
        const uint32_t f = __shfl(xl, (t & 7) * 8 + c, 64);
        const uint32_t rl = __shfl(xl, c * 8 + u, 64);
        const uint32_t rq = __shfl(xr, c * 8 + u, 64);
        if (t != c && valid) {
            xl ^= gf_mul_lds(ex, lg, f, rl);
            xr ^= gf_mul_lds(ex, lg, f, rq);
        }
    }
    if (singular) {
        if (lane == 0) { ne_out = 0; a.status[w] = 1; }
        return;
    }
    WAVE_SYNC();
    // D[u][q] for idx = u*k + q; Ainv[u][t] = xr of lane u*8 + t.
    // Every __shfl runs with the whole wave active: ds_bpermute reads 0 from a
    // source lane that is masked off, so no shuffle may sit inside a branch.
    const int kr = k - e;
    for (int base = 0; base < e * k; base += 64) {
        const int idx = base + lane;
        const int du = idx / k, dq = idx - du * k;
        const bool live = idx < e * k;
        const bool is_src = dq < kr;
        const uint32_t j = (live && is_src) ? insym[dq] : 0u;
        uint32_t csrc = 0;
        for (int tt = 0; tt < e; tt++) {
            const uint32_t ai = __shfl(xr, ((du & 7) * 8 + tt) & 63, 64);
            const int st = __shfl(my_sel, tt, 64);
            if (is_src) csrc ^= gf_mul_lds(ex, lg, ai, gf_inv_lds(ex, lg, (uint32_t)((k + st) ^ j)));
        }
        const uint32_t crep = __shfl(xr, ((du & 7) * 8 + (is_src ? 0 : dq - kr)) & 63, 64);
        const uint32_t c = is_src ? csrc : crep;
        if (live) {
            const CoefTab ct = make_coef_tab(c);
            tab[dq * R + du] = make_uint4(ct.a_lo, ct.a_hi, ct.b_lo, ct.b_hi);
            tc[dq * R + du] = ct.c;
        }
    }
    if (lane == 0) {
        ne_out = (uint8_t)e;
        a.status[w] = 0;
    }
}

template <int R>
__global__ __launch_bounds__(kBlock) void gf_decode_kernel(BatchArgs a) {
    extern __shared__ uint4 dyn[];
    __shared__ uint8_t s_exp[512];
    __shared__ uint8_t s_log[256];
    __shared__ uint32_t s_pfx[kMaxWpb + 1];
    __shared__ uint64_t s_base[kMaxWpb];
    __shared__ uint32_t s_stride[kMaxWpb];
    __shared__ uint32_t s_ncol[kMaxWpb];
    __shared__ uint8_t s_ne[kMaxWpb];
    constexpr int U = 4;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, k = a.k;
    uint8_t *regions = reinterpret_cast<uint8_t *>(dyn);
    for (int i = tid; i < 512; i += kBlock) s_exp[i] = c_gf.exp[i];
    for (int i = tid; i < 256; i += kBlock) s_log[i] = c_gf.log[i];
    __syncthreads();
    const uint64_t w0 = (uint64_t)blockIdx.x * a.wpb;
    const int nb = (int)min((uint64_t)a.wpb, a.nwin - w0);
    for (int wl = wave; wl < nb; wl += kBlock / 64) {
        plan_gf<R>(a, w0 + wl, lane, regions + (size_t)wl * a.win_lds, s_exp, s_log, s_ne[wl]);
        if (lane == 0) {
            uint64_t base; uint32_t stride, S;
            win_geom(a, w0 + wl, base, stride, S);
            s_base[wl] = base;
            s_stride[wl] = stride;
            s_ncol[wl] = (S + 15u) >> 4;
        }
    }
    __syncthreads();
    if (tid < 64) block_prefix(s_pfx, (tid < nb && s_ne[tid]) ? s_ncol[tid] : 0u, tid);
    __syncthreads();
    const uint32_t total = s_pfx[nb];
    int wl = 0;
    for (uint32_t s = tid; s < total; s += kBlock) {
        while (s >= s_pfx[wl + 1]) wl++;
        const uint32_t col = s - s_pfx[wl];
        uint8_t *base = reinterpret_cast<uint8_t *>(s_base[wl]) + col * 16u;
        const uint32_t stride = s_stride[wl];
        const int ne = s_ne[wl];
        const uint8_t *region = regions + (size_t)wl * a.win_lds;
        const uint4 *tab = reinterpret_cast<const uint4 *>(region);
        const uint32_t *tc = reinterpret_cast<const uint32_t *>(region + k * R * 16);
        const uint8_t *insym = region + k * R * 20;
        const uint8_t *outsym = insym + 64;
        uint4 acc[R];
#pragma unroll
        for (int m = 0; m < R; m++) acc[m] = make_uint4(0, 0, 0, 0);
        for (int q0 = 0; q0 < k; q0 += U) {
            uint4 v[U];
#pragma unroll
            for (int t = 0; t < U; t++)
                v[t] = (q0 + t < k) ? ld16(base + (size_t)insym[q0 + t] * stride) : make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int t = 0; t < U; t++) {
                if (q0 + t < k) {
                    const Split sp = split(v[t]);
                    const int row = (q0 + t) * R;
#pragma unroll
                    for (int m = 0; m < R; m++)
                        if (m < ne) gmac(acc[m], sp, tab[row + m], tc[row + m]);
                }
            }
        }
#pragma unroll
        for (int m = 0; m < R; m++)
            if (m < ne) st16(base + (size_t)outsym[m] * stride, acc[m]);
    }
}

// ========================================================= workloads ===
__global__ __launch_bounds__(kBlock) void synth_kernel(SynthArgs a) {
    __shared__ uint32_t s_len[kMaxK];
    __shared__ uint32_t s_S;
    const uint64_t w = a.w0 + blockIdx.x;
    const int tid = threadIdx.x, k = a.k;
    const uint64_t smtu = sm64(a.seed ^ TAG_MTU), slen = sm64(a.seed ^ TAG_LEN);
    const uint64_t spay = sm64(a.seed ^ TAG_PAY);
    if (tid == 0) s_S = 0;
    __syncthreads();
    if (tid < k) {
        s_len[tid] = pkt_len(a.workload, smtu, slen, w, tid, a.L);
        atomicMax(&s_S, s_len[tid]);
    }
    __syncthreads();
    const uint32_t hdr = a.workload == 0 ? 0u : 2u;
    const uint32_t S = hdr + s_S;
    if (tid == 0 && a.sym_len) a.sym_len[blockIdx.x] = S;
    uint8_t *win = a.win + (uint64_t)blockIdx.x * (uint64_t)(k + a.r) * a.stride;
    const uint32_t ncol = a.stride >> 4;
    for (uint32_t idx = tid; idx < (uint32_t)k * ncol; idx += kBlock) {
        const int j = (int)(idx / ncol);
        const uint32_t c = idx - (uint32_t)j * ncol;
        const uint32_t len = s_len[j];
        uint32_t out[4] = {0, 0, 0, 0};
        uint64_t cw = ~0ull, word = 0;
        for (int b = 0; b < 16; b++) {
            const uint32_t o = c * 16 + b;
            uint32_t byte = 0;
            if (hdr && o == 0) byte = len >> 8;
            else if (hdr && o == 1) byte = len & 0xFF;
            else if (o >= hdr && o < hdr + len) {
                const uint32_t po = o - hdr;
                const uint64_t wi = po >> 3;
                if (wi != cw) {
                    cw = wi;
                    word = sm64(spay + ((w << 24) | ((uint64_t)j << 16) | wi));
                }
                byte = (uint32_t)(word >> (8 * (po & 7))) & 0xFF;
            }
            out[b >> 2] |= byte << (8 * (b & 3));
        }
        st16(win + (size_t)j * a.stride + c * 16, make_uint4(out[0], out[1], out[2], out[3]));
    }
}

__global__ __launch_bounds__(kBlock) void erasure_kernel(EraseArgs a) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= a.nwin) return;
    const uint64_t w = a.w0 + i;
    const int k = a.k, r = a.r;
    const uint64_t all = (k + r >= 64) ? ~0ull : ((1ull << (k + r)) - 1);
    const uint64_t sera = sm64(a.seed ^ TAG_ERA);
    uint64_t p = all;
    if (a.erasure == 2) {
        for (int s = 0; s < k + r; s++)
            if ((uint32_t)sm64(sera + ((w << 8) | (uint64_t)s)) < P10) p &= ~(1ull << s);
    } else if (a.erasure == 1) {
        if (a.scheme == 1) {
            uint8_t perm[kMaxK];
            for (int j = 0; j < k; j++) perm[j] = (uint8_t)j;
            const int e = r < k ? r : k;
            for (int t = 0; t < e; t++) {
                const uint64_t h = sm64(sera + ((w << 8) | (uint64_t)t));
                const int u = t + (int)(h % (uint64_t)(k - t));
                const uint8_t tmp = perm[t]; perm[t] = perm[u]; perm[u] = tmp;
                p &= ~(1ull << perm[t]);
            }
        } else {
            for (int g = 0; g < r; g++) {
                const int n = (k - g + r - 1) / r;
                if (n <= 0) continue;
                const int idx = (int)(sm64(sera + ((w << 8) | (uint64_t)g)) % (uint64_t)n);
                p &= ~(1ull << (g + idx * r));
            }
        }
    }
    a.present[i] = p;
}

// Digest: one workgroup per window.
__global__ __launch_bounds__(kBlock) void digest_kernel(DigestArgs a) {
    __shared__ uint64_t s_red[kBlock / 64];
    const uint64_t wi = blockIdx.x;
    const int tid = threadIdx.x, n = a.k + a.r;
    const uint32_t S = a.sym_len ? a.sym_len[wi] : a.S_all;
    const uint32_t nw = (S + 7u) >> 3;
    const uint8_t *win = a.win + wi * (uint64_t)n * a.stride;
    uint64_t d = 0;
    for (uint32_t idx = tid; idx < (uint32_t)n * nw; idx += kBlock) {
        const uint32_t i = idx / nw, t = idx - i * nw;
        uint64_t word = *reinterpret_cast<const uint64_t *>(win + (size_t)i * a.stride + t * 8u);
        const uint32_t valid = S - t * 8u;
        if (valid < 8) word &= (1ull << (8 * valid)) - 1;
        d ^= sm64(word ^ (((uint64_t)i << 16) | t));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) d ^= __shfl_xor(d, o, 64);
    if ((tid & 63) == 0) s_red[tid >> 6] = d;
    __syncthreads();
    if (tid == 0) {
        uint64_t x = 0;
        for (int i = 0; i < kBlock / 64; i++) x ^= s_red[i];
        atomicXor(reinterpret_cast<unsigned long long *>(a.digest),
                  (unsigned long long)sm64(x + a.w0 + wi));
    }
}

// ========================================================== launchers ===
#define DISPATCH_R(R_, KERNEL, ...)                                                      \
    switch (R_) {                                                                        \
        case 1: hipLaunchKernelGGL(KERNEL<1>, __VA_ARGS__); break;                       \
        case 2: hipLaunchKernelGGL(KERNEL<2>, __VA_ARGS__); break;                       \
        case 3: hipLaunchKernelGGL(KERNEL<3>, __VA_ARGS__); break;                       \
        case 4: hipLaunchKernelGGL(KERNEL<4>, __VA_ARGS__); break;                       \
        case 5: hipLaunchKernelGGL(KERNEL<5>, __VA_ARGS__); break;                       \
        case 6: hipLaunchKernelGGL(KERNEL<6>, __VA_ARGS__); break;                       \
        case 7: hipLaunchKernelGGL(KERNEL<7>, __VA_ARGS__); break;                       \
        case 8: hipLaunchKernelGGL(KERNEL<8>, __VA_ARGS__); break;                       \
        default: return hipErrorInvalidValue;                                            \
    }

hipError_t launch_encode(int scheme, const BatchArgs &a, const LaunchPlan &p, hipStream_t s) {
    if (p.blocks == 0) return hipSuccess;
    const dim3 grid((unsigned)p.blocks), block(kBlock);
    if (scheme == 0) {
        DISPATCH_R(a.r, xor_encode_kernel, grid, block, 0, s, a);
    } else {
        DISPATCH_R(a.r, gf_encode_kernel, grid, block, p.lds_bytes, s, a);
    }
    return hipGetLastError();
}

hipError_t launch_decode(int scheme, const BatchArgs &a, const LaunchPlan &p, hipStream_t s) {
    if (p.blocks == 0) return hipSuccess;
    const dim3 grid((unsigned)p.blocks), block(kBlock);
    if (scheme == 0) {
        DISPATCH_R(a.r, xor_decode_kernel, grid, block, 0, s, a);
    } else {
        DISPATCH_R(a.r, gf_decode_kernel, grid, block, p.lds_bytes, s, a);
    }
    return hipGetLastError();
}

hipError_t launch_synth(const SynthArgs &a, hipStream_t s) {
    if (a.nwin == 0) return hipSuccess;
    hipLaunchKernelGGL(synth_kernel, dim3((unsigned)a.nwin), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_erasure(const EraseArgs &a, hipStream_t s) {
    if (a.nwin == 0) return hipSuccess;
    hipLaunchKernelGGL(erasure_kernel, dim3((unsigned)((a.nwin + kBlock - 1) / kBlock)), dim3(kBlock),
                       0, s, a);
    return hipGetLastError();
}

hipError_t launch_digest(const DigestArgs &a, hipStream_t s) {
    if (a.nwin == 0) return hipSuccess;
    hipLaunchKernelGGL(digest_kernel, dim3((unsigned)a.nwin), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

}  // namespace fecgpu
