/*
 * fec_oracle.h — CPU oracle for the FEC hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * link or call this.  The product (quic-fec-eps_amd/, libfecgpu.so) never
 * does: it has no CPU fallback.
 *
 * PARITY UNPINNED.  The reference (holzingk/quic-fec-eps, fec branch;
 * /root/reference/README.md:7) is mounted as a README only: no Rust source,
 * no Cargo.lock, no tests, no golden vectors.  This file
 * restates the coding contract the build owns
 * and is pinned only by
 *   - GF(2^8)/0x11D known-answer facts and an exhaustive
 *     cross-check against sympy.polys.galoistools (tests/test_oracle_field.py),
 *   - an independent numpy restatement (oracle/np_oracle.py) that generated
 *     the committed fixtures in tests/golden/ (tests/golden/make_golden.py),
 *   - algebraic invariants (decode∘erase∘encode = id, MDS decodability).
 * Decode output is pinned by construction (recovered bytes == originals).
 *
 * Layout (Appendix A.4): a window is (k + r) symbols of `stride` bytes,
 * sources 0..k-1 then repairs k..k+r-1; only bytes [0, S) of each symbol are
 * meaningful (A.3).
 */
#ifndef FEC_ORACLE_H
#define FEC_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* schemes: XOR groups, GF(2^8) Cauchy rows, GF(2^8) systematic Vandermonde
 * rows, GF(2^8) RFC 8681 random linear code rows (ORC_RLC(key0, dt): row i
 * from repair_key key0 + i at density threshold dt) */
enum { ORC_XOR = 0, ORC_GF256 = 1, ORC_GF256_VDM = 2, ORC_GF256_RLC = 3 };
#define ORC_RLC(key0, dt) (ORC_GF256_RLC | ((dt) << 4) | ((int)(key0) << 8))
#define ORC_KIND(s) ((s) & 0xF)
#define ORC_RLC_DT(s) (((s) >> 4) & 0xF)
#define ORC_RLC_KEY(s) (((s) >> 8) & 0xFFFF)
enum { ORC_FIXED = 0, ORC_LENPREFIX = 1 };
enum { ORC_OK = 0, ORC_UNRECOVERABLE = 1 };

/* A.1 field */
uint8_t orc_gf_mul(uint8_t a, uint8_t b);
uint8_t orc_gf_inv(uint8_t a);
uint8_t orc_gf_exp(int i);
int     orc_gf_log(uint8_t a);
/* A.2 matrix: C[i*k + j] = inv((k + i) ^ j) */
void    orc_cauchy(int k, int r, uint8_t *C);
/* systematic Vandermonde parity rows P[i*k + j] (Backblaze construction) */
void    orc_vandermonde(int k, int r, uint8_t *P);
/* parity rows of a GF scheme (ORC_GF256 -> Cauchy, ORC_GF256_VDM -> Vandermonde,
 * ORC_RLC(key0, dt) -> RFC 8681 coefficients) */
void    orc_matrix(int scheme, int k, int r, uint8_t *C);
/* RFC 8682 TinyMT32 outputs 1..n after tinymt32_init(seed) */
void    orc_tinymt32(uint32_t seed, int n, uint32_t *out);
/* RFC 8681 §3.6 generate_coding_coefficients, m = 8; -1 if dt > 15 */
int     orc_rlc_coefs(uint32_t key, int n, int dt, uint8_t *cc);
/* missing sources and e independent present repairs (greedy in repair order);
 * returns e (0: nothing missing) or -1 if the present repairs have rank < e */
int     orc_select_rows(int k, int r, const uint8_t *C, uint64_t present, int *miss, int *sel);

/* A.5 PRNG / workload */
uint64_t orc_sm64(uint64_t x);
/* packet length of source j of window w for a workload */
uint32_t orc_pkt_len(int workload, uint64_t seed, uint64_t w, int j, int k, uint32_t L);
/* symbol length S of window w */
uint32_t orc_sym_len(int workload, uint64_t seed, uint64_t w, int k, uint32_t L);
/* fill the k source symbols of window w (framing applied, zero padded to stride) */
void     orc_fill_window(int workload, uint64_t seed, uint64_t w, int k, int r, uint32_t L,
                         uint32_t stride, uint8_t *win);
/* present mask (bit i: symbol i received) for window w */
uint64_t orc_present(int erasure, uint64_t seed, uint64_t w, int scheme, int k, int r);

/* coding: in place on one window */
void orc_encode(int scheme, int k, int r, uint32_t S, uint32_t stride, uint8_t *win);
/* recovers missing sources in place; returns ORC_OK or ORC_UNRECOVERABLE.
 * For XOR, recoverable groups are recovered even when the window is not. */
int  orc_decode(int scheme, int k, int r, uint32_t S, uint32_t stride, uint64_t present,
                uint8_t *win);

/* A.6 digest of one window's emitted bytes: repairs, then sources (all of them) */
uint64_t orc_window_digest(int k, int r, uint32_t S, uint32_t stride, const uint8_t *win);

/* batch helpers (uniform stride, windows back to back), pthreads over windows */
void orc_encode_batch(int scheme, int k, int r, const uint32_t *S, uint32_t stride,
                      uint64_t nwin, uint8_t *wins, int nthreads);
void orc_decode_batch(int scheme, int k, int r, const uint32_t *S, uint32_t stride,
                      uint64_t nwin, const uint64_t *present, uint8_t *status, uint8_t *wins,
                      int nthreads);

/* CPU baseline codec (fec_cpu_simd.c): same contract and outputs,
 * AVX2 split-nibble tables or GFNI affine products; level 0 scalar, 1 AVX2,
 * 2 AVX2+GFNI (detected; set_level(-1) restores detection) */
int  orc_simd_detect(void);
int  orc_simd_level(void);
void orc_simd_set_level(int level);
void orc_encode_batch_simd(int scheme, int k, int r, const uint32_t *S, uint32_t stride,
                           uint64_t nwin, uint8_t *wins, int nthreads);
void orc_decode_batch_simd(int scheme, int k, int r, const uint32_t *S, uint32_t stride,
                           uint64_t nwin, const uint64_t *present, uint8_t *status, uint8_t *wins,
                           int nthreads);

/* parallel fill of nwin windows + S + present masks; returns source-packet bytes */
uint64_t orc_make_batch(int workload, uint64_t seed, uint64_t w0, uint64_t nwin, int scheme,
                        int erasure, int k, int r, uint32_t L, uint32_t stride, uint8_t *wins,
                        uint32_t *S, uint64_t *present, int nthreads);

/* ---- sliding-window RLC (RFC 8681, m = 8): fecgpu_sw_encode / _decode ----
 * Same header layout as fecgpu_sw_repair. */
typedef struct orc_sw_repair {
    uint64_t fss;
    uint16_t nss;
    uint16_t key;
    uint8_t  dt;
    uint8_t  reserved[3];
} orc_sw_repair;

/* rep[t] = sum_{j < nss_t} cc_t[j] * src[fss_t + j] over bytes [0, S) */
void    orc_sw_encode(const uint8_t *src, uint64_t nsrc, uint32_t S, uint32_t stride,
                      const orc_sw_repair *hdr, uint64_t nrep, uint8_t *rep);
/* Global Gauss-Jordan over every lost source (unknown) and every received
 * repair that covers one; recovers each determined unknown in place;
 * status[i] = 0 present / recovered, 1 lost.  Returns #recovered, or -1 if
 * there are more than 4096 unknowns (a test-size oracle). */
int64_t orc_sw_decode(uint8_t *src, const uint8_t *src_present, uint64_t nsrc, const uint8_t *rep,
                      const uint8_t *rep_present, const orc_sw_repair *hdr, uint64_t nrep,
                      uint32_t S, uint32_t stride, uint8_t *status);

/* Same statuses and recovered bytes as orc_sw_decode, by banded elimination
 * with no size limit (fec_sw_banded.c; the algorithm of the GPU's long-system
 * path).  Returns #recovered. */
int64_t orc_sw_decode_banded(uint8_t *src, const uint8_t *src_present, uint64_t nsrc, const uint8_t *rep,
                             const uint8_t *rep_present, const orc_sw_repair *hdr, uint64_t nrep,
                             uint32_t S, uint32_t stride, uint8_t *status);

/* CPU baseline of the sliding-window code (fec_cpu_simd.c): the same outputs as
 * orc_sw_encode / orc_sw_decode, vectorised at orc_simd_level() and spread over
 * nthreads (encode: repairs; decode: runs of whole linked systems).  Decode
 * needs the headers in fss order. */
void    orc_sw_encode_simd(const uint8_t *src, uint64_t nsrc, uint32_t S, uint32_t stride,
                           const orc_sw_repair *hdr, uint64_t nrep, uint8_t *rep, int nthreads);
int64_t orc_sw_decode_simd(uint8_t *src, const uint8_t *src_present, uint64_t nsrc, const uint8_t *rep,
                           const uint8_t *rep_present, const orc_sw_repair *hdr, uint64_t nrep,
                           uint32_t S, uint32_t stride, uint8_t *status, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
