/*
 * xrs_oracle.c -- CPU restatement of templexxx/xrs and of the arithmetic of its
 * dependencies (TEST INFRASTRUCTURE ONLY: the parity checker and the CPU
 * baseline timed by bench.py; the product never links this file).
 *
 * What is restated, and from where:
 *   - xrs.go (available): New :55-68, makeXORSet :77-100, Encode :103-128,
 *     checkSize :130-136, GetNeedVects :146-171, ReconstOne :175-221,
 *     Reconst :236-301, retrieveRS :305-320, Update :324-346,
 *     Replace :363-387.
 *   - github.com/templexxx/reedsolomon v1.1.3 (go.mod:6, NOT in the image):
 *     GF(2^8) with polynomial 0x11d; systematic encode matrix = identity on
 *     top of the Cauchy rows gen[i][j] = inv(i ^ j) (i parity index, j data
 *     index).  This is the published Cauchy construction and it reproduces
 *     the reference KAT xrs_test.go:108-115 bit for bit.  Reconst inverts the
 *     d x d survivor submatrix (result unique by the MDS property, so the
 *     inversion algorithm does not matter) and rebuilds each needed row from
 *     the survivors; Update/Replace XOR gen[d+r][row]*delta into parity.
 *   - github.com/templexxx/xorsimd v0.1.1 (go.mod:7, NOT in the image):
 *     Encode(dst, src) = XOR of all src into dst; dst may alias src[0].
 *
 * The CPU baseline (oxrs_*_batch) follows the same design as the reference's
 * dependency: 16-entry low/high-nibble product tables looked up with vpshufb
 * (AVX-512BW when the CPU has it, else AVX2; the dependency dispatches the same way)
 * and, like xrs.go Encode, a second pass for the piggyback XOR.
 */
#include "xrs_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#if defined(__x86_64__)
#include <immintrin.h>
#endif

/* ------------------------------------------------------------------ GF(2^8) */
static uint8_t g_exp[512];
static uint8_t g_log[256];
static int g_init = 0;

static void gf_init(void) {
  if (g_init) return;
  unsigned v = 1;
  for (int i = 0; i < 255; i++) {
    g_exp[i] = (uint8_t)v;
    g_log[v] = (uint8_t)i;
    v <<= 1;
    if (v & 0x100) v ^= 0x11d; /* primitive polynomial x^8+x^4+x^3+x^2+1 */
  }
  for (int i = 255; i < 512; i++) g_exp[i] = g_exp[i - 255];
  g_log[0] = 0;
  g_init = 1;
}

uint8_t oxrs_gf_mul(uint8_t a, uint8_t b) {
  gf_init();
  if (a == 0 || b == 0) return 0;
  return g_exp[g_log[a] + g_log[b]];
}

uint8_t oxrs_gf_inv(uint8_t a) {
  gf_init();
  if (a == 0) return 0;
  return g_exp[255 - g_log[a]];
}

/* dst[i] ^= c * src[i] */
static void mul_add(uint8_t c, const uint8_t *src, uint8_t *dst, size_t n) {
  if (c == 0) return;
  if (c == 1) {
    for (size_t i = 0; i < n; i++) dst[i] ^= src[i];
    return;
  }
  const unsigned lc = g_log[c];
  for (size_t i = 0; i < n; i++) {
    uint8_t s = src[i];
    if (s) dst[i] ^= g_exp[lc + g_log[s]];
  }
}

/* Gauss-Jordan inverse of an n x n matrix; 0 on success, -1 if singular. */
static int gf_invert(uint8_t *m, uint8_t *inv, int n) {
  uint8_t *a = (uint8_t *)malloc((size_t)n * n);
  memcpy(a, m, (size_t)n * n);
  memset(inv, 0, (size_t)n * n);
  for (int i = 0; i < n; i++) inv[i * n + i] = 1;
  for (int c = 0; c < n; c++) {
    int piv = -1;
    for (int r = c; r < n; r++)
      if (a[r * n + c]) { piv = r; break; }
    if (piv < 0) { free(a); return -1; }
    if (piv != c) {
      for (int k = 0; k < n; k++) {
        uint8_t t = a[c * n + k]; a[c * n + k] = a[piv * n + k]; a[piv * n + k] = t;
        t = inv[c * n + k]; inv[c * n + k] = inv[piv * n + k]; inv[piv * n + k] = t;
      }
    }
    uint8_t f = oxrs_gf_inv(a[c * n + c]);
    for (int k = 0; k < n; k++) {
      a[c * n + k] = oxrs_gf_mul(a[c * n + k], f);
      inv[c * n + k] = oxrs_gf_mul(inv[c * n + k], f);
    }
    for (int r = 0; r < n; r++) {
      if (r == c || a[r * n + c] == 0) continue;
      uint8_t g = a[r * n + c];
      for (int k = 0; k < n; k++) {
        a[r * n + k] ^= oxrs_gf_mul(g, a[c * n + k]);
        inv[r * n + k] ^= oxrs_gf_mul(g, inv[c * n + k]);
      }
    }
  }
  free(a);
  return 0;
}

/* --------------------------------------------------------------- codec New */
/* xrs.go:77-100 makeXORSet: data i goes to parity d+1+(i mod (p-1)), round robin. */
static void make_xorset(oxrs *x) {
  int d = x->d, p = x->p;
  memset(x->xs_len, 0, sizeof(x->xs_len));
  int j = d + 1;
  for (int i = 0; i < d; i++) {
    if (j > d + p - 1) j = d + 1;
    x->xs[j][x->xs_len[j]++] = i;
    j++;
  }
}

size_t oxrs_sizeof(void) { return sizeof(oxrs); }

/* xrs.go:55-68 New; reedsolomon.New validity [dep]: d>0, p>0, d+p<=256
 * (xrs_test.go:125-134 requires success for every d>=1, p>=2, d+p<=256). */
int oxrs_new(int d, int p, oxrs *x) {
  gf_init();
  if (p == 1) return OXRS_ERR_ILLEGAL_PARITY; /* xrs.go:56-59 */
  if (d <= 0 || p <= 0 || d + p > 256) return OXRS_ERR_ILLEGAL_VECTS;
  memset(x, 0, sizeof(*x));
  x->d = d;
  x->p = p;
  for (int i = 0; i < d; i++) x->gen[i][i] = 1;
  for (int i = d; i < d + p; i++)
    for (int j = 0; j < d; j++) x->gen[i][j] = oxrs_gf_inv((uint8_t)(i ^ j));
  make_xorset(x);
  return OXRS_OK;
}

/* xrs.go:130-136 */
static int check_size(size_t size) { return (size & 1) ? OXRS_ERR_SIZE_NOT_EVEN : OXRS_OK; }

/* xrs.go:146-171 GetNeedVects */
int oxrs_get_need_vects(const oxrs *x, int k, int *a_need, int *a_len, int b_need[2]) {
  int d = x->d;
  if (k < 0 || k >= d) return OXRS_ERR_ILLEGAL_DATA_INDEX;
  b_need[0] = d;
  b_need[1] = 0;
  for (int h = d + 1; h < d + x->p; h++)
    for (int t = 0; t < x->xs_len[h]; t++)
      if (x->xs[h][t] == k) b_need[1] = h;
  int n = 0;
  for (int t = 0; t < x->xs_len[b_need[1]]; t++)
    if (x->xs[b_need[1]][t] != k) a_need[n++] = x->xs[b_need[1]][t];
  *a_len = n;
  return OXRS_OK;
}

/* ------------------------------------------------------ RS layer [dep] */
int oxrs_rs_encode(const oxrs *x, uint8_t *const *vects, size_t size) {
  int d = x->d, p = x->p;
  for (int r = 0; r < p; r++) {
    memset(vects[d + r], 0, size);
    for (int j = 0; j < d; j++) mul_add(x->gen[d + r][j], vects[j], vects[d + r], size);
  }
  return OXRS_OK;
}

int oxrs_rs_reconst(const oxrs *x, uint8_t *const *vects, size_t size,
                    const int *dp_has, int n_has, const int *need, int n_need) {
  int d = x->d, n = x->d + x->p;
  if (n_need == 0) return OXRS_OK;
  if (n_has < d) return OXRS_ERR_TOO_FEW_SURVIVORS;
  for (int i = 0; i < n_has; i++)
    if (dp_has[i] < 0 || dp_has[i] >= n) return OXRS_ERR_ILLEGAL_INDEX;
  for (int i = 0; i < n_need; i++)
    if (need[i] < 0 || need[i] >= n) return OXRS_ERR_ILLEGAL_INDEX;
  /* survivors: the first d entries of dpHas */
  uint8_t *e = (uint8_t *)malloc((size_t)d * d), *einv = (uint8_t *)malloc((size_t)d * d);
  for (int i = 0; i < d; i++)
    for (int j = 0; j < d; j++) e[i * d + j] = x->gen[dp_has[i]][j];
  if (gf_invert(e, einv, d) != 0) { free(e); free(einv); return OXRS_ERR_SINGULAR; }
  /* row t of the rebuilt set = gen[t] * Einv (data rows: gen[t] = unit vector).
   * All outputs are computed into scratch first: order-independent. */
  uint8_t *coef = (uint8_t *)malloc((size_t)d);
  uint8_t *out = (uint8_t *)calloc((size_t)n_need, size ? size : 1);
  for (int q = 0; q < n_need; q++) {
    int t = need[q];
    for (int i = 0; i < d; i++) {
      uint8_t c = 0;
      for (int j = 0; j < d; j++) c ^= oxrs_gf_mul(x->gen[t][j], einv[j * d + i]);
      coef[i] = c;
    }
    for (int i = 0; i < d; i++) mul_add(coef[i], vects[dp_has[i]], out + (size_t)q * size, size);
  }
  for (int q = 0; q < n_need; q++) memcpy(vects[need[q]], out + (size_t)q * size, size);
  free(out); free(coef); free(e); free(einv);
  return OXRS_OK;
}

/* xorsimd.Encode(dst, src): dst = XOR of src (dst may alias src[0]). */
static void xor_into(uint8_t *dst, const uint8_t *src, size_t n) {
  for (size_t i = 0; i < n; i++) dst[i] ^= src[i];
}

/* --------------------------------------------------------------- XRS ops */
/* xrs.go:103-128 Encode */
int oxrs_encode(const oxrs *x, uint8_t *const *vects, int n, size_t size) {
  if (n < 1) return OXRS_ERR_ILLEGAL_VECTS;
  int err = check_size(size);
  if (err) return err;
  if (n != x->d + x->p) return OXRS_ERR_ILLEGAL_VECTS;
  oxrs_rs_encode(x, vects, size); /* xrs.go:112 */
  size_t half = size / 2;
  for (int bi = x->d + 1; bi < x->d + x->p; bi++) /* xrs.go:119-126 */
    for (int t = 0; t < x->xs_len[bi]; t++) xor_into(vects[bi] + half, vects[x->xs[bi][t]], half);
  return OXRS_OK;
}

/* xrs.go:175-221 ReconstOne */
int oxrs_reconst_one(const oxrs *x, uint8_t *const *vects, int n, size_t size, int k) {
  int d = x->d;
  int err = check_size(size);
  if (err) return err;
  int a_need[OXRS_MAX_VECTS], a_len, b_need[2];
  err = oxrs_get_need_vects(x, k, a_need, &a_len, b_need);
  if (err) return err;
  if (n != x->d + x->p) return OXRS_ERR_ILLEGAL_VECTS;
  size_t half = size / 2;
  uint8_t *bv[OXRS_MAX_VECTS];
  for (int i = 0; i < n; i++) bv[i] = vects[i] + half; /* :188-192 */
  int dp_has[OXRS_MAX_VECTS];
  for (int i = 0; i < d; i++) dp_has[i] = i;
  dp_has[k] = d; /* :195-199 */
  int bi = b_need[1];
  uint8_t *brs = (uint8_t *)calloc(1, half ? half : 1); /* :203-204 */
  bv[bi] = brs;
  int need[2] = {k, bi};
  err = oxrs_rs_reconst(x, bv, half, dp_has, d, need, 2); /* :205 */
  if (err) { free(brs); return err; }
  /* :213-219  a_k = vects[bi][half:] ^ bRS ^ XOR(a_need) */
  uint8_t *ak = vects[k];
  memcpy(ak, vects[bi] + half, half);
  xor_into(ak, brs, half);
  for (int t = 0; t < a_len; t++) xor_into(ak, vects[a_need[t]], half);
  free(brs);
  return OXRS_OK;
}

static int is_in(int e, const int *s, int n) {
  for (int i = 0; i < n; i++)
    if (s[i] == e) return 1;
  return 0;
}

/* xrs.go:305-320 retrieveRS */
int oxrs_retrieve_rs(const oxrs *x, uint8_t *const *vects, int n, size_t size,
                     const int *dp_has, int n_has) {
  (void)n;
  size_t half = size / 2;
  for (int i = 0; i < n_has; i++) {
    int h = dp_has[i];
    if (h > x->d && h < OXRS_MAX_VECTS)
      for (int t = 0; t < x->xs_len[h]; t++) xor_into(vects[h] + half, vects[x->xs[h][t]], half);
  }
  return OXRS_OK;
}

/* xrs.go:236-301 Reconst */
int oxrs_reconst(const oxrs *x, uint8_t *const *vects, int n, size_t size,
                 const int *dp_has, int n_has, const int *need, int n_need) {
  int d = x->d, p = x->p;
  if (n_need == 1 && need[0] < d) return oxrs_reconst_one(x, vects, n, size, need[0]); /* :238-240 */
  int err = check_size(size);
  if (err) return err;
  if (n != d + p) return OXRS_ERR_ILLEGAL_VECTS;
  size_t half = size / 2;
  uint8_t *av[OXRS_MAX_VECTS], *bv[OXRS_MAX_VECTS];
  for (int i = 0; i < n; i++) { av[i] = vects[i]; bv[i] = vects[i] + half; }
  int a_lost[OXRS_MAX_VECTS], n_lost = 0; /* :253-258 */
  for (int i = 0; i < d + p; i++)
    if (!is_in(i, dp_has, n_has)) a_lost[n_lost++] = i;
  err = oxrs_rs_reconst(x, av, half, dp_has, n_has, a_lost, n_lost); /* :259 */
  if (err) return err;
  oxrs_retrieve_rs(x, vects, n, size, dp_has, n_has);               /* :265 */
  err = oxrs_rs_reconst(x, bv, half, dp_has, n_has, need, n_need);   /* :275 */
  if (err) return err;
  /* :281-297  re-piggyback needed parity other than d */
  for (int q = 0; q < n_need; q++) {
    int i = need[q];
    if (i >= d && i != d)
      for (int t = 0; t < x->xs_len[i]; t++) xor_into(vects[i] + half, vects[x->xs[i][t]], half);
  }
  return OXRS_OK;
}

/* xrs.go:324-346 Update.  row outside [0,d) is rejected before any write
 * (the dependency's own check is not visible offline). */
int oxrs_update(const oxrs *x, const uint8_t *old_data, const uint8_t *new_data,
                size_t size, int row, uint8_t *const *parity) {
  int err = check_size(size);
  if (err) return err;
  if (row < 0 || row >= x->d) return OXRS_ERR_ILLEGAL_DATA_INDEX;
  uint8_t *delta = (uint8_t *)malloc(size ? size : 1);
  for (size_t i = 0; i < size; i++) delta[i] = old_data[i] ^ new_data[i];
  for (int r = 0; r < x->p; r++) mul_add(x->gen[x->d + r][row], delta, parity[r], size); /* :331 */
  int a_need[OXRS_MAX_VECTS], a_len, b_need[2];
  oxrs_get_need_vects(x, row, a_need, &a_len, b_need); /* :336 */
  size_t half = size / 2;
  xor_into(parity[b_need[1] - x->d] + half, delta, half); /* :340-344 */
  free(delta);
  return OXRS_OK;
}

/* xrs.go:363-387 Replace */
int oxrs_replace(const oxrs *x, uint8_t *const *data, const int *rows, int n,
                 size_t size, uint8_t *const *parity) {
  if (n < 1) return OXRS_ERR_ILLEGAL_VECTS;
  int err = check_size(size);
  if (err) return err;
  if (n > x->d) return OXRS_ERR_ILLEGAL_VECTS;
  for (int i = 0; i < n; i++)
    if (rows[i] < 0 || rows[i] >= x->d) return OXRS_ERR_ILLEGAL_DATA_INDEX;
  for (int r = 0; r < x->p; r++) /* :370 */
    for (int i = 0; i < n; i++) mul_add(x->gen[x->d + r][rows[i]], data[i], parity[r], size);
  size_t half = size / 2;
  for (int i = 0; i < n; i++) { /* :375-385 */
    int a_need[OXRS_MAX_VECTS], a_len, b_need[2];
    oxrs_get_need_vects(x, rows[i], a_need, &a_len, b_need);
    xor_into(parity[b_need[1] - x->d] + half, data[i], half);
  }
  return OXRS_OK;
}

/* ============================================ CPU baseline (AVX-512BW / AVX2) */
typedef struct { uint8_t lo[16], hi[16]; } nib_tab;

static void make_nib(uint8_t c, nib_tab *t) {
  for (int v = 0; v < 16; v++) {
    t->lo[v] = oxrs_gf_mul(c, (uint8_t)v);
    t->hi[v] = oxrs_gf_mul(c, (uint8_t)(v << 4));
  }
}

/* SIMD level of the baseline: 2 = AVX-512BW (64-byte vpshufb), 1 = AVX2,
 * 0 = scalar.  The reference's dependency picks the widest path the CPU has
 * (templexxx/cpu feature detection); OXRS_SIMD=avx2 or
 * =scalar caps it for A/B runs. */
int oxrs_simd_level(void) {
  static int hw = -1;
  if (hw < 0) {
    int l = 0;
#if defined(__x86_64__)
    __builtin_cpu_init();
    if (__builtin_cpu_supports("avx2")) l = 1;
    if (__builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw")) l = 2;
#endif
    hw = l;
  }
  const char *cap = getenv("OXRS_SIMD");  /* read per call: tests switch it */
  if (cap && strcmp(cap, "scalar") == 0) return 0;
  if (cap && strcmp(cap, "avx2") == 0 && hw > 1) return 1;
  return hw;
}

int oxrs_simd_available(void) { return oxrs_simd_level() > 0; }

#if defined(__x86_64__)
/* out[r] (=|^=) sum_j tab[r*nin+j] * in[j], r < nout, over n bytes (n % 32 == 0
 * handled by the vector loop, remainder scalar). */
__attribute__((target("avx2"))) static void gf_matmul_avx2(const nib_tab *tab, int nout, int nin,
                                                             const uint8_t *const *in,
                                                             uint8_t *const *out, size_t n,
                                                             int acc_out) {
  const __m256i mask = _mm256_set1_epi8(0x0f);
  size_t i = 0;
  for (; i + 32 <= n; i += 32) {
    __m256i acc[8];
    for (int r = 0; r < nout; r++)
      acc[r] = acc_out ? _mm256_loadu_si256((const __m256i *)(out[r] + i)) : _mm256_setzero_si256();
    for (int j = 0; j < nin; j++) {
      __m256i v = _mm256_loadu_si256((const __m256i *)(in[j] + i));
      __m256i lo = _mm256_and_si256(v, mask);
      __m256i hi = _mm256_and_si256(_mm256_srli_epi64(v, 4), mask);
      for (int r = 0; r < nout; r++) {
        const nib_tab *t = &tab[r * nin + j];
        __m256i tl = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)t->lo));
        __m256i th = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)t->hi));
        acc[r] = _mm256_xor_si256(acc[r], _mm256_xor_si256(_mm256_shuffle_epi8(tl, lo),
                                                           _mm256_shuffle_epi8(th, hi)));
      }
    }
    for (int r = 0; r < nout; r++) _mm256_storeu_si256((__m256i *)(out[r] + i), acc[r]);
  }
  for (; i < n; i++) {
    for (int r = 0; r < nout; r++) {
      uint8_t a = acc_out ? out[r][i] : 0;
      for (int j = 0; j < nin; j++) {
        uint8_t s = in[j][i];
        a ^= tab[r * nin + j].lo[s & 15] ^ tab[r * nin + j].hi[s >> 4];
      }
      out[r][i] = a;
    }
  }
}

__attribute__((target("avx2"))) static void xor_avx2(uint8_t *dst, const uint8_t *src, size_t n) {
  size_t i = 0;
  for (; i + 32 <= n; i += 32) {
    __m256i a = _mm256_loadu_si256((const __m256i *)(dst + i));
    __m256i b = _mm256_loadu_si256((const __m256i *)(src + i));
    _mm256_storeu_si256((__m256i *)(dst + i), _mm256_xor_si256(a, b));
  }
  for (; i < n; i++) dst[i] ^= src[i];
}

/* The same two loops on 64-byte zmm registers (AVX-512BW vpshufb); the
 * three-way XOR is one vpternlogq. */
__attribute__((target("avx512f,avx512bw"))) static void gf_matmul_avx512(
    const nib_tab *tab, int nout, int nin, const uint8_t *const *in, uint8_t *const *out,
    size_t n, int acc_out) {
  const __m512i mask = _mm512_set1_epi8(0x0f);
  size_t i = 0;
  for (; i + 64 <= n; i += 64) {
    __m512i acc[8];
    for (int r = 0; r < nout; r++)
      acc[r] = acc_out ? _mm512_loadu_si512((const void *)(out[r] + i)) : _mm512_setzero_si512();
    for (int j = 0; j < nin; j++) {
      __m512i v = _mm512_loadu_si512((const void *)(in[j] + i));
      __m512i lo = _mm512_and_si512(v, mask);
      __m512i hi = _mm512_and_si512(_mm512_srli_epi64(v, 4), mask);
      for (int r = 0; r < nout; r++) {
        const nib_tab *t = &tab[r * nin + j];
        __m512i tl = _mm512_broadcast_i32x4(_mm_loadu_si128((const __m128i *)t->lo));
        __m512i th = _mm512_broadcast_i32x4(_mm_loadu_si128((const __m128i *)t->hi));
        acc[r] = _mm512_ternarylogic_epi64(acc[r], _mm512_shuffle_epi8(tl, lo),
                                           _mm512_shuffle_epi8(th, hi), 0x96);
      }
    }
    for (int r = 0; r < nout; r++) _mm512_storeu_si512((void *)(out[r] + i), acc[r]);
  }
  if (i < n) {
    const uint8_t *in2[OXRS_MAX_VECTS];
    uint8_t *out2[8];
    for (int j = 0; j < nin; j++) in2[j] = in[j] + i;
    for (int r = 0; r < nout; r++) out2[r] = out[r] + i;
    gf_matmul_avx2(tab, nout, nin, in2, out2, n - i, acc_out);
  }
}

__attribute__((target("avx512f,avx512bw"))) static void xor_avx512(uint8_t *dst,
                                                                    const uint8_t *src, size_t n) {
  size_t i = 0;
  for (; i + 64 <= n; i += 64) {
    __m512i a = _mm512_loadu_si512((const void *)(dst + i));
    __m512i b = _mm512_loadu_si512((const void *)(src + i));
    _mm512_storeu_si512((void *)(dst + i), _mm512_xor_si512(a, b));
  }
  xor_avx2(dst + i, src + i, n - i);
}
#endif

static void gf_matmul_scalar(const nib_tab *tab, int nout, int nin, const uint8_t *const *in,
                             uint8_t *const *out, size_t n, int acc_out) {
  for (size_t i = 0; i < n; i++)
    for (int r = 0; r < nout; r++) {
      uint8_t a = acc_out ? out[r][i] : 0;
      for (int j = 0; j < nin; j++) {
        uint8_t s = in[j][i];
        a ^= tab[r * nin + j].lo[s & 15] ^ tab[r * nin + j].hi[s >> 4];
      }
      out[r][i] = a;
    }
}

/* out[r] = sum_j tab[r][j] * in[j]; acc_out: out[r] ^= that sum. */
static void gf_matmul_x(const nib_tab *tab, int nout, int nin, const uint8_t *const *in,
                        uint8_t *const *out, size_t n, int acc_out) {
#if defined(__x86_64__)
  const int level = oxrs_simd_level();
  if (level > 0) {
    for (int r0 = 0; r0 < nout; r0 += 8) {
      int nr = nout - r0 < 8 ? nout - r0 : 8;
      if (level > 1) gf_matmul_avx512(tab + (size_t)r0 * nin, nr, nin, in, out + r0, n, acc_out);
      else gf_matmul_avx2(tab + (size_t)r0 * nin, nr, nin, in, out + r0, n, acc_out);
    }
    return;
  }
#endif
  gf_matmul_scalar(tab, nout, nin, in, out, n, acc_out);
}

static void gf_matmul(const nib_tab *tab, int nout, int nin, const uint8_t *const *in,
                      uint8_t *const *out, size_t n) {
  gf_matmul_x(tab, nout, nin, in, out, n, 0);
}

static void xor_fast(uint8_t *dst, const uint8_t *src, size_t n) {
#if defined(__x86_64__)
  const int level = oxrs_simd_level();
  if (level > 1) { xor_avx512(dst, src, n); return; }
  if (level > 0) { xor_avx2(dst, src, n); return; }
#endif
  xor_into(dst, src, n);
}

/* Cache-blocked like the reference's dependency: the RS pass walks the vector
 * in 16 KiB position blocks, then the piggyback pass (xrs.go:118-126). */
#define OXRS_BLOCK 16384

typedef struct {
  const oxrs *x;
  uint8_t *base;
  size_t size, stride;
  long s0, s1;
  int k; /* reconst_one lost index */
  const nib_tab *tab;
  int ntab_out;
} job_t;

static void *encode_worker(void *arg) {
  job_t *jb = (job_t *)arg;
  const oxrs *x = jb->x;
  int d = x->d, p = x->p;
  size_t size = jb->size, half = size / 2;
  for (long s = jb->s0; s < jb->s1; s++) {
    uint8_t *st = jb->base + (size_t)s * jb->stride;
    for (size_t off = 0; off < size; off += OXRS_BLOCK) {
      size_t n = size - off < OXRS_BLOCK ? size - off : OXRS_BLOCK;
      const uint8_t *in[OXRS_MAX_VECTS];
      uint8_t *out[OXRS_MAX_VECTS];
      for (int j = 0; j < d; j++) in[j] = st + (size_t)j * size + off;
      for (int r = 0; r < p; r++) out[r] = st + (size_t)(d + r) * size + off;
      gf_matmul(jb->tab, p, d, in, out, n);
    }
    for (int bi = d + 1; bi < d + p; bi++)
      for (int t = 0; t < x->xs_len[bi]; t++)
        xor_fast(st + (size_t)bi * size + half, st + (size_t)x->xs[bi][t] * size, half);
  }
  return NULL;
}

static int run_jobs(void *(*fn)(void *), job_t *proto, long n_stripes, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t th[256];
  job_t jobs[256];
  long per = (n_stripes + threads - 1) / threads;
  int started = 0;
  for (int t = 0; t < threads; t++) {
    jobs[t] = *proto;
    jobs[t].s0 = t * per;
    jobs[t].s1 = (t + 1) * per < n_stripes ? (t + 1) * per : n_stripes;
    if (jobs[t].s0 >= jobs[t].s1) break;
    if (threads == 1) { fn(&jobs[t]); started = 0; break; }
    pthread_create(&th[t], NULL, fn, &jobs[t]);
    started++;
  }
  for (int t = 0; t < started; t++) pthread_join(th[t], NULL);
  return OXRS_OK;
}

int oxrs_encode_batch(const oxrs *x, uint8_t *base, size_t size, size_t stripe_stride,
                      long n_stripes, int threads) {
  if (size & 1) return OXRS_ERR_SIZE_NOT_EVEN;
  int d = x->d, p = x->p;
  nib_tab *tab = (nib_tab *)malloc(sizeof(nib_tab) * (size_t)d * p);
  for (int r = 0; r < p; r++)
    for (int j = 0; j < d; j++) make_nib(x->gen[d + r][j], &tab[r * d + j]);
  job_t proto = {x, base, size, stripe_stride, 0, 0, 0, tab, p};
  run_jobs(encode_worker, &proto, n_stripes, threads);
  free(tab);
  return OXRS_OK;
}

/* ReconstOne baseline: one GF pass over the d surviving b-halves producing
 * b_k and bRS (xrs.go:205), then the a_k XOR pass (xrs.go:213-219). */
typedef struct {
  nib_tab tab[2 * OXRS_MAX_VECTS];
  int has[OXRS_MAX_VECTS];
  int a_need[OXRS_MAX_VECTS], a_len, bi;
} r1_plan;

static void *reconst_one_worker(void *arg) {
  job_t *jb = (job_t *)arg;
  const oxrs *x = jb->x;
  const r1_plan *pl = (const r1_plan *)jb->tab;
  int d = x->d, k = jb->k;
  size_t size = jb->size, half = size / 2;
  uint8_t *brs = (uint8_t *)malloc(OXRS_BLOCK);
  for (long s = jb->s0; s < jb->s1; s++) {
    uint8_t *st = jb->base + (size_t)s * jb->stride;
    for (size_t off = 0; off < half; off += OXRS_BLOCK) {
      size_t n = half - off < OXRS_BLOCK ? half - off : OXRS_BLOCK;
      const uint8_t *in[OXRS_MAX_VECTS];
      uint8_t *out[2];
      for (int i = 0; i < d; i++) in[i] = st + (size_t)pl->has[i] * size + half + off;
      out[0] = st + (size_t)k * size + half + off;
      out[1] = brs;
      gf_matmul(pl->tab, 2, d, in, out, n);
      uint8_t *ak = st + (size_t)k * size + off;
      memcpy(ak, st + (size_t)pl->bi * size + half + off, n);
      xor_fast(ak, brs, n);
      for (int t = 0; t < pl->a_len; t++) xor_fast(ak, st + (size_t)pl->a_need[t] * size + off, n);
    }
  }
  free(brs);
  return NULL;
}

int oxrs_reconst_one_batch(const oxrs *x, uint8_t *base, size_t size, size_t stripe_stride,
                           long n_stripes, int k, int threads) {
  if (size & 1) return OXRS_ERR_SIZE_NOT_EVEN;
  int d = x->d;
  r1_plan *pl = (r1_plan *)calloc(1, sizeof(r1_plan));
  int b_need[2];
  int err = oxrs_get_need_vects(x, k, pl->a_need, &pl->a_len, b_need);
  if (err) { free(pl); return err; }
  pl->bi = b_need[1];
  for (int i = 0; i < d; i++) pl->has[i] = i;
  pl->has[k] = d;
  uint8_t *e = (uint8_t *)malloc((size_t)d * d), *einv = (uint8_t *)malloc((size_t)d * d);
  for (int i = 0; i < d; i++)
    for (int j = 0; j < d; j++) e[i * d + j] = x->gen[pl->has[i]][j];
  if (gf_invert(e, einv, d)) { free(e); free(einv); free(pl); return OXRS_ERR_SINGULAR; }
  for (int i = 0; i < d; i++) {
    uint8_t c = 0;
    for (int j = 0; j < d; j++) c ^= oxrs_gf_mul(x->gen[pl->bi][j], einv[j * d + i]);
    make_nib(einv[k * d + i], &pl->tab[i]);
    make_nib(c, &pl->tab[d + i]);
  }
  free(e); free(einv);
  job_t proto = {x, base, size, stripe_stride, 0, 0, k, (const nib_tab *)pl, 2};
  run_jobs(reconst_one_worker, &proto, n_stripes, threads);
  free(pl);
  return OXRS_OK;
}

/* Update baseline over a batch (BASELINE config 4; reference benchmark
 * xrs_test.go:600-625).  Stripe s holds [old, new, parity 0..p-1] vects of
 * `size` bytes at base + s * stripe_stride.  The reference's two passes:
 * rs.Update (xrs.go:331: delta = old ^ new, parity_r ^= G[r][row] * delta, in
 * cache blocks), then the piggyback pass over the a-half (xrs.go:340-344:
 * bv ^= old[:half] ^ new[:half]). */
static void *update_worker(void *arg) {
  job_t *jb = (job_t *)arg;
  const oxrs *x = jb->x;
  int d = x->d, p = x->p, row = jb->k;
  size_t size = jb->size, half = size / 2;
  uint8_t *delta = (uint8_t *)malloc(OXRS_BLOCK);
  int a_need[OXRS_MAX_VECTS], a_len, b_need[2];
  oxrs_get_need_vects(x, row, a_need, &a_len, b_need);
  for (long s = jb->s0; s < jb->s1; s++) {
    uint8_t *st = jb->base + (size_t)s * jb->stride;
    const uint8_t *old = st, *nw = st + size;
    uint8_t *par[OXRS_MAX_VECTS];
    for (int r = 0; r < p; r++) par[r] = st + (size_t)(2 + r) * size;
    for (size_t off = 0; off < size; off += OXRS_BLOCK) {
      size_t n = size - off < OXRS_BLOCK ? size - off : OXRS_BLOCK;
      memcpy(delta, old + off, n);
      xor_fast(delta, nw + off, n);
      const uint8_t *in[1] = {delta};
      uint8_t *out[OXRS_MAX_VECTS];
      for (int r = 0; r < p; r++) out[r] = par[r] + off;
      gf_matmul_x(jb->tab, p, 1, in, out, n, 1);
    }
    uint8_t *bv = par[b_need[1] - d] + half;
    xor_fast(bv, old, half);
    xor_fast(bv, nw, half);
  }
  free(delta);
  return NULL;
}

int oxrs_update_batch(const oxrs *x, uint8_t *base, size_t size, size_t stripe_stride,
                      long n_stripes, int row, int threads) {
  if (size & 1) return OXRS_ERR_SIZE_NOT_EVEN;
  if (row < 0 || row >= x->d) return OXRS_ERR_ILLEGAL_DATA_INDEX;
  nib_tab tab[OXRS_MAX_VECTS];
  for (int r = 0; r < x->p; r++) make_nib(x->gen[x->d + r][row], &tab[r]);
  job_t proto = {x, base, size, stripe_stride, 0, 0, row, tab, x->p};
  run_jobs(update_worker, &proto, n_stripes, threads);
  return OXRS_OK;
}

/* Replace baseline over a batch (BASELINE config 4, Replace(n); reference
 * benchmark xrs_test.go:627-680).  Stripe s holds [data 0..n-1, parity
 * 0..p-1]; rows[i] is data i's row.  rs.Replace (xrs.go:370: parity_r ^=
 * sum_i G[r][rows_i] * data_i, in cache blocks), then one piggyback pass per
 * row (xrs.go:375-385). */
typedef struct {
  nib_tab tab[8 * OXRS_MAX_VECTS];
  int n, bi[OXRS_MAX_VECTS];
} rep_plan;

static void *replace_worker(void *arg) {
  job_t *jb = (job_t *)arg;
  const oxrs *x = jb->x;
  const rep_plan *pl = (const rep_plan *)jb->tab;
  int d = x->d, p = x->p, nr = pl->n;
  size_t size = jb->size, half = size / 2;
  for (long s = jb->s0; s < jb->s1; s++) {
    uint8_t *st = jb->base + (size_t)s * jb->stride;
    uint8_t *par[OXRS_MAX_VECTS];
    for (int r = 0; r < p; r++) par[r] = st + (size_t)(nr + r) * size;
    for (size_t off = 0; off < size; off += OXRS_BLOCK) {
      size_t n = size - off < OXRS_BLOCK ? size - off : OXRS_BLOCK;
      const uint8_t *in[OXRS_MAX_VECTS];
      uint8_t *out[OXRS_MAX_VECTS];
      for (int i = 0; i < nr; i++) in[i] = st + (size_t)i * size + off;
      for (int r = 0; r < p; r++) out[r] = par[r] + off;
      gf_matmul_x(pl->tab, p, nr, in, out, n, 1);
    }
    for (int i = 0; i < nr; i++) xor_fast(par[pl->bi[i] - d] + half, st + (size_t)i * size, half);
  }
  return NULL;
}

int oxrs_replace_batch(const oxrs *x, uint8_t *base, size_t size, size_t stripe_stride,
                       long n_stripes, const int *rows, int n, int threads) {
  if (n < 1 || n > x->d || n > 8) return OXRS_ERR_ILLEGAL_VECTS;
  if (size & 1) return OXRS_ERR_SIZE_NOT_EVEN;
  rep_plan *pl = (rep_plan *)calloc(1, sizeof(rep_plan));
  pl->n = n;
  for (int i = 0; i < n; i++) {
    if (rows[i] < 0 || rows[i] >= x->d) { free(pl); return OXRS_ERR_ILLEGAL_DATA_INDEX; }
    int a_need[OXRS_MAX_VECTS], a_len, b_need[2];
    oxrs_get_need_vects(x, rows[i], a_need, &a_len, b_need);
    pl->bi[i] = b_need[1];
    for (int r = 0; r < x->p; r++) make_nib(x->gen[x->d + r][rows[i]], &pl->tab[r * n + i]);
  }
  job_t proto = {x, base, size, stripe_stride, 0, 0, 0, (const nib_tab *)pl, x->p};
  run_jobs(replace_worker, &proto, n_stripes, threads);
  free(pl);
  return OXRS_OK;
}
