/*
 * xrs_oracle.h -- CPU restatement of templexxx/xrs (TEST INFRASTRUCTURE ONLY).
 *
 * This header and oracle/xrs_oracle.c are the CHECKER for the HIP product path
 * and the timed CPU baseline in bench.py.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load them.  The product library
 * (xrs_amd/libxrs_hip.so) never links or calls anything declared here.
 *
 * Parity pinning: the reference is Go (no Go toolchain in this image) and its
 * arithmetic lives in two un-vendored modules, github.com/templexxx/reedsolomon
 * v1.1.3 (go.mod:6) and github.com/templexxx/xorsimd v0.1.1 (go.mod:7).  The
 * restatement below is pinned by the reference's only known-answer test,
 * TestXRS_Encode (/root/reference/xrs_test.go:102-122), and by the property
 * tests of xrs_test.go ported to tests/.
 */
#ifndef XRS_ORACLE_H
#define XRS_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OXRS_MAX_VECTS 256

/* Error codes; texts mirror xrs.go where the reference defines them. */
enum {
  OXRS_OK = 0,
  OXRS_ERR_ILLEGAL_PARITY = -1,   /* xrs.go:57  "illegal parity"              */
  OXRS_ERR_SIZE_NOT_EVEN = -2,    /* xrs.go:133 "vect size not even: %d"      */
  OXRS_ERR_ILLEGAL_DATA_INDEX = -3, /* xrs.go:149 "illegal data index: %d"    */
  OXRS_ERR_ILLEGAL_VECTS = -4,    /* [dep] reedsolomon config / vect count    */
  OXRS_ERR_TOO_FEW_SURVIVORS = -5,/* [dep] reedsolomon: len(dpHas) < d        */
  OXRS_ERR_ILLEGAL_INDEX = -6,    /* [dep] reedsolomon: index out of range    */
  OXRS_ERR_SINGULAR = -7,         /* [dep] reedsolomon: survivor matrix singular */
};

typedef struct oxrs {
  int d, p;
  uint8_t gen[OXRS_MAX_VECTS][OXRS_MAX_VECTS]; /* (d+p) x d encode matrix */
  int xs_len[OXRS_MAX_VECTS];                  /* XORSet[d+1+t] length, t<p-1 */
  int xs[OXRS_MAX_VECTS][OXRS_MAX_VECTS];      /* XORSet[d+1+t][k]            */
} oxrs;

/* GF(2^8) / 0x11d primitives */
uint8_t oxrs_gf_mul(uint8_t a, uint8_t b);
uint8_t oxrs_gf_inv(uint8_t a);

size_t oxrs_sizeof(void);
int oxrs_new(int d, int p, oxrs *x);
int oxrs_get_need_vects(const oxrs *x, int k, int *a_need, int *a_len, int b_need[2]);
int oxrs_encode(const oxrs *x, uint8_t *const *vects, int n, size_t size);
int oxrs_reconst_one(const oxrs *x, uint8_t *const *vects, int n, size_t size, int k);
int oxrs_reconst(const oxrs *x, uint8_t *const *vects, int n, size_t size,
                 const int *dp_has, int n_has, const int *need, int n_need);
int oxrs_retrieve_rs(const oxrs *x, uint8_t *const *vects, int n, size_t size,
                     const int *dp_has, int n_has);
int oxrs_update(const oxrs *x, const uint8_t *old_data, const uint8_t *new_data,
                size_t size, int row, uint8_t *const *parity);
int oxrs_replace(const oxrs *x, uint8_t *const *data, const int *rows, int n,
                 size_t size, uint8_t *const *parity);

/* Plain-RS restatement of the dependency (templexxx/reedsolomon call sites). */
int oxrs_rs_encode(const oxrs *x, uint8_t *const *vects, size_t size);
int oxrs_rs_reconst(const oxrs *x, uint8_t *const *vects, size_t size,
                    const int *dp_has, int n_has, const int *need, int n_need);

/* ---- CPU baseline (the reference's algorithm: 4-bit split tables, AVX-512BW or AVX2 vpshufb,
 *      two passes like xrs.go Encode: RS then piggyback XOR) over a contiguous
 *      batch: stripe s, shard i at base + s*stripe_stride + i*size. ---- */
int oxrs_simd_available(void);
int oxrs_simd_level(void); /* 2 = AVX-512BW, 1 = AVX2, 0 = scalar */
int oxrs_encode_batch(const oxrs *x, uint8_t *base, size_t size,
                      size_t stripe_stride, long n_stripes, int threads);
int oxrs_reconst_one_batch(const oxrs *x, uint8_t *base, size_t size,
                           size_t stripe_stride, long n_stripes, int k, int threads);
/* Update(row): stripe s = [old, new, parity 0..p-1]; Replace(rows[0..n)):
 * stripe s = [data 0..n-1, parity 0..p-1] (n <= 8). */
int oxrs_update_batch(const oxrs *x, uint8_t *base, size_t size, size_t stripe_stride,
                      long n_stripes, int row, int threads);
int oxrs_replace_batch(const oxrs *x, uint8_t *base, size_t size, size_t stripe_stride,
                       long n_stripes, const int *rows, int n, int threads);

#ifdef __cplusplus
}
#endif
#endif
