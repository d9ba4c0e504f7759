// kernels.hip -- gfx950 (MI355X, CDNA4) kernels for the X-Reed-Solomon codec.
//
// Hot path of templexxx/xrs: the GF(2^8) Cauchy multiply-accumulate over shard
// bytes (reedsolomon RS.Encode/Reconst/Update/Replace, called from
// /root/reference/xrs.go:112,205,259,275,331,370) plus the a/b-half piggyback
// XOR (xorsimd call sites xrs.go:125,219,295,316,344,383).
//
// Design (DESIGN.md has the roofline arithmetic):
//  * Pure HBM streaming, integer VALU work; no MFMA and no LDS on the data path.
//  * Each lane owns 16 bytes at offset o of the a-half AND the same 16 bytes of
//    the b-half (o + H) of every row it touches, so the piggyback XOR uses a-half
//    bytes the lane already holds: RS + piggyback is one pass over HBM.
//  * Loads/stores are global_load/store_dwordx4: one wave moves 1 KiB
//    contiguous per instruction per row (full 128-B lines).
//  * GF multiply by a constant c = three v_perm_b32 byte lookups (8-, 8- and
//    4-entry tables indexed by bits 0-2, 3-5, 6-7) XORed with v_bitop3_b32.
//    One v_perm looks up 4 bytes; the table dwords come from kernel-argument
//    SGPRs (gfx950 allows one SGPR operand per VALU op, the other half of an
//    8-entry table is moved to a VGPR once per 16 bytes).
//  * The headline shapes (12+4 Encode, 12+4 ReconstOne) are compile-time so
//    every load is in flight before the first multiply; other shapes use
//    runtime-count variants.  Misaligned / odd sizes take a byte-granular path.
#include <hip/hip_runtime.h>

#include <cxxabi.h>

#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "gf256.h"
#include "xrs_plan.h"

// Build parts: the Makefile compiles this file once per XRS_PART (1: launch
// trace + pair kernels, 2: staged, 3: update_rows, 4: rows), so the gfx950
// code generation of the kernel families runs in parallel.  Without
// XRS_PART (tools/, the host-sanitizer test build) one unit holds everything.
#ifndef XRS_PART
#define XRS_PART 0
#endif
#define XRS_HAS_PART(n) (XRS_PART == 0 || XRS_PART == (n))

namespace xrs {
namespace {

constexpr int kDyn = -1;  // count known only at run time
#ifndef XRS_BLOCK
#define XRS_BLOCK 256  // threads per block (-DXRS_BLOCK=... for A/B builds only)
#endif
constexpr int kBlock = XRS_BLOCK;
constexpr uint64_t kMaxBlocks = 0x7fffffffu;  // 1-D grid limit
constexpr uint64_t kLatencyGrid = 256;         // blocks: one per CU (MI355X: 256 CUs)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// Global (address space 1) views: global_load/store instead of flat_*.
typedef __attribute__((address_space(1))) u32x4 gu32x4;
typedef __attribute__((address_space(1))) uint8_t gu8;

__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // a ^ b ^ c
}

struct Sel {
  uint32_t s0, s1, s2;
};

__device__ __forceinline__ Sel sel_of(uint32_t x) {
  return {x & 0x07070707u, (x >> 3) & 0x07070707u, (x >> 6) & 0x03030303u};
}

// c * x on four bytes.  v_perm_b32(S0=hi, S1=lo, sel): selector byte 0..3 picks
// a byte of lo, 4..7 a byte of hi.
__device__ __forceinline__ uint32_t gmul(const GfTab& t, const Sel& s) {
  return x3(__builtin_amdgcn_perm(t.hi0, t.lo0, s.s0), __builtin_amdgcn_perm(t.hi1, t.lo1, s.s1),
            __builtin_amdgcn_perm(0u, t.top, s.s2));
}

// ---- fragment load/store: W dwords per lane per row ------------------------
// VEC: one 16-byte dwordx4 access (address 16-byte aligned), nontemporal:
// every shard byte is touched exactly once per launch (measured on MI355X:
// nt loads + nt stores +3% Encode, +7..11% ReconstOne; tools/kbench.hip).
// !VEC: nb (1..4) single-byte accesses (any alignment, ragged tail).
#ifndef XRS_LOAD_NT
#define XRS_LOAD_NT 1  // -DXRS_LOAD_NT=0: temporal 16-byte loads (A/B builds only)
#endif
template <bool VEC>
__device__ __forceinline__ void ld(uint32_t* v, uint64_t addr, int nb) {
  if constexpr (VEC) {
#if XRS_LOAD_NT
    const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const gu32x4*>(addr));
#else
    const u32x4 t = *reinterpret_cast<const gu32x4*>(addr);
#endif
    v[0] = t.x;
    v[1] = t.y;
    v[2] = t.z;
    v[3] = t.w;
  } else {
    const gu8* p = reinterpret_cast<const gu8*>(addr);
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (i < nb) x |= static_cast<uint32_t>(p[i]) << (8 * i);
    v[0] = x;
  }
}

template <bool VEC>
__device__ __forceinline__ void st(const uint32_t* v, uint64_t addr, int nb) {
  if constexpr (VEC) {
    u32x4 t;
    t.x = v[0];
    t.y = v[1];
    t.z = v[2];
    t.w = v[3];
    __builtin_nontemporal_store(t, reinterpret_cast<gu32x4*>(addr));
  } else {
    gu8* p = reinterpret_cast<gu8*>(addr);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (i < nb) p[i] = static_cast<uint8_t>(v[0] >> (8 * i));
  }
}

__device__ __forceinline__ uint64_t row_addr(const RowRef& r, uint64_t stripe, uint64_t off) {
  return r.ptr + stripe * r.stripe_stride + off;
}

// An indirect row (xrs_plan.h kRowInd): r.ptr is the address of stripe 0's
// entry in a table of row addresses (device-readable memory, e.g. the queue's
// pinned row tables), one entry every stripe_stride bytes.
__device__ __forceinline__ uint64_t row_base_ind(const RowRef& r, uint64_t stripe) {
  typedef __attribute__((address_space(1))) const uint64_t gu64;
  return *reinterpret_cast<gu64*>(r.ptr + stripe * (r.stripe_stride & ~kRowInd));
}

// ---- XCD-aware block order -------------------------------------------------
// The dispatcher hands block i to XCD i % 8 (MI355X: 8 XCDs x 32 CUs, one L2
// each).  Block order maps hardware block b to the logical block it works on:
// groups of 8*K logical blocks, each XCD taking K consecutive ones, so every
// XCD streams contiguous pieces of the batch instead of every 8th 4 KiB piece.
// K = 0 keeps the plain order.  Blocks past the last whole group keep their
// own index, so the map is a bijection on [0, nblk) for any K.  Measured on
// MI355X (tools/mapprobe.hip, profiles/r01_mapprobe3.log): Encode 8 MiB
// unpadded 4.06 -> 5.99 TB/s, ReconstOne 1 MiB unpadded 5.13 -> 5.89 TB/s,
// Encode 4 KiB 5.79 -> 6.02 TB/s, ReconstOne 4 KiB 6.10 -> 6.36 TB/s.
struct BlockOrder {
  uint32_t nblk;  // blocks in the grid
  uint32_t k;     // logical blocks per XCD per group; 0: plain order
};

__device__ __forceinline__ uint64_t logical_of(const BlockOrder& o, uint32_t b) {
  if (o.k == 0) return b;
  const uint32_t q = b >> 3, g = q / o.k;
  const uint64_t span = 8ull * o.k;
  if ((g + 1) * span > o.nblk) return b;
  return g * span + (b & 7u) * static_cast<uint64_t>(o.k) + (q - g * o.k);
}

__device__ __forceinline__ uint64_t logical_block(const BlockOrder& o) {
  return logical_of(o, blockIdx.x);
}

// ============================================================ pair kernel
// Encode / Replace / Update:  for o in [0, H):
//   dst_r[o]   (^)= sum_c coef[c][r] * src_c[o]
//   dst_r[H+o] (^)= sum_c coef[c][r] * src_c[H+o]  ^  XOR_{c: pb[c]==r} src_c[o]
template <int P, int C, bool VEC>
struct PairArgs {
  static constexpr int CM = C == kDyn ? kMaxSrc : C;
  GfTab tab[CM][P];
  RowRef src[CM];
  RowRef dst[P];
  uint32_t pbmask[P];  // bit c: XOR src_c's a-half into dst_r's b-half
  int n_src;
  BlockOrder order;
  uint64_t half;    // H
  uint64_t chunks;  // lanes per stripe
  uint64_t total;   // n_stripes * chunks
  uint64_t off0;    // first byte of each half this launch covers
  uint64_t last;    // ragged end: the last chunk starts here (overlap), else ~0
};

template <int P, int W>
__device__ __forceinline__ void pair_mac1(uint32_t (&acc_a)[P][W], uint32_t (&acc_b)[P][W],
                                          const GfTab* tab, const uint32_t* xa,
                                          const uint32_t* xb) {
#pragma unroll
  for (int w = 0; w < W; ++w) {
    const Sel sa = sel_of(xa[w]), sb = sel_of(xb[w]);
#pragma unroll
    for (int r = 0; r < P; ++r) {
      acc_a[r][w] ^= gmul(tab[r], sa);
      acc_b[r][w] ^= gmul(tab[r], sb);
    }
  }
}

template <int P, int W>
__device__ __forceinline__ void pair_mac2(uint32_t (&acc_a)[P][W], uint32_t (&acc_b)[P][W],
                                          const GfTab* tab0, const GfTab* tab1,
                                          const uint32_t* xa0, const uint32_t* xb0,
                                          const uint32_t* xa1, const uint32_t* xb1) {
  // Selectors for all W dwords of both sources first, then one output at a
  // time: each table dword moved to a VGPR is reused 2*W times.
  Sel sa0[W], sb0[W], sa1[W], sb1[W];
#pragma unroll
  for (int w = 0; w < W; ++w) {
    sa0[w] = sel_of(xa0[w]);
    sb0[w] = sel_of(xb0[w]);
    sa1[w] = sel_of(xa1[w]);
    sb1[w] = sel_of(xb1[w]);
  }
#pragma unroll
  for (int r = 0; r < P; ++r) {
#pragma unroll
    for (int w = 0; w < W; ++w) {
      acc_a[r][w] = x3(acc_a[r][w], gmul(tab0[r], sa0[w]), gmul(tab1[r], sa1[w]));
      acc_b[r][w] = x3(acc_b[r][w], gmul(tab0[r], sb0[w]), gmul(tab1[r], sb1[w]));
    }
  }
}

// acc ^= x & m  (m = all-ones or zero, wave-uniform): one v_bitop3, no branch
// (a branch per output lets the compiler turn the chain into a dynamically
// indexed accumulator array, which lands in scratch).
__device__ __forceinline__ uint32_t xor_masked(uint32_t acc, uint32_t x, uint32_t m) {
  return __builtin_amdgcn_bitop3_b32(acc, x, m, 0x78);  // a ^ (b & c)
}

// Piggyback of source c (runtime pattern): output r takes src_c's a-half if
// bit c of pbmask[r] is set.
template <int P, int W>
__device__ __forceinline__ void piggyback(uint32_t (&acc_b)[P][W], const uint32_t* pbmask, int c,
                                          const uint32_t* xa) {
#pragma unroll
  for (int r = 0; r < P; ++r) {
    const uint32_t m = 0u - ((pbmask[r] >> c) & 1u);
#pragma unroll
    for (int w = 0; w < W; ++w) acc_b[r][w] = xor_masked(acc_b[r][w], xa[w], m);
  }
}

// PLAIN: the plain block order known at compile time (no logical_block map);
// used by the 12+4 Encode from 512 KiB halves, which streams fastest in the
// plain order (launch_pair_t).  It also gives that launch, the bench's
// dominant one, its own name in rocprofv3 --stats (the 4 KiB Encode runs the
// same <4, 12, false, true, 128> shape in the XCD order).
template <int P, int C, bool ACC, bool VEC, int BS = kBlock, bool PLAIN = false>
__global__ __launch_bounds__(BS) void pair_kernel(const PairArgs<P, C, VEC> a) {
#define XRS_IND 0
#define XRS_ROW row_addr
#include "kbody_pair.h"
#undef XRS_ROW
#undef XRS_IND
}

// The pair kernel on indirect rows (the queue's batches of callers' own
// buffers, xrs_plan.h kRowInd): runtime source count, plain block size.
template <int P, bool ACC, bool VEC, int C = kDyn>
__global__ __launch_bounds__(kBlock) void pair_ind_kernel(const PairArgs<P, C, VEC> a) {
  constexpr int BS = kBlock;
  constexpr bool PLAIN = false;
#define XRS_IND 1
#include "kbody_pair.h"
#undef XRS_IND
}

// ============================================================ rows kernel
// ReconstOne / Reconst steps / retrieveRS:  for o in [0, len):
//   dst_r[o] (^)= sum_m coef[m][r] * msrc_m[o]  ^  XOR_{x: xmask[x]>>r & 1} xsrc_x[o]
template <int R, int NM, int NX, bool VEC>
struct RowsArgs {
  static constexpr int MM = NM == kDyn ? kMaxSrc : (NM > 0 ? NM : 1);
  static constexpr int XM = NX == kDyn ? kMaxXor : (NX > 0 ? NX : 1);
  GfTab tab[MM][R];
  RowRef msrc[MM];
  RowRef xsrc[XM];
  uint32_t xmask[XM];
  RowRef dst[R];
  int nm, nx;
  int grouped;  // runtime counts: issue loads in groups (small grids)
  BlockOrder order;
  uint64_t len;
  uint64_t chunks;
  uint64_t total;
  uint64_t off0;
  uint64_t last;  // ragged end: the last chunk starts here (overlap), else ~0
};

template <int R, int W>
__device__ __forceinline__ void rows_mac1(uint32_t (&acc)[R][W], const GfTab* tab,
                                          const uint32_t* x) {
#pragma unroll
  for (int w = 0; w < W; ++w) {
    const Sel s = sel_of(x[w]);
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r][w] ^= gmul(tab[r], s);
  }
}

template <int R, int W>
__device__ __forceinline__ void rows_mac2(uint32_t (&acc)[R][W], const GfTab* tab0,
                                          const GfTab* tab1, const uint32_t* x0,
                                          const uint32_t* x1) {
  Sel s0[W], s1[W];
#pragma unroll
  for (int w = 0; w < W; ++w) {
    s0[w] = sel_of(x0[w]);
    s1[w] = sel_of(x1[w]);
  }
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int w = 0; w < W; ++w) acc[r][w] = x3(acc[r][w], gmul(tab0[r], s0[w]), gmul(tab1[r], s1[w]));
}

template <int R, int W>
__device__ __forceinline__ void rows_xor(uint32_t (&acc)[R][W], uint32_t mask, const uint32_t* x) {
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint32_t m = 0u - ((mask >> r) & 1u);
#pragma unroll
    for (int w = 0; w < W; ++w) acc[r][w] = xor_masked(acc[r][w], x[w], m);
  }
}

template <int R, int NM, int NX, bool ACC, bool VEC, int BS = kBlock>
__global__ __launch_bounds__(BS) void rows_kernel(const RowsArgs<R, NM, NX, VEC> a) {
#define XRS_IND 0
#define XRS_ROW row_addr
#include "kbody_rows.h"
#undef XRS_ROW
#undef XRS_IND
}

// The rows kernel on indirect rows (xrs_plan.h kRowInd): runtime counts.
template <int R, bool ACC, bool VEC, int NM = kDyn, int NX = kDyn>
__global__ __launch_bounds__(kBlock) void rows_ind_kernel(const RowsArgs<R, NM, NX, VEC> a) {
  constexpr int BS = kBlock;
#define XRS_IND 1
#include "kbody_rows.h"
#undef XRS_IND
}

// ============================================================ staged kernel
// General Reconst in one pass (xrs_plan.h StagedPlan): lost a-halves are
// rebuilt once and feed the retrieveRS and re-piggyback XORs from registers;
// survivors' b-halves are returned to RS form in registers, written back (the
// reference's side effect) and feed the b-half rebuild.  Every row is read
// once and every written row is written once.
template <int NL, int NN, bool VEC>
struct StagedArgs {
  GfTab at[kStSrc][NL > 0 ? NL : 1];
  GfTab bt[kStSrc][NN > 0 ? NN : 1];
  RowRef asrc[kStSrc], bsrc[kStB];
  RowRef adst[kStOut], bdst[kStOut];
  uint32_t bret[kStB];
  uint32_t nmask[kStOut];
  uint32_t rmask[kStOut];  // the nonzero bret[] entries, compacted (late variant)
  int rb[kStOut];          // ... and their b-row indexes
  uint32_t bstore;
  int nd, na, nb, nl, nn, nr;
  BlockOrder order;
  uint64_t half, chunks, total, off0;
};

// acc ^= abar(mask): wave-uniform branches, the masks have few bits set.
template <int NL, int W>
__device__ __forceinline__ void abar_xor(uint32_t* acc, uint32_t mask, const uint32_t (&xa)[kStSrc][W],
                                         const uint32_t (&al)[NL > 0 ? NL : 1][W]) {
#pragma unroll
  for (int j = 0; j < kStSrc; ++j)
    if ((mask >> j) & 1u)
#pragma unroll
      for (int w = 0; w < W; ++w) acc[w] ^= xa[j][w];
#pragma unroll
  for (int q = 0; q < NL; ++q)
    if ((mask >> (kStSrc + q)) & 1u)
#pragma unroll
      for (int w = 0; w < W; ++w) acc[w] ^= al[q][w];
}

template <int NL, int NN, bool VEC>
__global__ __launch_bounds__(kBlock) void staged_kernel(const StagedArgs<NL, NN, VEC> a) {
  constexpr int W = VEC ? 4 : 1;
  constexpr int L1 = NL > 0 ? NL : 1, N1 = NN > 0 ? NN : 1;
  const uint64_t gid = logical_block(a.order) * kBlock + threadIdx.x;
  if (gid >= a.total) return;
  const uint64_t stripe = gid / a.chunks;
  const uint64_t off = a.off0 + (gid - stripe * a.chunks) * (4 * W);
  const int nb = VEC ? 16 : static_cast<int>(a.half - off < 4 ? a.half - off : 4);

  uint32_t xa[kStSrc][W], xb[kStSrc][W];
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int m = 0; m < kStSrc; ++m)
    if (m < a.na) ld<VEC>(xa[m], row_addr(a.asrc[m], stripe, off), nb);
#pragma unroll
  for (int m = 0; m < kStSrc; ++m)
    if (m < a.nb) ld<VEC>(xb[m], row_addr(a.bsrc[m], stripe, off), nb);
  __builtin_amdgcn_s_setprio(0);

  // Stage 1: lost a-halves (xrs.go:247-262).
  uint32_t al[L1][W];
#pragma unroll
  for (int q = 0; q < L1; ++q)
#pragma unroll
    for (int w = 0; w < W; ++w) al[q][w] = 0u;
  if constexpr (NL > 0) {
#pragma unroll
    for (int m = 0; m < kStSrc; m += 2) {
      if (m + 1 < a.nd) rows_mac2<NL, W>(al, a.at[m], a.at[m + 1], xa[m], xa[m + 1]);
      else if (m < a.nd) rows_mac1<NL, W>(al, a.at[m], xa[m]);
    }
#pragma unroll
    for (int q = 0; q < NL; ++q)
      if (q < a.nl) st<VEC>(al[q], row_addr(a.adst[q], stripe, off), nb);
  }

  // Stage 2: retrieveRS on surviving piggybacked parity (xrs.go:305-320).
#pragma unroll
  for (int m = 0; m < kStSrc; ++m)
    if (m < a.nb && a.bret[m]) {
      abar_xor<NL, W>(xb[m], a.bret[m], xa, al);
      if ((a.bstore >> m) & 1u) st<VEC>(xb[m], row_addr(a.bsrc[m], stripe, off), nb);
    }

  // Stages 3+4: needed b-halves, re-piggybacked (xrs.go:270-298).
  if constexpr (NN > 0) {
    uint32_t ob[N1][W];
#pragma unroll
    for (int u = 0; u < NN; ++u) {
#pragma unroll
      for (int w = 0; w < W; ++w) ob[u][w] = 0u;
      if (a.nmask[u]) abar_xor<NL, W>(ob[u], a.nmask[u], xa, al);
    }
#pragma unroll
    for (int m = 0; m < kStSrc; m += 2) {
      if (m + 1 < a.nd) rows_mac2<NN, W>(ob, a.bt[m], a.bt[m + 1], xb[m], xb[m + 1]);
      else if (m < a.nd) rows_mac1<NN, W>(ob, a.bt[m], xb[m]);
    }
#pragma unroll
    for (int u = 0; u < NN; ++u)
      if (u < a.nn) st<VEC>(ob[u], row_addr(a.bdst[u], stripe, off), nb);
  }
}

// Late-b variant: the abar XORs are folded into a few accumulators right
// after stage 1, so the a-rows are dead before the b-rows are loaded (about
// 110 VGPRs instead of 185: twice the waves per SIMD, half the loads in
// flight per wave).
template <int NL, int NN, bool VEC>
__global__ __launch_bounds__(kBlock) void staged_late_kernel(const StagedArgs<NL, NN, VEC> a) {
  const int nd = a.nd;
  constexpr int W = VEC ? 4 : 1;
  constexpr int L1 = NL > 0 ? NL : 1, N1 = NN > 0 ? NN : 1;
  const uint64_t gid = logical_block(a.order) * kBlock + threadIdx.x;
  if (gid >= a.total) return;
  const uint64_t stripe = gid / a.chunks;
  const uint64_t off = a.off0 + (gid - stripe * a.chunks) * (4 * W);
  const int nb = VEC ? 16 : static_cast<int>(a.half - off < 4 ? a.half - off : 4);

  uint32_t xa[kStSrc][W], al[L1][W], rx[kStOut][W], ob[N1][W];
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int m = 0; m < kStSrc; ++m)
    if (m < a.na) ld<VEC>(xa[m], row_addr(a.asrc[m], stripe, off), nb);
  __builtin_amdgcn_s_setprio(0);
#pragma unroll
  for (int q = 0; q < L1; ++q)
#pragma unroll
    for (int w = 0; w < W; ++w) al[q][w] = 0u;
  if constexpr (NL > 0) {
#pragma unroll
    for (int m = 0; m < kStSrc; m += 2) {
      if (m + 1 < nd) rows_mac2<NL, W>(al, a.at[m], a.at[m + 1], xa[m], xa[m + 1]);
      else if (m < nd) rows_mac1<NL, W>(al, a.at[m], xa[m]);
    }
#pragma unroll
    for (int q = 0; q < NL; ++q)
      if (q < a.nl) st<VEC>(al[q], row_addr(a.adst[q], stripe, off), nb);
  }
#pragma unroll
  for (int r = 0; r < kStOut; ++r) {
#pragma unroll
    for (int w = 0; w < W; ++w) rx[r][w] = 0u;
    if (r < a.nr) abar_xor<NL, W>(rx[r], a.rmask[r], xa, al);
  }
#pragma unroll
  for (int u = 0; u < N1; ++u) {
#pragma unroll
    for (int w = 0; w < W; ++w) ob[u][w] = 0u;
    if (u < NN && a.nmask[u]) abar_xor<NL, W>(ob[u], a.nmask[u], xa, al);
  }

  uint32_t xb[kStSrc][W];
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int m = 0; m < kStSrc; ++m)
    if (m < a.nb) ld<VEC>(xb[m], row_addr(a.bsrc[m], stripe, off), nb);
  __builtin_amdgcn_s_setprio(0);
#pragma unroll
  for (int m = 0; m < kStSrc; ++m)
#pragma unroll
    for (int r = 0; r < kStOut; ++r)
      if (r < a.nr && a.rb[r] == m) {
#pragma unroll
        for (int w = 0; w < W; ++w) xb[m][w] ^= rx[r][w];
        st<VEC>(xb[m], row_addr(a.bsrc[m], stripe, off), nb);
      }
  if constexpr (NN > 0) {
#pragma unroll
    for (int m = 0; m < kStSrc; m += 2) {
      if (m + 1 < nd) rows_mac2<NN, W>(ob, a.bt[m], a.bt[m + 1], xb[m], xb[m + 1]);
      else if (m < nd) rows_mac1<NN, W>(ob, a.bt[m], xb[m]);
    }
#pragma unroll
    for (int u = 0; u < NN; ++u)
      if (u < a.nn) st<VEC>(ob[u], row_addr(a.bdst[u], stripe, off), nb);
  }
}

// Compile-time variant of the late-b kernel for the clean loss patterns of a
// d = ND codec whose a-rows are exactly the ND survivors (lost data vects at
// 12+4: na = 12, nb = 12 + surviving piggybacked parity past dpHas[:d]).
// Every load is unconditional and every store comes after the loads of its
// phase, so the waitcnt pass never has to assume a conditional memory op
// is outstanding (the runtime-count kernels wait for vmcnt(0) at every
// guarded load).  Phase A: ND a-row loads, lost a-halves, the retrieveRS and
// re-piggyback XOR terms, the lost a-half stores.  Phase B: NB b-row loads,
// retrieveRS XORs, the needed b-halves, then every b store.
template <int ND, int NL, int W>
__device__ __forceinline__ void abar_ct(uint32_t* acc, uint32_t mask, const uint32_t (&xa)[ND][W],
                                        const uint32_t (&al)[NL][W]) {
#pragma unroll
  for (int j = 0; j < ND; ++j)
    if ((mask >> j) & 1u)
#pragma unroll
      for (int w = 0; w < W; ++w) acc[w] ^= xa[j][w];
#pragma unroll
  for (int q = 0; q < NL; ++q)
    if ((mask >> (kStSrc + q)) & 1u)
#pragma unroll
      for (int w = 0; w < W; ++w) acc[w] ^= al[q][w];
}

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) u32x2 gu32x2;

// W dwords per lane (4: dwordx4, 2: dwordx2), nontemporal, any alignment.
template <int W>
__device__ __forceinline__ void ldw(uint32_t* v, uint64_t addr) {
  if constexpr (W == 4) {
    ld<true>(v, addr, 16);
  } else {
    const u32x2 t = __builtin_nontemporal_load(reinterpret_cast<const gu32x2*>(addr));
    v[0] = t.x;
    v[1] = t.y;
  }
}
template <int W>
__device__ __forceinline__ void stw(const uint32_t* v, uint64_t addr) {
  if constexpr (W == 4) {
    st<true>(v, addr, 16);
  } else {
    u32x2 t;
    t.x = v[0];
    t.y = v[1];
    __builtin_nontemporal_store(t, reinterpret_cast<gu32x2*>(addr));
  }
}

// NPRE: b-rows whose loads are issued with the a-rows (0: after stage 1,
// "late"; NB: every row's load in flight at once, "early").
template <int ND, int NB, int NL, int NN, int BS, int NPRE = 0>
__global__ __launch_bounds__(BS) void staged_ct_kernel(const StagedArgs<NL, NN, true> a) {
  static_assert(NPRE >= 0 && NPRE <= NB, "NPRE");
  constexpr int W = 4;
  const uint64_t gid = logical_block(a.order) * BS + threadIdx.x;
  if (gid >= a.total) return;
  const uint64_t stripe = gid / a.chunks;
  const uint64_t off = a.off0 + (gid - stripe * a.chunks) * (4 * W);

  uint32_t xa[ND][W], al[NL][W], rx[kStOut][W], ob[NN][W], xb[NB][W];
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int m = 0; m < ND; ++m) ldw<W>(xa[m], row_addr(a.asrc[m], stripe, off));
#pragma unroll
  for (int m = 0; m < NPRE; ++m) ldw<W>(xb[m], row_addr(a.bsrc[m], stripe, off));
  __builtin_amdgcn_s_setprio(0);
  // Stage 1: lost a-halves (xrs.go:247-262).
#pragma unroll
  for (int q = 0; q < NL; ++q)
#pragma unroll
    for (int w = 0; w < W; ++w) al[q][w] = 0u;
#pragma unroll
  for (int m = 0; m + 1 < ND; m += 2) rows_mac2<NL, W>(al, a.at[m], a.at[m + 1], xa[m], xa[m + 1]);
  if constexpr (ND & 1) rows_mac1<NL, W>(al, a.at[ND - 1], xa[ND - 1]);
  // XOR terms of stage 2 (retrieveRS, xrs.go:305-320) and stage 4
  // (re-piggyback, :281-297), from the a-rows and the rebuilt a-halves.
#pragma unroll
  for (int r = 0; r < kStOut; ++r) {
#pragma unroll
    for (int w = 0; w < W; ++w) rx[r][w] = 0u;
    if (r < a.nr) abar_ct<ND, NL, W>(rx[r], a.rmask[r], xa, al);
  }
#pragma unroll
  for (int u = 0; u < NN; ++u) {
#pragma unroll
    for (int w = 0; w < W; ++w) ob[u][w] = 0u;
    if (a.nmask[u]) abar_ct<ND, NL, W>(ob[u], a.nmask[u], xa, al);
  }
#pragma unroll
  for (int q = 0; q < NL; ++q) stw<W>(al[q], row_addr(a.adst[q], stripe, off));

  if constexpr (NPRE < NB) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int m = NPRE; m < NB; ++m) ldw<W>(xb[m], row_addr(a.bsrc[m], stripe, off));
    __builtin_amdgcn_s_setprio(0);
  }
#pragma unroll
  for (int m = 0; m < NB; ++m)
#pragma unroll
    for (int r = 0; r < kStOut; ++r)
      if (r < a.nr && a.rb[r] == m)
#pragma unroll
        for (int w = 0; w < W; ++w) xb[m][w] ^= rx[r][w];
  // Stage 3: needed b-halves from the RS-form b-rows (xrs.go:270-275).
#pragma unroll
  for (int m = 0; m + 1 < ND; m += 2) rows_mac2<NN, W>(ob, a.bt[m], a.bt[m + 1], xb[m], xb[m + 1]);
  if constexpr (ND & 1) rows_mac1<NN, W>(ob, a.bt[ND - 1], xb[ND - 1]);
#pragma unroll
  for (int m = 0; m < NB; ++m)
    if ((a.bstore >> m) & 1u) stw<W>(xb[m], row_addr(a.bsrc[m], stripe, off));
#pragma unroll
  for (int u = 0; u < NN; ++u) stw<W>(ob[u], row_addr(a.bdst[u], stripe, off));
}

// Wave-specialised variant of staged_ct_kernel: a block of 2*T lanes works on
// T chunks.  Lanes [0, T) ("a-lanes") load the ND a-rows, rebuild the lost
// a-halves and form the retrieveRS / re-piggyback XOR terms; lanes [T, 2T)
// ("b-lanes") issue their NB b-row loads at the same time.  The XOR terms go
// through LDS (one barrier), then the b-lanes finish stages 2-4.  Every wave
// pays one memory round trip, as Encode does, and holds only its own rows
// (the one-wave-does-both kernels pay two round trips, or hold every row at
// once at 144-161 VGPRs).
template <int ND, int NB, int NL, int NN, int T, int OCC = 1>
__global__ __launch_bounds__(2 * T) __attribute__((amdgpu_waves_per_eu(OCC)))
void staged_ws_kernel(const StagedArgs<NL, NN, true> a) {
  constexpr int W = 4;
  __shared__ uint4 xfer[kStOut + NN][T];  // rx[0..nr), then ob[0..NN)
  const bool blane = threadIdx.x >= T;
  const uint32_t t = blane ? threadIdx.x - T : threadIdx.x;
  const uint64_t gid = logical_block(a.order) * T + t;
  const bool valid = gid < a.total;
  const uint64_t stripe = gid / a.chunks;
  const uint64_t off = a.off0 + (gid - stripe * a.chunks) * (4 * W);
  uint32_t xb[NB][W];
  if (!blane) {
    if (valid) {
      uint32_t xa[ND][W], al[NL][W];
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int m = 0; m < ND; ++m) ldw<W>(xa[m], row_addr(a.asrc[m], stripe, off));
      __builtin_amdgcn_s_setprio(0);
      // Stage 1: lost a-halves (xrs.go:247-262).
#pragma unroll
      for (int q = 0; q < NL; ++q)
#pragma unroll
        for (int w = 0; w < W; ++w) al[q][w] = 0u;
#pragma unroll
      for (int m = 0; m + 1 < ND; m += 2) rows_mac2<NL, W>(al, a.at[m], a.at[m + 1], xa[m], xa[m + 1]);
      if constexpr (ND & 1) rows_mac1<NL, W>(al, a.at[ND - 1], xa[ND - 1]);
      // XOR terms of stage 2 (retrieveRS, xrs.go:305-320) and stage 4
      // (re-piggyback, :281-297) for the b-lanes.
#pragma unroll
      for (int r = 0; r < kStOut; ++r)
        if (r < a.nr) {
          uint32_t v[W] = {0u, 0u, 0u, 0u};
          abar_ct<ND, NL, W>(v, a.rmask[r], xa, al);
          xfer[r][t] = make_uint4(v[0], v[1], v[2], v[3]);
        }
#pragma unroll
      for (int u = 0; u < NN; ++u) {
        uint32_t v[W] = {0u, 0u, 0u, 0u};
        if (a.nmask[u]) abar_ct<ND, NL, W>(v, a.nmask[u], xa, al);
        xfer[kStOut + u][t] = make_uint4(v[0], v[1], v[2], v[3]);
      }
#pragma unroll
      for (int q = 0; q < NL; ++q) stw<W>(al[q], row_addr(a.adst[q], stripe, off));
    }
  } else if (valid) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int m = 0; m < NB; ++m) ldw<W>(xb[m], row_addr(a.bsrc[m], stripe, off));
    __builtin_amdgcn_s_setprio(0);
  }
  // LDS only: the b-lanes' row loads stay in flight across the barrier.
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  if (!blane || !valid) return;
#pragma unroll
  for (int m = 0; m < NB; ++m)
#pragma unroll
    for (int r = 0; r < kStOut; ++r)
      if (r < a.nr && a.rb[r] == m) {
        const uint4 v = xfer[r][t];
        xb[m][0] ^= v.x;
        xb[m][1] ^= v.y;
        xb[m][2] ^= v.z;
        xb[m][3] ^= v.w;
      }
  uint32_t ob[NN][W];
#pragma unroll
  for (int u = 0; u < NN; ++u) {
    const uint4 v = xfer[kStOut + u][t];
    ob[u][0] = v.x;
    ob[u][1] = v.y;
    ob[u][2] = v.z;
    ob[u][3] = v.w;
  }
  // Stage 3: needed b-halves from the RS-form b-rows (xrs.go:270-275).
#pragma unroll
  for (int m = 0; m + 1 < ND; m += 2) rows_mac2<NN, W>(ob, a.bt[m], a.bt[m + 1], xb[m], xb[m + 1]);
  if constexpr (ND & 1) rows_mac1<NN, W>(ob, a.bt[ND - 1], xb[ND - 1]);
#pragma unroll
  for (int m = 0; m < NB; ++m)
    if ((a.bstore >> m) & 1u) stw<W>(xb[m], row_addr(a.bsrc[m], stripe, off));
#pragma unroll
  for (int u = 0; u < NN; ++u) stw<W>(ob[u], row_addr(a.bdst[u], stripe, off));
}

// Wave-specialised 12+4-style Encode (compile-time source count C, P = 4,
// 16-byte chunks, halves a multiple of 16 bytes): a block of 2*T lanes works
// on T chunks.  Lanes [0, T) load the C data a-halves, form the four parity
// a-halves and store them, and leave the piggyback terms (data c rides on
// parity 1 + c % 3, xrs.go:77-100) in LDS; lanes [T, 2T) load the C data
// b-halves and form the four RS b-halves at the same time; one barrier; the
// b-lanes add the piggyback terms and store.  Each lane holds one half's rows
// (the pair kernel holds both, 170 VGPRs, two waves per SIMD).
template <int C, int T>
__global__ __launch_bounds__(2 * T) void enc_ws_kernel(const PairArgs<4, C, true> a) {
  constexpr int P = 4, W = 4;
  __shared__ uint4 xfer[P - 1][T];
  const bool blane = threadIdx.x >= T;
  const uint32_t t = blane ? threadIdx.x - T : threadIdx.x;
  const uint64_t gid = logical_block(a.order) * T + t;
  const bool valid = gid < a.total;
  const uint64_t stripe = gid / a.chunks;
  const uint64_t off = a.off0 + (gid - stripe * a.chunks) * (4 * W) + (blane ? a.half : 0);
  uint32_t acc[P][W];
  if (valid) {
    uint32_t x[C][W];
#pragma unroll
    for (int c = 0; c < C; ++c) ldw<W>(x[c], row_addr(a.src[c], stripe, off));
#pragma unroll
    for (int r = 0; r < P; ++r)
#pragma unroll
      for (int w = 0; w < W; ++w) acc[r][w] = 0u;
#pragma unroll
    for (int c = 0; c + 1 < C; c += 2) rows_mac2<P, W>(acc, a.tab[c], a.tab[c + 1], x[c], x[c + 1]);
    if constexpr (C & 1) rows_mac1<P, W>(acc, a.tab[C - 1], x[C - 1]);
    if (!blane) {
      uint32_t pg[P - 1][W];
#pragma unroll
      for (int r = 0; r < P - 1; ++r)
#pragma unroll
        for (int w = 0; w < W; ++w) pg[r][w] = 0u;
#pragma unroll
      for (int c = 0; c < C; ++c)
#pragma unroll
        for (int w = 0; w < W; ++w) pg[c % (P - 1)][w] ^= x[c][w];
#pragma unroll
      for (int r = 0; r < P - 1; ++r) xfer[r][t] = make_uint4(pg[r][0], pg[r][1], pg[r][2], pg[r][3]);
#pragma unroll
      for (int r = 0; r < P; ++r) stw<W>(acc[r], row_addr(a.dst[r], stripe, off));
    }
  }
  // LDS only: no wait on the a-lanes' stores at the barrier.
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  if (!blane || !valid) return;
#pragma unroll
  for (int r = 1; r < P; ++r) {
    const uint4 v = xfer[r - 1][t];
    acc[r][0] ^= v.x;
    acc[r][1] ^= v.y;
    acc[r][2] ^= v.z;
    acc[r][3] ^= v.w;
  }
#pragma unroll
  for (int r = 0; r < P; ++r) stw<W>(acc[r], row_addr(a.dst[r], stripe, off));
}

// Persistent form of staged_ws_kernel for 2 lost data vects from 256 to 768
// KiB halves: one block of 2*T lanes per CU takes T-chunk tiles from a launch-wide
// counter, as the hardware dispatcher hands out blocks (so the tiles in
// flight stay a compact stretch of the batch), and the two roles run one tile
// apart.  Per tile j: the a-lanes load tile j's a-rows, rebuild and store the
// lost a-halves and leave the XOR terms in LDS slot j & 1, while lane 0 takes
// tile j+1 from the counter into nexttile[(j+1) & 1]; one barrier; the
// b-lanes, whose b-rows of tile j were issued before it, finish stages 2-4 of
// tile j and issue tile j+1's b-rows, while the a-lanes are already loading
// tile j+1.  Each role's GF work and stores overlap the other role's loads
// and no block turnover sits between tiles.  Slot s is rewritten two tiles
// later, after a barrier that the b-lanes reach only once they have read it.
// Tile v is logical block v of the XCD order (K = the tiles of one
// half-vect, so each XCD works through one stripe per group).
//
// Kernel-argument reads in the loops go through a pointer the compiler
// cannot see through (kargs): each tile re-reads its tables and row refs
// with scalar loads instead of hoisting all of them into SGPRs, which
// spills.  (Taking the address of the by-value argument copies it to
// scratch instead.)
#define XRS_KC __attribute__((address_space(4)))
template <class A>
__device__ __forceinline__ const XRS_KC A* kargs() {
  const XRS_KC A* p = (const XRS_KC A*)(__builtin_amdgcn_kernarg_segment_ptr());
  asm volatile("" : "+s"(p));
  return p;
}
__device__ __forceinline__ GfTab kld(const XRS_KC GfTab& r) {
  return GfTab{r.lo0, r.hi0, r.lo1, r.hi1, r.top};
}
__device__ __forceinline__ RowRef kld(const XRS_KC RowRef& r) { return RowRef{r.ptr, r.stripe_stride}; }
__device__ __forceinline__ BlockOrder kld(const XRS_KC BlockOrder& r) { return BlockOrder{r.nblk, r.k}; }
template <int R>
__device__ __forceinline__ void ktabs(GfTab (&t)[R], const XRS_KC GfTab* src) {
#pragma unroll
  for (int r = 0; r < R; ++r) t[r] = kld(src[r]);
}

// ctr: the launch's counter slot (ctr[0] hands out tiles, ctr[1] counts the
// blocks done) and busy, the slot's host word (tile_counters below): the last
// block out resets both counters and then clears busy, so the slot is free
// for the next launch on any stream without a host-side reset.
template <int ND, int NB, int NL, int NN, int T>
__global__ __launch_bounds__(2 * T) void staged_wsp_kernel(const StagedArgs<NL, NN, true> a,
                                                            const uint32_t ntiles, uint32_t* ctr,
                                                            uint32_t* busy) {
  using Args = StagedArgs<NL, NN, true>;
  constexpr int W = 4;
  __shared__ uint4 xfer[2][kStOut + NN][T];
  __shared__ uint32_t nexttile[2];
  // Wave-uniform role (T is a multiple of 64): two separate loops, so neither
  // role's rows are live while the other role's code runs.
  const bool blane = __builtin_amdgcn_readfirstlane(threadIdx.x) >= T;
  const uint32_t t = blane ? threadIdx.x - T : threadIdx.x;
  uint32_t v = blockIdx.x;  // each block's first tile; the rest from *ctr
  if (!blane) {
    for (uint32_t j = 0; v < ntiles; ++j) {
      const XRS_KC Args* q = kargs<Args>();
      const uint32_t s = j & 1u;
      uint32_t nv = 0;
      if (threadIdx.x == 0) nv = atomicAdd(ctr, 1u) + gridDim.x;
      const uint64_t gid = logical_of(kld(q->order), v) * T + t;
      if (gid < q->total) {
        const uint64_t chunks = q->chunks;
        const uint64_t stripe = gid / chunks;
        const uint64_t off = q->off0 + (gid - stripe * chunks) * (4 * W);
        uint32_t xa[ND][W], al[NL][W];
#pragma unroll
        for (int m = 0; m < ND; ++m) ldw<W>(xa[m], row_addr(kld(q->asrc[m]), stripe, off));
        // Stage 1: lost a-halves (xrs.go:247-262).
#pragma unroll
        for (int l = 0; l < NL; ++l)
#pragma unroll
          for (int w = 0; w < W; ++w) al[l][w] = 0u;
#pragma unroll
        for (int m = 0; m + 1 < ND; m += 2) {
          GfTab t0[NL], t1[NL];
          ktabs<NL>(t0, q->at[m]);
          ktabs<NL>(t1, q->at[m + 1]);
          rows_mac2<NL, W>(al, t0, t1, xa[m], xa[m + 1]);
        }
        if constexpr (ND & 1) {
          GfTab t0[NL];
          ktabs<NL>(t0, q->at[ND - 1]);
          rows_mac1<NL, W>(al, t0, xa[ND - 1]);
        }
        // XOR terms of stage 2 (retrieveRS, xrs.go:305-320) and stage 4
        // (re-piggyback, :281-297) for the b-lanes.
        const int nr = q->nr;
#pragma unroll
        for (int r = 0; r < kStOut; ++r)
          if (r < nr) {
            uint32_t x[W] = {0u, 0u, 0u, 0u};
            abar_ct<ND, NL, W>(x, q->rmask[r], xa, al);
            xfer[s][r][t] = make_uint4(x[0], x[1], x[2], x[3]);
          }
#pragma unroll
        for (int u = 0; u < NN; ++u) {
          uint32_t x[W] = {0u, 0u, 0u, 0u};
          const uint32_t nm = q->nmask[u];
          if (nm) abar_ct<ND, NL, W>(x, nm, xa, al);
          xfer[s][kStOut + u][t] = make_uint4(x[0], x[1], x[2], x[3]);
        }
#pragma unroll
        for (int l = 0; l < NL; ++l) stw<W>(al[l], row_addr(kld(q->adst[l]), stripe, off));
      }
      if (threadIdx.x == 0) nexttile[s ^ 1u] = nv;
      // LDS only: no wait on this wave's stores at the barrier.
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
      v = __builtin_amdgcn_readfirstlane(nexttile[s ^ 1u]);
    }
    // This block takes no more tiles.  The last block to get here resets the
    // slot.  No fence is needed (a release at agent scope writes back the
    // XCD's L2 on gfx950, +5-11 us per launch measured): lane 0's last tile
    // atomic has returned (the loop exit reads its value) before its arrival
    // is issued, so every tile atomic of the launch is performed before the
    // last arrival; the resets are exchanges whose returned values the busy
    // store's value depends on, so they are performed before the host sees
    // the slot free.  The dependency is one the compiler cannot fold: ctr[1]
    // returns gridDim.x (< 2^31), so (r0 & r1) == ~0u is false and the store
    // writes 0, but only the returned values say so; the explicit vmcnt(0)
    // wait (gfx9 encoding: vmcnt 0, expcnt 7, lgkmcnt 15) states the order
    // in the code object as well.  tests/test_kernel_resources.py
    // (test_persistent_slot_reset_order) checks the disassembly: both
    // returning swaps, then s_waitcnt vmcnt(0), then the busy store.
    if (threadIdx.x == 0 && atomicAdd(ctr + 1, 1u) == gridDim.x - 1) {
      const uint32_t r0 = __hip_atomic_exchange(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t r1 =
          __hip_atomic_exchange(ctr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_s_waitcnt(0x0F70);
      __hip_atomic_store(busy, (r0 & r1) == ~0u ? 1u : 0u, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    }
    return;
  }
  uint32_t xb[NB][W];
  if (v < ntiles) {
    const uint64_t gid = logical_of(a.order, v) * T + t;
    if (gid < a.total) {
      const uint64_t stripe = gid / a.chunks;
      const uint64_t off = a.off0 + (gid - stripe * a.chunks) * (4 * W);
#pragma unroll
      for (int m = 0; m < NB; ++m) ldw<W>(xb[m], row_addr(a.bsrc[m], stripe, off));
    }
  }
  for (uint32_t j = 0; v < ntiles; ++j) {
    const XRS_KC Args* q = kargs<Args>();
    const uint32_t s = j & 1u;
    const BlockOrder order = kld(q->order);
    const uint64_t total = q->total, chunks = q->chunks, off0 = q->off0;
    const uint64_t gid = logical_of(order, v) * T + t;
    // LDS only: this tile's b-row loads stay in flight across the barrier.
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    if (gid < total) {
      const uint64_t stripe = gid / chunks;
      const uint64_t off = off0 + (gid - stripe * chunks) * (4 * W);
      const int nr = q->nr;
#pragma unroll
      for (int r = 0; r < kStOut; ++r)
        if (r < nr) {
          const int rb = q->rb[r];
          const uint4 x = xfer[s][r][t];
#pragma unroll
          for (int m = 0; m < NB; ++m)
            if (rb == m) {
              xb[m][0] ^= x.x;
              xb[m][1] ^= x.y;
              xb[m][2] ^= x.z;
              xb[m][3] ^= x.w;
            }
        }
      uint32_t ob[NN][W];
#pragma unroll
      for (int u = 0; u < NN; ++u) {
        const uint4 x = xfer[s][kStOut + u][t];
        ob[u][0] = x.x;
        ob[u][1] = x.y;
        ob[u][2] = x.z;
        ob[u][3] = x.w;
      }
      // Stage 3: needed b-halves from the RS-form b-rows (xrs.go:270-275).
#pragma unroll
      for (int m = 0; m + 1 < ND; m += 2) {
        GfTab t0[NN], t1[NN];
        ktabs<NN>(t0, q->bt[m]);
        ktabs<NN>(t1, q->bt[m + 1]);
        rows_mac2<NN, W>(ob, t0, t1, xb[m], xb[m + 1]);
      }
      if constexpr (ND & 1) {
        GfTab t0[NN];
        ktabs<NN>(t0, q->bt[ND - 1]);
        rows_mac1<NN, W>(ob, t0, xb[ND - 1]);
      }
      const uint32_t bstore = q->bstore;
#pragma unroll
      for (int m = 0; m < NB; ++m)
        if ((bstore >> m) & 1u) stw<W>(xb[m], row_addr(kld(q->bsrc[m]), stripe, off));
#pragma unroll
      for (int u = 0; u < NN; ++u) stw<W>(ob[u], row_addr(kld(q->bdst[u]), stripe, off));
    }
    const uint32_t vn = __builtin_amdgcn_readfirstlane(nexttile[s ^ 1u]);
    if (vn < ntiles) {
      const uint64_t gn = logical_of(order, vn) * T + t;
      if (gn < total) {
        const uint64_t sn = gn / chunks;
        const uint64_t on = off0 + (gn - sn * chunks) * (4 * W);
#pragma unroll
        for (int m = 0; m < NB; ++m) ldw<W>(xb[m], row_addr(kld(q->bsrc[m]), sn, on));
      }
    }
    v = vn;
  }
}

// Runtime-count form of staged_ws_kernel (any codec with d <= 16, lost parity
// in the pattern, nl != nn): a-lanes load na a-rows, b-lanes nb b-rows, each
// role's guarded loads issued together (each role waits once, so the
// vmcnt(0) the waitcnt pass puts after guarded loads costs no extra round
// trip).  Same conditions as staged_late_kernel: every retrieveRS row is
// written back and there are at most kStOut of them.
template <int NL, int NN, int T, int NBM = kStSrc>
__global__ __launch_bounds__(2 * T) void staged_ws_rt_kernel(const StagedArgs<NL, NN, true> a) {
  constexpr int W = 4;
  constexpr int L1 = NL > 0 ? NL : 1, N1 = NN > 0 ? NN : 1;
  __shared__ uint4 xfer[kStOut + N1][T];
  const bool blane = threadIdx.x >= T;
  const uint32_t t = blane ? threadIdx.x - T : threadIdx.x;
  const uint64_t gid = logical_block(a.order) * T + t;
  const bool valid = gid < a.total;
  const uint64_t stripe = gid / a.chunks;
  const uint64_t off = a.off0 + (gid - stripe * a.chunks) * (4 * W);
  const int nd = a.nd;
  uint32_t xb[NBM][W];
  if (!blane) {
    if (valid) {
      uint32_t xa[kStSrc][W], al[L1][W];
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int m = 0; m < kStSrc; ++m)
        if (m < a.na) ldw<W>(xa[m], row_addr(a.asrc[m], stripe, off));
      __builtin_amdgcn_s_setprio(0);
#pragma unroll
      for (int q = 0; q < L1; ++q)
#pragma unroll
        for (int w = 0; w < W; ++w) al[q][w] = 0u;
      if constexpr (NL > 0) {
        // Stage 1: lost a-halves (xrs.go:247-262).
#pragma unroll
        for (int m = 0; m < kStSrc; m += 2) {
          if (m + 1 < nd) rows_mac2<NL, W>(al, a.at[m], a.at[m + 1], xa[m], xa[m + 1]);
          else if (m < nd) rows_mac1<NL, W>(al, a.at[m], xa[m]);
        }
      }
      // XOR terms of stages 2 and 4 for the b-lanes.
#pragma unroll
      for (int r = 0; r < kStOut; ++r)
        if (r < a.nr) {
          uint32_t v[W] = {0u, 0u, 0u, 0u};
          abar_xor<NL, W>(v, a.rmask[r], xa, al);
          xfer[r][t] = make_uint4(v[0], v[1], v[2], v[3]);
        }
#pragma unroll
      for (int u = 0; u < NN; ++u) {
        uint32_t v[W] = {0u, 0u, 0u, 0u};
        if (a.nmask[u]) abar_xor<NL, W>(v, a.nmask[u], xa, al);
        xfer[kStOut + u][t] = make_uint4(v[0], v[1], v[2], v[3]);
      }
      if constexpr (NL > 0) {
#pragma unroll
        for (int q = 0; q < NL; ++q)
          if (q < a.nl) stw<W>(al[q], row_addr(a.adst[q], stripe, off));
      }
    }
  } else if (valid) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int m = 0; m < NBM; ++m)
      if (m < a.nb) ldw<W>(xb[m], row_addr(a.bsrc[m], stripe, off));
    __builtin_amdgcn_s_setprio(0);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  if (!blane || !valid) return;
#pragma unroll
  for (int m = 0; m < NBM; ++m)
#pragma unroll
    for (int r = 0; r < kStOut; ++r)
      if (r < a.nr && a.rb[r] == m) {
        const uint4 v = xfer[r][t];
        xb[m][0] ^= v.x;
        xb[m][1] ^= v.y;
        xb[m][2] ^= v.z;
        xb[m][3] ^= v.w;
        stw<W>(xb[m], row_addr(a.bsrc[m], stripe, off));
      }
  if constexpr (NN > 0) {
    uint32_t ob[NN][W];
#pragma unroll
    for (int u = 0; u < NN; ++u) {
      const uint4 v = xfer[kStOut + u][t];
      ob[u][0] = v.x;
      ob[u][1] = v.y;
      ob[u][2] = v.z;
      ob[u][3] = v.w;
    }
    // Stage 3: needed b-halves from the RS-form b-rows (xrs.go:270-275).
#pragma unroll
    for (int m = 0; m < kStSrc; m += 2) {
      if (m + 1 < nd) rows_mac2<NN, W>(ob, a.bt[m], a.bt[m + 1], xb[m], xb[m + 1]);
      else if (m < nd) rows_mac1<NN, W>(ob, a.bt[m], xb[m]);
    }
#pragma unroll
    for (int u = 0; u < NN; ++u)
      if (u < a.nn) stw<W>(ob[u], row_addr(a.bdst[u], stripe, off));
  }
}

// ============================================================ update_rows kernel
// Update with a per-stripe data row (xrs_plan.h UpdRowsPlan).  The row's
// coefficient tables are read from the kernel arguments with a per-lane index
// (lanes of one wave may serve different stripes when H < 1 KiB).
template <int P, bool VEC>
struct UpdRowsArgs {
  GfTab tab[kMaxSrc][P];
  int32_t pbq[kMaxSrc];
  RowRef old_row, new_row;
  RowRef dst[P];
  const int32_t* rows;
  int row0, nrows;
  BlockOrder order;
  uint64_t half, chunks, total, off0;
};

template <int P, bool VEC>
__global__ __launch_bounds__(kBlock) void update_rows_kernel(const UpdRowsArgs<P, VEC> a) {
#define XRS_IND 0
#define XRS_ROW row_addr
#include "kbody_update.h"
#undef XRS_ROW
#undef XRS_IND
}

// update_rows on indirect rows (xrs_plan.h kRowInd).
template <int P, bool VEC>
__global__ __launch_bounds__(kBlock) void update_rows_ind_kernel(const UpdRowsArgs<P, VEC> a) {
#define XRS_IND 1
#include "kbody_update.h"
#undef XRS_IND
}

}  // namespace

// ============================================================ launch trace
// Diagnostic record of which kernel instantiations this process launched
// (xrs_trace_kernels / xrs_traced_kernels): smoke() and the dispatch tests
// name the kernels they exercised.  Off: one relaxed atomic load per launch.
// Shared by every build part (defined in part 1, see the end of the file).
extern std::atomic<bool> g_trace;
extern std::mutex g_trace_mu;
extern std::vector<std::pair<std::string, uint64_t>> g_trace_log;  // (kernel, launches)

namespace {

// Device symbol name -> "pair_kernel<4, 12, false, true, 128, true>" (the
// name rocprofv3 prints, without namespaces, return type and parameters).
std::string clean_kernel_name(const char* sym) {
  if (!sym) return "?";
  std::string n(sym);
  int st = 0;
  if (char* dm = abi::__cxa_demangle(sym, nullptr, nullptr, &st)) {
    n = dm;
    std::free(dm);
  }
  if (n.compare(0, 5, "void ") == 0) n.erase(0, 5);
  for (const char* ns : {"xrs::(anonymous namespace)::", "(anonymous namespace)::", "xrs::"})
    for (size_t i; (i = n.find(ns)) != std::string::npos;) n.erase(i, std::strlen(ns));
  int depth = 0;  // drop the parameter list: the first '(' outside <...>
  for (size_t i = 0; i < n.size(); ++i) {
    if (n[i] == '<') ++depth;
    else if (n[i] == '>') --depth;
    else if (n[i] == '(' && depth == 0) {
      n.resize(i);
      break;
    }
  }
  return n;
}

template <auto K>
const char* kernel_name(hipStream_t s) {
  static const std::string n =
      clean_kernel_name(hipKernelNameRefByPtr(reinterpret_cast<const void*>(K), s));
  return n.c_str();
}

void trace_note(const char* name) {
  std::lock_guard<std::mutex> g(g_trace_mu);
  for (auto& e : g_trace_log)
    if (e.first == name) {
      ++e.second;
      return;
    }
  g_trace_log.emplace_back(name, 1);
}

// hipLaunchKernelGGL with the trace hook; KERNEL is a parenthesised
// template-id, e.g. XRS_LAUNCH((pair_kernel<4, 12, false, true>), grid, block, stream, args).
#define XRS_LAUNCH(KERNEL, GRID, BLOCK, STREAM, ...)                                   \
  do {                                                                                 \
    if (g_trace.load(std::memory_order_relaxed)) trace_note(kernel_name<&KERNEL>(STREAM)); \
    hipLaunchKernelGGL(KERNEL, GRID, BLOCK, 0, STREAM, __VA_ARGS__);                    \
  } while (0)

// ============================================================ launchers
inline bool aligned16(uint64_t v) { return (v & 15u) == 0; }

enum class Shape { kPair, kRows, kStaged };

// K per kernel shape and half-vect length, from interleaved medians of every
// order on MI355X (profiles/r01_mapprobe2.log, r01_mapprobe3.log):
//  * pair (Encode/Update/Replace): K = 32 is best or within 1% at 4 KiB-8 MiB;
//  * rows (ReconstOne): vects up to 8 KiB want one range per XCD (K =
//    nblk/8; 4,128-B vects +12%, 6 KiB +7%: profiles/r01_order_sweep_sizes.log),
//    16-128 KiB vects the plain order, >= 512 KiB vects K = half / 8 KiB up
//    to 256 (1 MiB: 64, 8 MiB: 256; profiles/r01_order_sweep.log);
//  * staged (general Reconst): 4 KiB vects one range per XCD (+6-7% over
//    K = 32), 512 KiB-2 MiB vects K = 128, >= 2 MiB vects the plain order
//    (8 MiB: K = 256 lost 5-9%), K = 32 between
//    (profiles/r01_order_sweep_staged.log).
// The byte-granular (!VEC) path keeps the plain order.  XRS_BLOCK_ORDER=<K>
// overrides (0: plain order; "full": one range per XCD) for A/B runs.
BlockOrder block_order(Shape shape, bool vec, uint64_t len, uint64_t blocks, int bs = kBlock) {
  BlockOrder o{static_cast<uint32_t>(blocks), 0};
  if (!vec) return o;
  if (const char* e = std::getenv("XRS_BLOCK_ORDER")) {
    if (std::strcmp(e, "full") == 0) o.k = static_cast<uint32_t>(blocks / 8);
    else o.k = static_cast<uint32_t>(std::strtoul(e, nullptr, 10));
    return o;
  }
  switch (shape) {
    case Shape::kPair: o.k = 32; break;
    case Shape::kStaged:
      if (len <= 2048) o.k = static_cast<uint32_t>(blocks / 8);
      else if (len < (256u << 10)) o.k = 32;
      else o.k = 128;  // (plain order above 1 MiB halves: 2-11% slower at
      break;           // 2, 8, 16 MiB vects, profiles/r02_staged_bigorder.log)
    case Shape::kRows:
      if (bs == 1024 && len >= (256u << 10)) {  // 16 KiB blocks: K = half / 4 KiB,
        // 64 from 1 MiB halves (12+4 ReconstOne at 4 / 8 / 16 MiB vects +2 /
        // +5 / +4% over 256: profiles/r02_bigorder.log, r02_enc_k0.log)
        o.k = len >= (1u << 20) ? 64 : static_cast<uint32_t>(len >> 12);
        break;
      }
      if (len <= 4096) o.k = static_cast<uint32_t>(blocks / 8);
      else if (len >= (256u << 10)) o.k = static_cast<uint32_t>(std::min<uint64_t>(256, len >> 13));
      break;
  }
  return o;
}

// Threads per block for a kernel family: `def`, or the env override when it
// names a size this build instantiates for that family.
int env_block(const char* var, int def) {
  const char* e = std::getenv(var);
  if (!e || !*e) return def;
  const int v = std::atoi(e);
  return (v == 256 || v == def) ? v : def;
}

// Wave-specialised staged kernel: T chunks per block of 2*T lanes.
template <int NL, int NN, int T, int OCC = 1>
int launch_staged_ws(StagedArgs<NL, NN, true> a, const StagedPlan& p, hipStream_t stream) {
  const uint64_t blocks = (a.total + T - 1) / T;
  if (blocks > kMaxBlocks) return static_cast<int>(hipErrorInvalidConfiguration);
  a.order = block_order(Shape::kStaged, true, p.half, blocks, T);
  if (const char* e = std::getenv("XRS_WS_ORDER")) {  // A/B knob
    a.order.k = std::strcmp(e, "full") == 0 ? static_cast<uint32_t>(blocks / 8)
                                            : static_cast<uint32_t>(std::strtoul(e, nullptr, 10));
  }
  const dim3 g(static_cast<unsigned>(blocks));
  if constexpr (NL == 1) {
    // one lost parity vect (12+4: P12 -> nb = 15, P13..15 -> nb = 14)
    if (p.nb == 15) {
      XRS_LAUNCH((staged_ws_kernel<12, 15, NL, NN, T, OCC>), g, dim3(2 * T), stream, a);
      return static_cast<int>(hipGetLastError());
    }
  }
  if (p.nb == 12)
    XRS_LAUNCH((staged_ws_kernel<12, 12, NL, NN, T, OCC>), g, dim3(2 * T), stream, a);
  else if (p.nb == 13)
    XRS_LAUNCH((staged_ws_kernel<12, 13, NL, NN, T, OCC>), g, dim3(2 * T), stream, a);
  else
    XRS_LAUNCH((staged_ws_kernel<12, 14, NL, NN, T, OCC>), g, dim3(2 * T), stream, a);
  return static_cast<int>(hipGetLastError());
}

// Compute units of the stream's device (cached per device).
int cu_count(hipStream_t s) {
  static std::atomic<int> cache[64];
  int dev = 0;
  if (hipStreamGetDevice(s, &dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  int n = cache[dev].load(std::memory_order_relaxed);
  if (n > 0) return n;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
    n = 256;
  cache[dev].store(n, std::memory_order_relaxed);
  return n;
}

// Persistent wave-specialised staged kernel (staged_wsp_kernel): one block
// of 2*T lanes per compute unit (XRS_WSP_PER_CU: more, A/B; XRS_WSP_GRID: an
// exact block count, so tests give every block many tiles), K = the tiles of
// one half-vect (XRS_WS_ORDER overrides).  The tile counter is a slot of the
// launch stream's device's ring (tile_counters), claimed here and released by
// the kernel itself.  Returns kNotLaunched when no slot is free; the caller
// then runs the one-shot kernel.
constexpr int kNotLaunched = -1;

// Tile counters of the persistent kernels, per device: kCtrSlots slots of two
// counters (one 128-B line each) in device memory, zero when free, and one
// pinned host word per slot, 1 while a launch holds it.  A launch claims a
// slot with a host compare-and-swap; the kernel's last block resets the
// counters and clears the word (a system-scope release store), so a slot is
// never shared by two launches in flight, whatever their streams, and a
// launch costs no allocation, memset or free (round 4's stream-ordered
// counter cost 2-7 us per synchronous call, profiles/r04_wsp_overhead.log).
constexpr int kCtrSlots = 256;
constexpr int kCtrLine = 32;   // uint32 per counter slot (128 B)
constexpr int kBusyLine = 16;  // uint32 per host word (64 B)
struct CtrRing {
  uint32_t* ctr = nullptr;       // device memory, kCtrSlots * kCtrLine words
  uint32_t* busy = nullptr;      // pinned host memory, kCtrSlots * kBusyLine words
  uint32_t* busy_dev = nullptr;  // its device address
  std::atomic<uint32_t> next{0};
};

CtrRing* ctr_ring(int dev) {
  static std::mutex mu;
  static CtrRing* rings[64] = {};
  static bool tried[64] = {};
  if (dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> g(mu);
  if (!tried[dev]) {
    tried[dev] = true;
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev && hipSetDevice(dev) != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
    auto* r = new CtrRing();
    hipStream_t z = nullptr;
    void* dp = nullptr;
    bool ok = hipMalloc(reinterpret_cast<void**>(&r->ctr), kCtrSlots * kCtrLine * sizeof(uint32_t)) == hipSuccess;
    // zeroed on a private stream: no null-stream barrier against the user's work
    ok = ok && hipStreamCreateWithFlags(&z, hipStreamNonBlocking) == hipSuccess;
    ok = ok && hipMemsetAsync(r->ctr, 0, kCtrSlots * kCtrLine * sizeof(uint32_t), z) == hipSuccess &&
         hipStreamSynchronize(z) == hipSuccess;
    if (z) (void)hipStreamDestroy(z);
    ok = ok && hipHostMalloc(reinterpret_cast<void**>(&r->busy), kCtrSlots * kBusyLine * sizeof(uint32_t),
                             hipHostMallocMapped) == hipSuccess;
    ok = ok && hipHostGetDevicePointer(&dp, r->busy, 0) == hipSuccess;
    if (ok) {
      std::memset(r->busy, 0, kCtrSlots * kBusyLine * sizeof(uint32_t));
      r->busy_dev = static_cast<uint32_t*>(dp);
      rings[dev] = r;
    } else {
      (void)hipGetLastError();
      if (r->ctr) (void)hipFree(r->ctr);
      if (r->busy) (void)hipHostFree(r->busy);
      delete r;
    }
    if (prev >= 0 && prev != dev) (void)hipSetDevice(prev);
  }
  return rings[dev];
}

// A free slot of ring r, now held by the caller (its busy word set), or -1.
int claim_slot(CtrRing* r) {
  for (int i = 0; i < kCtrSlots; ++i) {
    const uint32_t s = r->next.fetch_add(1, std::memory_order_relaxed) % kCtrSlots;
    uint32_t expect = 0;
    if (__atomic_compare_exchange_n(r->busy + s * kBusyLine, &expect, 1u, false, __ATOMIC_ACQ_REL,
                                    __ATOMIC_ACQUIRE))
      return static_cast<int>(s);
  }
  return -1;
}

template <int NL, int NN, int T>
int launch_staged_wsp(StagedArgs<NL, NN, true> a, const StagedPlan& p, hipStream_t stream) {
  const uint64_t tiles = (a.total + T - 1) / T;
  if (tiles > kMaxBlocks) return static_cast<int>(hipErrorInvalidConfiguration);
  a.order = block_order(Shape::kStaged, true, p.half, tiles, T);
  a.order.k = static_cast<uint32_t>(std::max<uint64_t>(1, a.chunks / T));
  if (const char* e = std::getenv("XRS_WS_ORDER")) {  // A/B knob
    a.order.k = std::strcmp(e, "full") == 0 ? static_cast<uint32_t>(tiles / 8)
                                            : static_cast<uint32_t>(std::strtoul(e, nullptr, 10));
  }
  uint64_t per_cu = 1;
  if (const char* e = std::getenv("XRS_WSP_PER_CU")) per_cu = std::max<uint64_t>(1, std::strtoul(e, nullptr, 10));
  uint64_t grid = per_cu * static_cast<uint64_t>(cu_count(stream));
  if (const char* e = std::getenv("XRS_WSP_GRID")) grid = std::max<uint64_t>(1, std::strtoul(e, nullptr, 10));
  grid = std::min<uint64_t>(tiles, grid);
  const dim3 g(static_cast<unsigned>(grid));
  const uint32_t nt = static_cast<uint32_t>(tiles);
  int dev = -1;
  if (hipStreamGetDevice(stream, &dev) != hipSuccess) {
    (void)hipGetLastError();
    return kNotLaunched;
  }
  CtrRing* ring = ctr_ring(dev);
  const int slot = ring ? claim_slot(ring) : -1;
  if (slot < 0) return kNotLaunched;
  uint32_t* ctr = ring->ctr + slot * kCtrLine;
  uint32_t* busy = ring->busy_dev + slot * kBusyLine;
  (void)hipGetLastError();  // report this launch's error, not an earlier call's
  if (p.nb == 12)
    XRS_LAUNCH((staged_wsp_kernel<12, 12, NL, NN, T>), g, dim3(2 * T), stream, a, nt, ctr, busy);
  else if (p.nb == 13)
    XRS_LAUNCH((staged_wsp_kernel<12, 13, NL, NN, T>), g, dim3(2 * T), stream, a, nt, ctr, busy);
  else
    XRS_LAUNCH((staged_wsp_kernel<12, 14, NL, NN, T>), g, dim3(2 * T), stream, a, nt, ctr, busy);
  const hipError_t e = hipGetLastError();
  // not launched: the kernel will not release the slot, so release it here
  if (e != hipSuccess) __atomic_store_n(ring->busy + slot * kBusyLine, 0u, __ATOMIC_RELEASE);
  return static_cast<int>(e);
}

// Other codecs' clean lost-data patterns (na = nd = ND, nb = ND..ND+2: the
// surviving piggybacked parity past dpHas[:d]), 256 chunks per block.
template <int ND, int NL, int NN, int T = 256>
int launch_staged_ws_nd(StagedArgs<NL, NN, true> a, const StagedPlan& p, hipStream_t stream) {
  const uint64_t blocks = (a.total + T - 1) / T;
  if (blocks > kMaxBlocks) return static_cast<int>(hipErrorInvalidConfiguration);
  a.order = block_order(Shape::kStaged, true, p.half, blocks, T);
  const dim3 g(static_cast<unsigned>(blocks));
  if (p.nb == ND)
    XRS_LAUNCH((staged_ws_kernel<ND, ND, NL, NN, T>), g, dim3(2 * T), stream, a);
  else if (p.nb == ND + 1)
    XRS_LAUNCH((staged_ws_kernel<ND, ND + 1, NL, NN, T>), g, dim3(2 * T), stream, a);
  else
    XRS_LAUNCH((staged_ws_kernel<ND, ND + 2, NL, NN, T>), g, dim3(2 * T), stream, a);
  return static_cast<int>(hipGetLastError());
}

// NPRE < 0: every b-row early (NPRE = NB).
template <int NL, int NN, int BS, int NPRE>
int launch_staged_ct_bs(StagedArgs<NL, NN, true> a, const StagedPlan& p, hipStream_t stream) {
  const uint64_t blocks = (a.total + BS - 1) / BS;
  if (blocks > kMaxBlocks) return static_cast<int>(hipErrorInvalidConfiguration);
  a.order = block_order(Shape::kStaged, true, p.half, blocks, BS);
  const dim3 g(static_cast<unsigned>(blocks));
  if (p.nb == 12)
    XRS_LAUNCH((staged_ct_kernel<12, 12, NL, NN, BS, NPRE < 0 ? 12 : NPRE>), g, dim3(BS), stream, a);
  else if (p.nb == 13)
    XRS_LAUNCH((staged_ct_kernel<12, 13, NL, NN, BS, NPRE < 0 ? 13 : NPRE>), g, dim3(BS), stream, a);
  else
    XRS_LAUNCH((staged_ct_kernel<12, 14, NL, NN, BS, NPRE < 0 ? 14 : NPRE>), g, dim3(BS), stream, a);
  return static_cast<int>(hipGetLastError());
}

template <int NL, int NN, bool VEC>
int launch_staged_t(const StagedPlan& p, hipStream_t stream) {
  StagedArgs<NL, NN, VEC> a;
  std::memset(&a, 0, sizeof(a));
  const GF& gf = GF::get();
  for (int m = 0; m < kStSrc; ++m) {
    for (int q = 0; q < NL; ++q) a.at[m][q] = gf.tab(p.acoef[m][q]);
    for (int u = 0; u < NN; ++u) a.bt[m][u] = gf.tab(p.bcoef[m][u]);
    a.asrc[m] = p.asrc[m];
  }
  for (int m = 0; m < kStB; ++m) {
    a.bsrc[m] = p.bsrc[m];
    a.bret[m] = p.bret[m];
  }
  for (int q = 0; q < kStOut; ++q) {
    a.adst[q] = p.adst[q];
    a.bdst[q] = p.bdst[q];
    a.nmask[q] = p.nmask[q];
  }
  a.bstore = p.bstore;
  a.nr = 0;
  bool late = true;
  for (int m = 0; m < kStB; ++m) {
    if (!p.bret[m]) continue;
    if (a.nr == kStOut || !((p.bstore >> m) & 1u)) {
      late = false;
      break;
    }
    a.rb[a.nr] = m;
    a.rmask[a.nr++] = p.bret[m];
  }
  a.nd = p.nd;
  a.na = p.na;
  a.nb = p.nb;
  a.nl = p.nl;
  a.nn = p.nn;
  a.half = p.half;
  a.off0 = p.off0;
  a.chunks = VEC ? (p.end - p.off0) / 16 : (p.end - p.off0 + 3) / 4;
  a.total = a.chunks * p.n_stripes;
  if (a.total == 0) return 0;
  const uint64_t blocks = (a.total + kBlock - 1) / kBlock;
  if (blocks > kMaxBlocks) return static_cast<int>(hipErrorInvalidConfiguration);
  a.order = block_order(Shape::kStaged, VEC, p.half, blocks);
  // Late-b wins on grids that fill the chip (bandwidth-bound; measured:
  // profiles/r01_bench_multi_staged.log).  A grid smaller than one block per
  // CU is latency-bound: there the all-loads-first kernel pays one memory
  // round trip instead of two (a per-stripe call on host-mapped staging: one
  // PCIe round trip).  XRS_STAGED_LATE=0 / =1 forces either kernel.
  if (p.nb > kStSrc) {
    // Wide b-side (launch_staged checked: aligned, no ragged end, every
    // retrieveRS row written back, at most kStOut of them): only the
    // wave-specialised kernel holds kStB b-rows, on any grid.
    if constexpr (VEC) {
      if (!late) return kStagedDecline;
      if constexpr (NL == NN && NL >= 2 && NL <= 3) {
        // 16+p lost data vects on full grids: the compile-time form
        // (nb = 16..18; profiles/r02_staged_ws_nd16.log).  XRS_STAGED_CT=0
        // keeps the runtime one.
        const char* cv = std::getenv("XRS_STAGED_CT");
        if (p.nd == 16 && p.na == 16 && p.nl == NL && p.nn == NN && p.nb <= 18 &&
            blocks >= kLatencyGrid && !(cv && cv[0] == '0'))
          return launch_staged_ws_nd<16, NL, NN>(a, p, stream);
      }
      constexpr int T = 256;
      const uint64_t wblocks = (a.total + T - 1) / T;
      a.order = block_order(Shape::kStaged, true, p.half, wblocks, T);
      (void)hipGetLastError();
      XRS_LAUNCH((staged_ws_rt_kernel<NL, NN, T, kStB>), dim3(static_cast<unsigned>(wblocks)),
                         dim3(2 * T), stream, a);
      return static_cast<int>(hipGetLastError());
    } else {
      return kStagedDecline;
    }
  }
  const char* lv = std::getenv("XRS_STAGED_LATE");
  if (lv && *lv) late = late && lv[0] != '0';
  else late = late && blocks >= kLatencyGrid;
  (void)hipGetLastError();  // report this launch's error, not an earlier call's
  // (A compile-time survivor count, ND = 12, let the scheduler hoist the
  // b-row loads: 225-232 VGPRs plus scratch, also with a sched_barrier
  // between the a- and b-phases.  Runtime nd only.)
  if constexpr (VEC && NL == NN && NL >= 2 && NL <= 3) {
    // Compile-time counts for 2-3 lost data vects of d = 6, 8, 10, 14 codecs
    // (na = nd, nb = nd..nd+2): the wave-specialised kernel.  Against the
    // runtime one-wave late kernel (profiles/r02_staged_ws_nd.log): 4 KiB
    // vects +4 to +12% (10+4, 8+4, 6+3, 14+4, 10+2); 1 MiB vects +2 to +4% at
    // d = 6 and 14.  XRS_STAGED_CT=0 / XRS_STAGED_WS=0 turn it off.
    const char* cv = std::getenv("XRS_STAGED_CT");
    const char* wv = std::getenv("XRS_STAGED_WS");
    // From 256 KiB halves, 512 chunks per block for 2 lost, and for 3 lost at
    // d = 8, 10 (1 MiB vects: vs the runtime kernel 10+4 +0.7 / +0.9%, 8+4
    // +1.4 / +5.2%, where 256-chunk blocks lost 1-5%; vs 256-chunk blocks
    // 6+3 +1.6 / -3.4%, 14+4 +3.8 / -0.3%: profiles/r02_staged_ws_nd512.log;
    // at 4 KiB 512 loses 2%).
    const bool t512 = p.half >= (256u << 10) && (NL == 2 || p.nd == 8 || p.nd == 10);
    const bool nd_ct = late && p.na == p.nd && p.nl == NL && p.nn == NN && p.nb >= p.nd &&
                       p.nb <= p.nd + 2 && !(cv && cv[0] == '0') && !(wv && wv[0] == '0');
    if (nd_ct && t512) {
      switch (p.nd) {
        case 6: return launch_staged_ws_nd<6, NL, NN, 512>(a, p, stream);
        case 8: return launch_staged_ws_nd<8, NL, NN, 512>(a, p, stream);
        case 10: return launch_staged_ws_nd<10, NL, NN, 512>(a, p, stream);
        case 14: return launch_staged_ws_nd<14, NL, NN, 512>(a, p, stream);
        default: break;
      }
    }
    if (nd_ct) {
      switch (p.nd) {
        case 6: return launch_staged_ws_nd<6, NL, NN>(a, p, stream);
        case 8: return launch_staged_ws_nd<8, NL, NN>(a, p, stream);
        case 10: return launch_staged_ws_nd<10, NL, NN>(a, p, stream);
        case 14: return launch_staged_ws_nd<14, NL, NN>(a, p, stream);
        default: break;
      }
    }
  }
  if constexpr (VEC && NL == NN && NL >= 2) {
    // Compile-time counts for 12+4 losses of data vects (na = nd = 12,
    // nb = 12..14); XRS_STAGED_CT=0 keeps the runtime-count kernel (A/B).
    const char* cv = std::getenv("XRS_STAGED_CT");
    const bool ct = late && p.nd == 12 && p.na == 12 && p.nl == NL && p.nn == NN &&
                    p.nb >= 12 && p.nb <= 14 && !(cv && cv[0] == '0');
    if (ct) {
      // (8 bytes per lane, twice the lanes at 56-70 VGPRs: 2-10% slower,
      // profiles/r02_multi2.log; 128-, 512- and 1024-thread blocks: 0-7%
      // slower at 4 KiB, within 1% at 1 MiB, profiles/r02_multi_bs.log.)
      // Every row's load up front (one round trip, 144-161 VGPRs) on halves
      // under 256 KiB: +2.6-2.8% on 2-3 lost at 4 KiB vects, +1-2.6% at
      // 256 KiB; at 1 MiB the two-phase kernel is 1-5% faster
      // (profiles/r02_multi3.log, r02_multi_order_e{0,1}.log).
      // XRS_STAGED_EARLY=0 / =1 forces either (A/B, tests).
      const char* ev = std::getenv("XRS_STAGED_EARLY");
      const bool early = (ev && *ev) ? ev[0] == '1' : p.half < (256u << 10);
      // (b-row loads split between the phases, 4 / 6 / 8 with the a-rows:
      // within 1% of the better end; 128-thread blocks x every block order:
      // the defaults within 1% of the best at 4 KiB, 256 KiB and 1 MiB:
      // profiles/r02_staged_npre.log, r02_staged_bs_order.log; the late
      // kernel in 512- and 1024-thread blocks, K = 8..128, from 512 KiB to
      // 8 MiB vects: -3..+2.3%, within noise: r02_staged_big_{bs,confirm}.log;
      // each survivor's a- and b-half loads back to back: +-1%, r02_staged_il.log)
      // 2-3 lost: the wave-specialised kernel, 256 chunks per 512-lane block
      // (bytes moved, interleaved medians vs the kernels above: 2 lost @ 4 KiB
      // / 64 KiB / 256 KiB / 1 MiB +5.5 / +0.5 / +2.1 / 0%, 3 lost +4.0 /
      // +0.5 / +1.4 / +6.5%; 4 lost -1..-7%, so it keeps the one-wave kernel;
      // 64-, 128- and 512-chunk blocks and a 5-wave VGPR cap: no better
      // overall; profiles/r02_staged_ws.log).  XRS_STAGED_WS=0 / 64 / 128 /
      // 256 / 512 / 128o5 forces it off or a block size (A/B, tests).
      // 2 lost from 512 KiB vects: 512 chunks per block (+1.2 / +2.3 / +4.2%
      // at 1 MiB / 512 KiB / 2 MiB vects over 256; at 256 KiB vects -4%).
      const char* wv = std::getenv("XRS_STAGED_WS");
      // 2 lost from 256 to 768 KiB halves: the persistent form, 512 chunks
      // per tile (bytes moved, interleaved medians vs the one-shot 512-chunk
      // kernel, profiles/r04_wsp_ab.log: 512 KiB / 768 KiB / 1 MiB / 1.5 MiB
      // vects +2.9 / -0.1 / +4.2 / +2.6%; 2 / 4 / 8 MiB -1.8 / +0.7 / -14.7%,
      // so larger halves keep the one-shot kernel; 3 lost -2..-4% and
      // 256-chunk tiles -5..-21%, profiles/r04_wsp_sizes.log).
      // Only launches of at least XRS_WSP_MIN_TILES tiles per CU (default
      // 4: 16 stripes of 1 MiB).  With the self-resetting counter slots
      // (tile_counters) a synchronous call costs what the kernel does:
      // 1 / 4 / 16 / 64 / 256 stripes of 1 MiB (0.25 .. 64 tiles per CU)
      // -0.1 / +0.6 / -3.3 / -7.7 / -37 us against the one-shot kernel
      // (tools/wsp_call_overhead.py, profiles/r05_wsp_overhead.log; the
      // round-4 per-launch alloc + memset + free cost +7.0 / +2.4 us at 4 /
      // 16 stripes, r04_wsp_overhead.log, hence a gate of 16 tiles then).
      // XRS_WSP=0 turns it off, =512 / =256 forces it (A/B, tests).
      const char* pv = std::getenv("XRS_WSP");
      const bool wsp_off = pv && pv[0] == '0';
      const char* mt = std::getenv("XRS_WSP_MIN_TILES");
      const uint64_t min_tiles = (mt && *mt) ? std::strtoull(mt, nullptr, 10) : uint64_t(4);
      int wsp = kNotLaunched;
      if (pv && std::strcmp(pv, "256") == 0) wsp = launch_staged_wsp<NL, NN, 256>(a, p, stream);
      else if (pv && std::strcmp(pv, "512") == 0) wsp = launch_staged_wsp<NL, NN, 512>(a, p, stream);
      else if (NL == 2 && !wsp_off && (!wv || !*wv || std::strcmp(wv, "rt") == 0) &&
               p.half >= (256u << 10) && p.half <= (768u << 10) &&
               a.total >= uint64_t(512) * min_tiles * static_cast<uint64_t>(cu_count(stream)))
        wsp = launch_staged_wsp<NL, NN, 512>(a, p, stream);
      if (wsp != kNotLaunched) return wsp;
      if (!wv || !*wv || std::strcmp(wv, "rt") == 0) {
        if (NL == 2 && p.half >= (256u << 10)) return launch_staged_ws<NL, NN, 512>(a, p, stream);
        if (NL <= 3) return launch_staged_ws<NL, NN, 256>(a, p, stream);
      } else {
        if (std::strcmp(wv, "128") == 0) return launch_staged_ws<NL, NN, 128>(a, p, stream);
        if (std::strcmp(wv, "256") == 0) return launch_staged_ws<NL, NN, 256>(a, p, stream);
        if (std::strcmp(wv, "64") == 0) return launch_staged_ws<NL, NN, 64>(a, p, stream);
        if (std::strcmp(wv, "512") == 0) return launch_staged_ws<NL, NN, 512>(a, p, stream);
        if (std::strcmp(wv, "128o5") == 0) return launch_staged_ws<NL, NN, 128, 5>(a, p, stream);
      }
      if (early) return launch_staged_ct_bs<NL, NN, kBlock, -1>(a, p, stream);
      return launch_staged_ct_bs<NL, NN, kBlock, 0>(a, p, stream);
    }
  }
  if constexpr (VEC && NL == 1 && NN == 1) {
    // One lost and needed parity vect of 12+4 (P12: nb = 15; P13-P15:
    // nb = 14), every a-row a survivor: the compile-time wave-specialised
    // kernel (reference bench xrs_test.go:523-574 patterns).
    // XRS_STAGED_CT=0 keeps the runtime-count one below.
    const char* cv = std::getenv("XRS_STAGED_CT");
    const char* wv = std::getenv("XRS_STAGED_WS");
    const bool ct1 = late && p.nd == 12 && p.na == 12 && p.nl == 1 && p.nn == 1 && p.nb >= 12 &&
                     p.nb <= 15 && !(cv && cv[0] == '0') && !(wv && *wv);
    if (ct1) {
      if (p.half >= (256u << 10)) return launch_staged_ws<1, 1, 512>(a, p, stream);
      return launch_staged_ws<1, 1, 256>(a, p, stream);
    }
  }
  if constexpr (VEC) {
    // Runtime-count wave-specialised kernel for one lost and needed vect
    // with parity in the pattern (12+4, lost P12 / P13: +3.4 / +1.3% at 4 KiB,
    // +3.3 / +0.2% at 1 MiB).  With more outputs it wins or loses by pattern
    // (12+4 lost {0, 13}: +8% at 4 KiB, -2% at 1 MiB) and loses 3-10% on
    // lost data at 10+4 and 6+3, so the one-wave late kernel stays there
    // (profiles/r02_staged_ws_rt.log).  XRS_STAGED_WS=rt forces it for every
    // runtime-count launch, =0 never.
    const char* wv = std::getenv("XRS_STAGED_WS");
    const bool ws_rt = (wv && *wv) ? std::strcmp(wv, "rt") == 0 : (NL == 1 && NN == 1);
    if (late && ws_rt) {
      constexpr int T = 256;
      const uint64_t wblocks = (a.total + T - 1) / T;
      a.order = block_order(Shape::kStaged, true, p.half, wblocks, T);
      XRS_LAUNCH((staged_ws_rt_kernel<NL, NN, T>), dim3(static_cast<unsigned>(wblocks)),
                         dim3(2 * T), stream, a);
      return static_cast<int>(hipGetLastError());
    }
  }
  if (late)
    XRS_LAUNCH((staged_late_kernel<NL, NN, VEC>), dim3(static_cast<unsigned>(blocks)),
                       dim3(kBlock), stream, a);
  else
    XRS_LAUNCH((staged_kernel<NL, NN, VEC>), dim3(static_cast<unsigned>(blocks)),
                       dim3(kBlock), stream, a);
  return static_cast<int>(hipGetLastError());
}

// Exact-count instantiations for lost-data-only Reconst (nl == nn, the common
// case); everything else runs the 4/4 kernel with zero padding.
template <bool VEC>
int launch_staged_r(const StagedPlan& p, hipStream_t s) {
  if constexpr (VEC) {
    if (p.nl == p.nn) {
      switch (p.nl) {
        case 1: return launch_staged_t<1, 1, VEC>(p, s);
        case 2: return launch_staged_t<2, 2, VEC>(p, s);
        case 3: return launch_staged_t<3, 3, VEC>(p, s);
        default: break;
      }
    }
  }
  return launch_staged_t<4, 4, VEC>(p, s);
}

template <int P, bool VEC, bool IND = false>
int launch_update_rows_t(const UpdRowsPlan& p, hipStream_t stream) {
  UpdRowsArgs<P, VEC> a;
  std::memset(&a, 0, sizeof(a));
  for (int j = 0; j < p.nrows; ++j) {
    for (int q = 0; q < P; ++q) a.tab[j][q] = p.tab[j][q];
    a.pbq[j] = p.pbq[j];
  }
  a.old_row = p.old_row;
  a.new_row = p.new_row;
  for (int q = 0; q < P; ++q) a.dst[q] = p.dst[q];
  a.rows = reinterpret_cast<const int32_t*>(p.rows);
  a.row0 = p.row0;
  a.nrows = p.nrows;
  a.half = p.half;
  a.off0 = p.off0;
  a.chunks = VEC ? (p.end - p.off0) / 16 : (p.end - p.off0 + 3) / 4;
  a.total = a.chunks * p.n_stripes;
  if (a.total == 0) return 0;
  const uint64_t blocks = (a.total + kBlock - 1) / kBlock;
  if (blocks > kMaxBlocks) return static_cast<int>(hipErrorInvalidConfiguration);
  a.order = block_order(Shape::kPair, VEC, p.half, blocks);
  (void)hipGetLastError();  // report this launch's error, not an earlier call's
  if constexpr (IND)
    XRS_LAUNCH((update_rows_ind_kernel<P, VEC>), dim3(static_cast<unsigned>(blocks)), dim3(kBlock),
               stream, a);
  else
    XRS_LAUNCH((update_rows_kernel<P, VEC>), dim3(static_cast<unsigned>(blocks)),
                       dim3(kBlock), stream, a);
  return static_cast<int>(hipGetLastError());
}

template <bool VEC, bool IND = false>
int launch_update_rows_p(const UpdRowsPlan& p, hipStream_t s) {
  switch (p.P) {
    case 1: return launch_update_rows_t<1, VEC, IND>(p, s);
    case 2: return launch_update_rows_t<2, VEC, IND>(p, s);
    case 3: return launch_update_rows_t<3, VEC, IND>(p, s);
    case 4: return launch_update_rows_t<4, VEC, IND>(p, s);
    default: return static_cast<int>(hipErrorInvalidValue);
  }
}

// Kernel arguments of a pair / rows plan (everything but the block order).
template <int P, int C, bool VEC>
void fill_pair_args(PairArgs<P, C, VEC>& a, const PairPlan& p) {
  const int n = p.C;
  for (int c = 0; c < n; ++c) {
    for (int r = 0; r < P; ++r) a.tab[c][r] = p.tab[c][r];
    a.src[c] = p.src[c];
  }
  for (int r = 0; r < P; ++r) {
    a.dst[r] = p.dst[r];
    a.pbmask[r] = 0;
  }
  for (int c = 0; c < n; ++c)
    if (p.pb[c] >= 0) a.pbmask[p.pb[c]] |= 1u << c;
  a.n_src = n;
  a.half = p.half;
  a.off0 = p.off0;
  a.chunks = VEC ? (p.end - p.off0 + 15) / 16 : (p.end - p.off0 + 3) / 4;
  a.last = (VEC && p.overlap) ? p.end - 16 : ~uint64_t(0);
  a.total = a.chunks * p.n_stripes;
}

template <int R, int NM, int NX, bool VEC>
void fill_rows_args(RowsArgs<R, NM, NX, VEC>& a, const RowsPlan& p) {
  for (int m = 0; m < p.NM; ++m) {
    for (int r = 0; r < R; ++r) a.tab[m][r] = p.tab[m][r];
    a.msrc[m] = p.msrc[m];
  }
  for (int x = 0; x < p.NX; ++x) {
    a.xsrc[x] = p.xsrc[x];
    a.xmask[x] = p.xmask[x];
  }
  for (int r = 0; r < R; ++r) a.dst[r] = p.dst[r];
  a.nm = p.NM;
  a.nx = p.NX;
  a.len = p.len;
  a.off0 = p.off0;
  a.chunks = VEC ? (p.end - p.off0 + 15) / 16 : (p.end - p.off0 + 3) / 4;
  a.last = (VEC && p.overlap) ? p.end - 16 : ~uint64_t(0);
  a.total = a.chunks * p.n_stripes;
}

// Indirect-row launches (xrs_plan.h kRowInd: the queue's batches of callers'
// own buffers): runtime counts, 256-thread blocks, the family's block order.
// Small batches of host-resident rows are bound by PCIe round trips, not by
// the kernel's shape, so the bodies read every row base first (one round
// trip) and group their data loads (kbody_*.h, XRS_IND).
template <int P, bool ACC, bool VEC>
int launch_pair_ind_t(const PairPlan& p, hipStream_t stream) {
  PairArgs<P, kDyn, VEC> a;
  fill_pair_args(a, p);
  if (a.total == 0) return 0;
  const uint64_t blocks = (a.total + kBlock - 1) / kBlock;
  if (blocks > kMaxBlocks) return static_cast<int>(hipErrorInvalidConfiguration);
  a.order = block_order(Shape::kPair, VEC, p.half, blocks);
  (void)hipGetLastError();  // report this launch's error, not an earlier call's
  XRS_LAUNCH((pair_ind_kernel<P, ACC, VEC>), dim3(static_cast<unsigned>(blocks)), dim3(kBlock),
             stream, a);
  return static_cast<int>(hipGetLastError());
}

template <bool ACC, bool VEC>
int launch_pair_ind_p(const PairPlan& p, hipStream_t s) {
  switch (p.P) {
    case 1: return launch_pair_ind_t<1, ACC, VEC>(p, s);
    case 2: return launch_pair_ind_t<2, ACC, VEC>(p, s);
    case 3: return launch_pair_ind_t<3, ACC, VEC>(p, s);
    case 4: return launch_pair_ind_t<4, ACC, VEC>(p, s);
    default: return static_cast<int>(hipErrorInvalidValue);
  }
}

template <int R, bool ACC, bool VEC>
int launch_rows_ind_t(const RowsPlan& p, hipStream_t stream) {
  RowsArgs<R, kDyn, kDyn, VEC> a;
  fill_rows_args(a, p);
  if (a.total == 0) return 0;
  const uint64_t blocks = (a.total + kBlock - 1) / kBlock;
  if (blocks > kMaxBlocks) return static_cast<int>(hipErrorInvalidConfiguration);
  a.order = block_order(Shape::kRows, VEC, p.len, blocks);
  a.grouped = true;  // (the indirect body always runs the grouped loop)
  (void)hipGetLastError();  // report this launch's error, not an earlier call's
  XRS_LAUNCH((rows_ind_kernel<R, ACC, VEC>), dim3(static_cast<unsigned>(blocks)), dim3(kBlock),
             stream, a);
  return static_cast<int>(hipGetLastError());
}

template <bool ACC, bool VEC>
int launch_rows_ind_r(const RowsPlan& p, hipStream_t s) {
  switch (p.R) {
    case 1: return launch_rows_ind_t<1, ACC, VEC>(p, s);
    case 2: return launch_rows_ind_t<2, ACC, VEC>(p, s);
    case 3: return launch_rows_ind_t<3, ACC, VEC>(p, s);
    case 4: return launch_rows_ind_t<4, ACC, VEC>(p, s);
    default: return static_cast<int>(hipErrorInvalidValue);
  }
}

template <int P, int C, bool ACC, bool VEC>
int launch_pair_t(const PairPlan& p, hipStream_t stream) {
  PairArgs<P, C, VEC> a;
  const int n = p.C;
  fill_pair_args(a, p);
  if (a.total == 0) return 0;
  // 128-thread blocks for the 16-byte kernels on halves up to 4 KiB (Encode
  // at 4 KiB +1-2.5% over 256: profiles/r01_blocksize.log) and for 12+
  // sources at any size (interleaved A/B at 1 / 4 MiB: 12+4 +1.4 / -0.3%,
  // 14+4 0 / +6%, 16+4 +8% @ 1 MiB, 20-28+4 -2..+7%); fewer sources keep 256
  // (8+4, 10+2, 4+2: -1.4..-4.7% with 128): profiles/r02_pairblock_ab*.log.
  // XRS_PAIR_BLOCK=256 / 128 forces either.
  const char* pb = std::getenv("XRS_PAIR_BLOCK");
  const int bs = !VEC ? kBlock
                      : (pb && *pb) ? env_block("XRS_PAIR_BLOCK", 128)
                                    : (p.half <= 4096 || n >= 12 ? 128 : kBlock);
  const uint64_t blocks = (a.total + bs - 1) / bs;
  if (blocks > kMaxBlocks) return static_cast<int>(hipErrorInvalidConfiguration);
  a.order = block_order(Shape::kPair, VEC, p.half, blocks, bs);
  // The 12+4 Encode from 1 MiB vects up streams 2-5% faster in the plain
  // block order (1, 1.5, 2, 4, 8 MiB; 768 KiB even, 512 KiB -1.3%); other
  // codecs at 1 MiB lose 1-3% with it (profiles/r02_enc_k0*.log).
  // Update / Replace (accumulating) on halves up to 4 KiB: each XCD a
  // contiguous eighth of the grid, as the rows kernel at 4 KiB (Replace(1, 2,
  // 4, 8) @ 4 KiB +4-10%, @ 8 KiB +3-7%; Update +2%:
  // profiles/r02_updrep_order*.log).
  // A batch of 48 GiB or more of 12+4 stripes streams best in K = 128
  // instead (8,192 x 1 MiB = 128 GiB: plain 6.04 TB/s, K = 128 6.13; 64 GiB:
  // 6.13 / 6.15; 32 GiB: plain +2.3%: profiles/r02_c5_order.log).
  const bool forced = std::getenv("XRS_BLOCK_ORDER") != nullptr;
  const bool enc12 = P == 4 && C == 12 && !ACC && bs == 128 && p.half >= (512u << 10) && !forced;
  const bool huge = p.n_stripes * 32 * p.half >= (48ull << 30);
  const bool plain12 = enc12 && !huge;
  if (plain12) a.order.k = 0;
  if (enc12 && huge) a.order.k = 128;
  if (ACC && VEC && p.half <= 4096 && !forced) a.order.k = static_cast<uint32_t>(blocks / 8);
  (void)hipGetLastError();  // report this launch's error, not an earlier call's
  if constexpr (VEC && P == 4 && C != kDyn && !ACC) {
    // The wave-specialised Encode (enc_ws_kernel), 256 chunks per block of
    // 512 lanes, on halves a multiple of 16 bytes up to 128 KiB (bytes moved,
    // interleaved medians vs the pair kernel, profiles/r04_encws_mid.log:
    // 4 / 8 / 32 / 64 / 128 / 256 KiB vects +3.6 / +3.8 / +4.2 / +4.7 /
    // -0.5 / +3.7%; 384 KiB -1%, 512 KiB -3%, 1 MiB -1.6..+1.1%, so larger
    // halves keep the pair kernel; r04_encws_4k.log, r04_encws_order.log).
    // The same holds for 8+4 and 10+4 (4 / 64 KiB vects +4.5 / +0.9% and
    // +8.8 / +1.9%), not for 14+4, 16+4 (-1.9..+1.5%) or 20+4 (-13..-19%,
    // 134 VGPRs): profiles/r04_encws_codecs.log.  XRS_ENC_WS forces it for
    // every d+4 compile-time shape (A/B); =0 turns it off, =128 / 256 / 512
    // sets the block size (12+4; 256 for the others), any other value forces
    // it on with 256 chunks per block.
    const char* ew = std::getenv("XRS_ENC_WS");
    const bool ws_on = (ew && *ew) ? ew[0] != '0' : (C <= 12 && p.half <= (128u << 10));
    // (Ragged halves keep the pair kernel: the overlapping-last-chunk form of
    // this kernel measured 3.3-12% slower at 4,100 / 4,098 / 2,052 / 65,540 B
    // and +0.8% at 262,146 B, profiles/r05_encws_ragged.log.)
    if (ws_on && p.half % 16 == 0) {
      int T = 256;  // the block size launched below, which also sets the grid
      if (C == 12 && ew && (std::strcmp(ew, "128") == 0 || std::strcmp(ew, "512") == 0))
        T = std::strcmp(ew, "128") == 0 ? 128 : 512;
      const uint64_t tb = (a.total + T - 1) / T;
      if (tb > kMaxBlocks) return static_cast<int>(hipErrorInvalidConfiguration);
      a.order = block_order(Shape::kPair, VEC, p.half, tb, T);
      if (const char* e = std::getenv("XRS_ENC_WS_ORDER"))  // A/B
        a.order.k = static_cast<uint32_t>(std::strtoul(e, nullptr, 10));
      const dim3 g(static_cast<unsigned>(tb));
      if constexpr (C == 12) {
        if (T == 128) XRS_LAUNCH((enc_ws_kernel<12, 128>), g, dim3(256), stream, a);
        else if (T == 512) XRS_LAUNCH((enc_ws_kernel<12, 512>), g, dim3(1024), stream, a);
        else XRS_LAUNCH((enc_ws_kernel<12, 256>), g, dim3(512), stream, a);
      } else {
        XRS_LAUNCH((enc_ws_kernel<C, 256>), g, dim3(512), stream, a);
      }
      return static_cast<int>(hipGetLastError());
    }
  }
  if constexpr (VEC && P == 4 && C == 12 && !ACC) {
    if (plain12) {
      XRS_LAUNCH((pair_kernel<P, C, ACC, VEC, 128, true>), dim3(static_cast<unsigned>(blocks)),
                         dim3(128), stream, a);
      return static_cast<int>(hipGetLastError());
    }
  }
  if constexpr (VEC) {
    if (bs == 128) {
      XRS_LAUNCH((pair_kernel<P, C, ACC, VEC, 128>), dim3(static_cast<unsigned>(blocks)),
                         dim3(128), stream, a);
      return static_cast<int>(hipGetLastError());
    }
  }
  XRS_LAUNCH((pair_kernel<P, C, ACC, VEC>), dim3(static_cast<unsigned>(blocks)),
                     dim3(kBlock), stream, a);
  return static_cast<int>(hipGetLastError());
}

// Compile-time source counts per output count for a whole Encode (every load
// issued before the first multiply): 12+4 (the headline) and the common
// codecs around it.  Anything else runs the runtime-count kernel.
template <int P>
struct EncodeShapes;
template <>
struct EncodeShapes<2> {
  using type = std::integer_sequence<int, 4, 6, 8, 10, 12>;
};
template <>
struct EncodeShapes<3> {
  using type = std::integer_sequence<int, 6, 8, 10, 12>;
};
template <>
struct EncodeShapes<4> {
  using type = std::integer_sequence<int, 8, 10, 12, 14, 16, 20>;
};

template <int P, bool VEC, int... Cs>
int launch_encode_ct(const PairPlan& p, hipStream_t s, std::integer_sequence<int, Cs...>) {
  int rc = -1;
  (void)((p.C == Cs && (rc = launch_pair_t<P, Cs, false, VEC>(p, s), true)) || ...);
  return rc;
}

// Padding to a compile-time Encode shape: a source count without its own
// instantiation runs the smallest instantiated count above it when that adds
// at most kPadRows rows.  A padding row is an all-zero row (zero_rows(), read
// with stripe stride 0, so every stripe reads the same few cache lines): its
// GF products and its piggyback XOR are zero, and the kernel is unchanged (a
// guard on the piggyback instead raised the 12+4 Encode from 170 to 258
// VGPRs).
constexpr int kPadRows = 3;

// The zero rows of the device the launch stream belongs to (not the calling
// thread's current device: a batched call may run on another GPU's stream).
uint64_t zero_rows_for(hipStream_t s) {
  int dev = -1;
  if (hipStreamGetDevice(s, &dev) != hipSuccess) return 0;
  return zero_rows(dev);
}

template <int... Cs>
int pad_count(int c, std::integer_sequence<int, Cs...>) {
  int best = -1;
  (void)((Cs > c && Cs <= c + kPadRows && (best < 0 || Cs < best) && (best = Cs, true)) || ...);
  return best;
}

bool pad_disabled() {
  const char* e = std::getenv("XRS_PAD");
  return e && e[0] == '0';
}

// Compile-time source counts of an accumulating launch with four outputs:
// Replace(n) at p = 4, n = 1..8 (the reference's Replace benchmark,
// xrs_test.go:627-680).
template <bool VEC, int... Cs>
int launch_replace_ct(const PairPlan& p, hipStream_t s, std::integer_sequence<int, Cs...>) {
  int rc = -1;
  (void)((p.C == Cs && (rc = launch_pair_t<4, Cs, true, VEC>(p, s), true)) || ...);
  return rc;
}

template <int P, bool ACC, bool VEC>
int launch_pair_c(const PairPlan& p, hipStream_t s) {
  if constexpr (!ACC && VEC && P >= 2) {
    if (p.encode_xs && !std::getenv("XRS_ENCODE_DYN")) {
      const int rc = launch_encode_ct<P, VEC>(p, s, typename EncodeShapes<P>::type{});
      if (rc != -1) return rc;
      const int cs = pad_count(p.C, typename EncodeShapes<P>::type{});
      // Halves up to 4 KiB only: Encode at 4 KiB vects +1..+12% over the
      // runtime kernel on ten codecs; from 16 KiB vects the runtime kernel is
      // as fast or faster (-10..+4%, 1 MiB -5..+2%;
      // profiles/r03_pad_ab2.log, r03_pad_ab3.log).
      const uint64_t z = (cs > 0 && p.C > 0 && p.half <= 4096 && !pad_disabled()) ? zero_rows_for(s) : 0;
      if (z) {
        PairPlan q = p;
        for (int c = p.C; c < cs; ++c) {
          q.src[c] = RowRef{z, 0};
          for (int r = 0; r < kMaxOut; ++r) q.tab[c][r] = GfTab{0, 0, 0, 0, 0};
          q.pb[c] = -1;
        }
        q.C = cs;
        (void)hipGetLastError();
        const int prc = launch_encode_ct<P, VEC>(q, s, typename EncodeShapes<P>::type{});
        if (prc != -1) return prc;
      }
    }
  }
  if constexpr (ACC && VEC && P == 4) {
    // Compile-time Replace(n): +0.5-2% at 8 MiB for every n and +2-4% at
    // 4 KiB for n >= 5; at 4 KiB with n <= 4 the runtime kernel is as fast
    // or up to 4% faster (profiles/r02_replace_ab.log).
    if ((p.half > 4096 || p.C >= 5) && !std::getenv("XRS_REPLACE_DYN")) {
      const int rc = launch_replace_ct<VEC>(p, s, std::integer_sequence<int, 1, 2, 3, 4, 5, 6, 7, 8>{});
      if (rc != -1) return rc;
    }
  }
  // (Compile-time Update (C=2) and Replace(4) shapes measured no faster than
  // the runtime kernel at 8 MiB: profiles/r01_bench_configs_c4_ct.log.)
  return launch_pair_t<P, kDyn, ACC, VEC>(p, s);
}

template <bool ACC, bool VEC>
int launch_pair_p(const PairPlan& p, hipStream_t s) {
  switch (p.P) {
    case 1: return launch_pair_c<1, ACC, VEC>(p, s);
    case 2: return launch_pair_c<2, ACC, VEC>(p, s);
    case 3: return launch_pair_c<3, ACC, VEC>(p, s);
    case 4: return launch_pair_c<4, ACC, VEC>(p, s);
    default: return static_cast<int>(hipErrorInvalidValue);
  }
}

template <int R, int NM, int NX, bool ACC, bool VEC>
int launch_rows_t(const RowsPlan& p, hipStream_t stream) {
  RowsArgs<R, NM, NX, VEC> a;
  fill_rows_args(a, p);
  if (a.total == 0) return 0;
  // 1024-thread blocks for rows of >= 256 KiB (ReconstOne at 1 MiB vects:
  // +3-5% over 256, profiles/r01_blocksize.log); XRS_ROWS_BLOCK=256 for A/B.
  // Also 1024 for the compile-time shapes of 18-22 rows on rows of up to
  // 4 KiB (ReconstOne 16+4 / 14+4 @ 4 KiB +3.5% / +1.9%; 12+3 even; 12+4, 16
  // rows, -10%: profiles/r02_rows_bs.log).  XRS_ROWS_BLOCK=1024 forces it at
  // any length (A/B), =256 turns both rules off.
  constexpr bool kWide = NM != kDyn && NM + NX >= 18 && NM + NX <= 22;
  const char* rbv = std::getenv("XRS_ROWS_BLOCK");
  const bool force1024 = rbv && std::atoi(rbv) == 1024;
  const bool big = p.len >= (256u << 10) || (kWide && p.len <= 4096) || force1024;
  const int bs = (VEC && big) ? env_block("XRS_ROWS_BLOCK", 1024) : kBlock;
  const uint64_t blocks = (a.total + bs - 1) / bs;
  if (blocks > kMaxBlocks) return static_cast<int>(hipErrorInvalidConfiguration);
  a.order = block_order(Shape::kRows, VEC, p.len, blocks, bs);
  // XRS_ROWS_GROUPED=0 / =1 forces either runtime-count loop (A/B, tests).
  const char* gv = std::getenv("XRS_ROWS_GROUPED");
  a.grouped = (gv && *gv) ? gv[0] != '0' : blocks * bs < kLatencyGrid * kBlock;
  (void)hipGetLastError();  // report this launch's error, not an earlier call's
  if constexpr (VEC) {
    if (bs == 1024) {
      XRS_LAUNCH((rows_kernel<R, NM, NX, ACC, VEC, 1024>),
                         dim3(static_cast<unsigned>(blocks)), dim3(1024), stream, a);
      return static_cast<int>(hipGetLastError());
    }
  }
  XRS_LAUNCH((rows_kernel<R, NM, NX, ACC, VEC>), dim3(static_cast<unsigned>(blocks)),
                     dim3(kBlock), stream, a);
  return static_cast<int>(hipGetLastError());
}

// Compile-time (NM, NX) of ReconstOne (two outputs; NM = d survivors' b-halves,
// NX = |XORSet(bi)| rows XORed in) for 12+4 (the headline) and the common
// codecs: (d, p) -> NX in {floor, ceil}(d / (p-1)).
template <int NM, int NX>
struct Shape2 {};
template <bool VEC, int... NMs, int... NXs>
int launch_reconst_one_ct(const RowsPlan& p, hipStream_t s, Shape2<NMs, NXs>...) {
  int rc = -1;
  (void)(((p.NM == NMs && p.NX == NXs) && (rc = launch_rows_t<2, NMs, NXs, false, VEC>(p, s), true)) ||
         ...);
  return rc;
}

template <int R, bool ACC, bool VEC>
int launch_rows_c(const RowsPlan& p, hipStream_t s) {
  if constexpr (R == 2 && !ACC && VEC) {  // (the byte path of these shapes would use scratch)
    // More than 22 rows in a 1024-thread block (rows of >= 256 KiB) would
    // spill (128 VGPRs at most); those run the runtime-count kernel
    // (20+4 ReconstOne @ 1 MiB: 0.66 compile-time with scratch, 0.76 runtime;
    // profiles/r02_others_ab.log).
    const bool fits = p.len < (256u << 10) || p.NM + p.NX <= 22;
    if (fits && !std::getenv("XRS_ROWS_DYN")) {
      auto ct = [&](const RowsPlan& q) {
        return launch_reconst_one_ct<VEC>(
            q, s, Shape2<12, 4>{},                     // 12+4
            Shape2<4, 4>{}, Shape2<6, 3>{},            // 4+2, 6+3
            Shape2<8, 2>{}, Shape2<8, 3>{},            // 8+4
            Shape2<10, 3>{}, Shape2<10, 4>{},          // 10+4
            Shape2<12, 6>{},                           // 12+3
            Shape2<14, 4>{}, Shape2<14, 5>{},          // 14+4
            Shape2<16, 5>{}, Shape2<16, 6>{},          // 16+4
            Shape2<20, 6>{}, Shape2<20, 7>{},          // 20+4
            Shape2<10, 10>{});                         // 10+2
      };
      const int rc = ct(p);
      if (rc != -1) return rc;
      // (Padding to the nearest (NM, NX) instantiation, as Encode does, lost
      // 0.5-7% against the runtime kernel: profiles/r03_pad_ab.log.)
    }
  }
  return launch_rows_t<R, kDyn, kDyn, ACC, VEC>(p, s);
}

template <bool ACC, bool VEC>
int launch_rows_r(const RowsPlan& p, hipStream_t s) {
  switch (p.R) {
    case 1: return launch_rows_c<1, ACC, VEC>(p, s);
    case 2: return launch_rows_c<2, ACC, VEC>(p, s);
    case 3: return launch_rows_c<3, ACC, VEC>(p, s);
    case 4: return launch_rows_c<4, ACC, VEC>(p, s);
    default: return static_cast<int>(hipErrorInvalidValue);
  }
}

// Each half (or row) of `len` bytes runs as [0, bulk) on the 16-byte kernels
// and [bulk, len) on the byte-granular ones (bulk = len rounded down to 16).
// MI355X executes global dwordx4 accesses at any byte alignment (the
// runtime's unaligned access mode): exact, and 3-9% slower than aligned ones
// (tools/unaligned_probe.hip, profiles/r01_unaligned_probe.log), so neither
// misaligned rows / strides nor a ragged length force the byte path any more
// (4-5x slower: profiles/r01_odd_probe.log).  XRS_UNALIGNED_VEC=0 restores
// the strict rule for A/B runs: 16-byte kernels only when every row, stride
// and len is 16-byte aligned.
//
// Ragged end without a second launch (`overlap_ok`: the launch writes each
// output byte as a pure function of input bytes at the same offset, i.e. no
// accumulate and no output row that is also an input row): when len >= 16 is
// not a multiple of 16, the 16-byte launch covers [0, len) with one more
// chunk per row, starting at len - 16.  It overlaps the previous chunk, whose
// bytes it rewrites with the same values.  The separate byte-granular tail
// launch touched one line per row per stripe and cost 10-35% at 4,100-byte
// vects (profiles/r01_odd_probe.log).  XRS_TAIL=launch restores it (A/B).
template <class Plan, class F>
int split_launch(Plan p, uint64_t len, bool aligned, F launch, bool overlap_ok = false) {
  const char* e = std::getenv("XRS_UNALIGNED_VEC");
  uint64_t bulk = len & ~uint64_t(15);
  if (e && e[0] == '0' && !(aligned && bulk == len)) bulk = 0;
  const char* tv = std::getenv("XRS_TAIL");
  if (overlap_ok && bulk && bulk < len && !(tv && std::strcmp(tv, "launch") == 0)) {
    p.off0 = 0;
    p.end = len;
    p.overlap = true;
    return launch(p, true);
  }
  int rc = 0;
  if (bulk) {
    p.off0 = 0;
    p.end = bulk;
    rc = launch(p, true);
  }
  if (!rc && len > bulk) {
    p.off0 = bulk;
    p.end = len;
    rc = launch(p, false);
  }
  return rc;
}

bool row_aligned(const RowRef& r) { return aligned16(r.ptr) && aligned16(r.stripe_stride); }
bool row_ind(const RowRef& r) { return (r.stripe_stride & kRowInd) != 0; }

// Two rows of `len` bytes share a byte in some pair of stripes s, t <
// n_stripes (row a of stripe s against row b of stripe t), or step
// differently (then assume they may meet).  With equal strides S the rows
// meet iff |delta - m*S| < len for some m in (-n_stripes, n_stripes), delta =
// b.ptr - a.ptr; the nearest m are floor(delta / S) and the next one, clamped.
bool rows_overlap(const RowRef& a, const RowRef& b, uint64_t len, uint64_t n_stripes) {
  if (a.stripe_stride != b.stripe_stride) return true;
  const __int128 delta = static_cast<__int128>(b.ptr) - static_cast<__int128>(a.ptr);
  const __int128 S = a.stripe_stride;
  auto near = [&](__int128 m) {
    const __int128 r = delta - m * S;
    return (r < 0 ? -r : r) < static_cast<__int128>(len);
  };
  if (S == 0 || n_stripes <= 1) return near(0);
  const __int128 hi = static_cast<__int128>(n_stripes) - 1, lo = -hi;
  __int128 q = delta / S;
  if (delta % S != 0 && delta < 0) --q;  // floor
  const __int128 m0 = q < lo ? lo : (q > hi ? hi : q), m1 = q + 1 < lo ? lo : (q + 1 > hi ? hi : q + 1);
  return near(m0) || near(m1);
}

}  // namespace

#if XRS_HAS_PART(1)
uint64_t zero_rows(int dev) {
  constexpr uint64_t kZeroRowBytes = 1u << 20;  // >= a whole vect of every padded launch
  static std::mutex mu;
  static uint64_t buf[64] = {};
  if (dev < 0 || dev >= 64) return 0;
  std::lock_guard<std::mutex> g(mu);
  if (!buf[dev]) {
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev && hipSetDevice(dev) != hipSuccess) return 0;
    void* p = nullptr;
    hipStream_t z = nullptr;
    bool ok = hipMalloc(&p, kZeroRowBytes) == hipSuccess;
    // zeroed on a private stream: no null-stream barrier against the user's work
    ok = ok && hipStreamCreateWithFlags(&z, hipStreamNonBlocking) == hipSuccess;
    ok = ok && hipMemsetAsync(p, 0, kZeroRowBytes, z) == hipSuccess && hipStreamSynchronize(z) == hipSuccess;
    if (z) (void)hipStreamDestroy(z);
    if (ok) buf[dev] = reinterpret_cast<uint64_t>(p);
    else if (p) (void)hipFree(p);
    if (prev >= 0 && prev != dev) (void)hipSetDevice(prev);
  }
  return buf[dev];
}

std::atomic<bool> g_trace{false};
std::mutex g_trace_mu;
std::vector<std::pair<std::string, uint64_t>> g_trace_log;

void trace_event(const char* name) {
  if (g_trace.load(std::memory_order_relaxed)) trace_note(name);
}

void trace_kernels(bool on) {
  std::lock_guard<std::mutex> g(g_trace_mu);
  if (on) g_trace_log.clear();
  g_trace.store(on, std::memory_order_relaxed);
}

size_t traced_kernels(char* buf, size_t cap) {
  std::string out;
  {
    std::lock_guard<std::mutex> g(g_trace_mu);
    for (const auto& e : g_trace_log) out += e.first + " " + std::to_string(e.second) + "\n";
  }
  if (buf && cap) {
    const size_t n = out.size() < cap - 1 ? out.size() : cap - 1;
    std::memcpy(buf, out.data(), n);
    buf[n] = 0;
  }
  return out.size();
}

int launch_pair(const PairPlan& p0, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (p0.P < 1 || p0.P > kMaxOut || p0.C < 0 || p0.C > kMaxSrc) return static_cast<int>(hipErrorInvalidValue);
  bool ind = false;
  for (int c = 0; c < p0.C; ++c) ind = ind || row_ind(p0.src[c]);
  for (int r = 0; r < p0.P; ++r) ind = ind || row_ind(p0.dst[r]);
  if (ind) {  // every row indirect; ragged end as a byte-granular second launch
    for (int c = 0; c < p0.C; ++c)
      if (!row_ind(p0.src[c])) return static_cast<int>(hipErrorInvalidValue);
    for (int r = 0; r < p0.P; ++r)
      if (!row_ind(p0.dst[r])) return static_cast<int>(hipErrorInvalidValue);
    PairPlan pp = p0;
    pp.overlap = false;
    return split_launch(pp, p0.half, false, [s](const PairPlan& p, bool vec) {
      if (p.acc) return vec ? launch_pair_ind_p<true, true>(p, s) : launch_pair_ind_p<true, false>(p, s);
      return vec ? launch_pair_ind_p<false, true>(p, s) : launch_pair_ind_p<false, false>(p, s);
    });
  }
  bool al = true;
  for (int c = 0; c < p0.C; ++c) al = al && row_aligned(p0.src[c]);
  for (int r = 0; r < p0.P; ++r) al = al && row_aligned(p0.dst[r]);
  PairPlan pp = p0;
  pp.overlap = false;
  bool pure = !p0.acc;  // no accumulate, and no destination that is also a source
  for (int r = 0; r < p0.P && pure; ++r)
    for (int c = 0; c < p0.C && pure; ++c) pure = !rows_overlap(p0.dst[r], p0.src[c], 2 * p0.half, p0.n_stripes);
  return split_launch(pp, p0.half, al, [s](const PairPlan& p, bool vec) {
    if (p.acc) return vec ? launch_pair_p<true, true>(p, s) : launch_pair_p<true, false>(p, s);
    return vec ? launch_pair_p<false, true>(p, s) : launch_pair_p<false, false>(p, s);
  }, pure);
}
#endif  // XRS_HAS_PART(1)

#if XRS_HAS_PART(2)
bool tile_counters(int dev) { return ctr_ring(dev) != nullptr; }

int launch_staged(const StagedPlan& p0, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  for (int m = 0; m < p0.na; ++m)  // indirect rows: the step plan (rows kernels) runs them
    if (row_ind(p0.asrc[m])) return kStagedDecline;
  if (p0.nd < 1 || p0.nd > p0.na || p0.nd > p0.nb || p0.na > kStSrc || p0.nb > kStB || p0.nl < 0 ||
      p0.nl > kStOut || p0.nn < 0 || p0.nn > kStOut)
    return static_cast<int>(hipErrorInvalidValue);
  bool al = true;
  for (int m = 0; m < p0.na; ++m) al = al && row_aligned(p0.asrc[m]);
  for (int m = 0; m < p0.nb; ++m) al = al && row_aligned(p0.bsrc[m]);
  for (int q = 0; q < p0.nl; ++q) al = al && row_aligned(p0.adst[q]);
  for (int u = 0; u < p0.nn; ++u) al = al && row_aligned(p0.bdst[u]);
  if (p0.nb > kStSrc) {  // wide b-side: one 16-byte wave-specialised launch or none
    const char* uv = std::getenv("XRS_UNALIGNED_VEC");  // as split_launch
    int nr = 0;
    bool ok = p0.half % 16 == 0 && (al || !(uv && uv[0] == '0'));
    for (int m = 0; m < p0.nb; ++m)
      if (p0.bret[m]) {
        ++nr;
        ok = ok && ((p0.bstore >> m) & 1u);
      }
    if (!ok || nr > kStOut) return kStagedDecline;
  }
  return split_launch(p0, p0.half, al, [s](const StagedPlan& p, bool vec) {
    return vec ? launch_staged_r<true>(p, s) : launch_staged_r<false>(p, s);
  });
}
#endif  // XRS_HAS_PART(2)

#if XRS_HAS_PART(3)
int launch_update_rows(const UpdRowsPlan& p0, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (p0.P < 1 || p0.P > kMaxOut || p0.nrows < 1 || p0.nrows > kMaxSrc || (!p0.rows && p0.nrows != 1))
    return static_cast<int>(hipErrorInvalidValue);
  bool ind = row_ind(p0.old_row) || row_ind(p0.new_row);
  for (int q = 0; q < p0.P; ++q) ind = ind || row_ind(p0.dst[q]);
  if (ind) {  // every row indirect (the queue's callers' buffers)
    bool all = row_ind(p0.old_row) && row_ind(p0.new_row);
    for (int q = 0; q < p0.P; ++q) all = all && row_ind(p0.dst[q]);
    if (!all) return static_cast<int>(hipErrorInvalidValue);
    return split_launch(p0, p0.half, false, [s](const UpdRowsPlan& p, bool vec) {
      return vec ? launch_update_rows_p<true, true>(p, s) : launch_update_rows_p<false, true>(p, s);
    });
  }
  bool al = row_aligned(p0.old_row) && row_aligned(p0.new_row);
  for (int q = 0; q < p0.P; ++q) al = al && row_aligned(p0.dst[q]);
  return split_launch(p0, p0.half, al, [s](const UpdRowsPlan& p, bool vec) {
    return vec ? launch_update_rows_p<true>(p, s) : launch_update_rows_p<false>(p, s);
  });
}

#endif  // XRS_HAS_PART(3)

#if XRS_HAS_PART(4)
int launch_rows(const RowsPlan& p0, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (p0.R < 1 || p0.R > kMaxOut || p0.NM < 0 || p0.NM > kMaxSrc || p0.NX < 0 || p0.NX > kMaxXor)
    return static_cast<int>(hipErrorInvalidValue);
  bool ind = false, all = true;
  auto note = [&](const RowRef& r) { (row_ind(r) ? ind : all) = row_ind(r); };
  for (int m = 0; m < p0.NM; ++m) note(p0.msrc[m]);
  for (int x = 0; x < p0.NX; ++x) note(p0.xsrc[x]);
  for (int r = 0; r < p0.R; ++r) note(p0.dst[r]);
  if (ind) {  // every row indirect (the queue's callers' buffers)
    if (!all) return static_cast<int>(hipErrorInvalidValue);
    RowsPlan rp = p0;
    rp.overlap = false;
    return split_launch(rp, p0.len, false, [s](const RowsPlan& p, bool vec) {
      if (p.acc) return vec ? launch_rows_ind_r<true, true>(p, s) : launch_rows_ind_r<true, false>(p, s);
      return vec ? launch_rows_ind_r<false, true>(p, s) : launch_rows_ind_r<false, false>(p, s);
    });
  }
  bool al = true;
  for (int m = 0; m < p0.NM; ++m) al = al && row_aligned(p0.msrc[m]);
  for (int x = 0; x < p0.NX; ++x) al = al && row_aligned(p0.xsrc[x]);
  for (int r = 0; r < p0.R; ++r) al = al && row_aligned(p0.dst[r]);
  RowsPlan rp = p0;
  rp.overlap = false;
  bool pure = !p0.acc;  // no accumulate, and no destination that is also a source
  for (int r = 0; r < p0.R && pure; ++r) {
    for (int m = 0; m < p0.NM && pure; ++m) pure = !rows_overlap(p0.dst[r], p0.msrc[m], p0.len, p0.n_stripes);
    for (int x = 0; x < p0.NX && pure; ++x) pure = !rows_overlap(p0.dst[r], p0.xsrc[x], p0.len, p0.n_stripes);
  }
  return split_launch(rp, p0.len, al, [s](const RowsPlan& p, bool vec) {
    if (p.acc) return vec ? launch_rows_r<true, true>(p, s) : launch_rows_r<true, false>(p, s);
    return vec ? launch_rows_r<false, true>(p, s) : launch_rows_r<false, false>(p, s);
  }, pure);
}

#endif  // XRS_HAS_PART(4)

}  // namespace xrs
