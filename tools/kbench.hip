// kbench.hip -- kernel microbenchmarks for A/B experiments on the GPU box.
// Not part of the product.  Includes the product kernels (same TU) so the
// variants below reuse gmul/sel_of/x3 and can be checked against them.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I xrs_amd/csrc tools/kbench.hip -o tools/kbench
//   tools/kbench [which]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../xrs_amd/csrc/kernels.hip"
#include "gf256.h"

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                   \
    }                                                                                 \
  } while (0)

namespace xrs {
namespace {

// ---------------------------------------------------------------- utilities
__global__ void fill_kernel(uint32_t* p, uint64_t n, uint32_t seed) {
  uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  for (; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = x;
  }
}

__global__ void checksum_kernel(const uint32_t* p, uint64_t n, unsigned long long* out) {
  uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  unsigned long long s = 0;
  for (; i < n; i += (uint64_t)gridDim.x * blockDim.x) s += (unsigned long long)p[i] * (1 + (i & 1023));
  atomicAdd(out, s);
}

unsigned long long checksum(const void* p, uint64_t bytes) {
  unsigned long long* d;
  CK(hipMalloc(&d, 8));
  CK(hipMemset(d, 0, 8));
  hipLaunchKernelGGL(checksum_kernel, dim3(4096), dim3(256), 0, 0, (const uint32_t*)p, bytes / 4, d);
  unsigned long long h;
  CK(hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost));
  CK(hipFree(d));
  return h;
}

__global__ void copy_kernel(const u32x4* __restrict__ a, u32x4* __restrict__ b, uint64_t n) {
  uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  for (; i < n; i += (uint64_t)gridDim.x * blockDim.x) b[i] = a[i];
}

__global__ void read_kernel(const u32x4* __restrict__ a, uint64_t n, uint32_t* sink) {
  uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t s = 0;
  for (; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    u32x4 v = a[i];
    s ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (s == 0x12345678u) sink[0] = s;
}

// ------------------------------------------------- ReconstOne-shaped variants
// 2 outputs, 12 GF sources, 4 XOR sources (target output 1).  U chunks per
// thread (u-major: each wave instruction stays 1 KiB contiguous), optional
// nontemporal loads/stores.
template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void r1_var(const RowsArgs<2, 12, 4, true> a) {
  constexpr int R = 2, NM = 12, NX = 4;
  const uint64_t lane_chunk = static_cast<uint64_t>(blockIdx.x) * (256 * U) + threadIdx.x;
  const uint64_t chunks = a.chunks;  // per stripe
  const uint64_t stripe = lane_chunk / chunks;
  if (stripe >= a.total / chunks) return;
  const uint64_t c0 = lane_chunk - stripe * chunks;
  uint32_t xm[U][NM][4], xx[U][NX][4];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint64_t off = (c0 + u * 256) * 16;
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      const u32x4* p = reinterpret_cast<const u32x4*>(row_addr(a.msrc[m], stripe, off));
      u32x4 t = NTL ? __builtin_nontemporal_load(p) : *p;
      xm[u][m][0] = t.x; xm[u][m][1] = t.y; xm[u][m][2] = t.z; xm[u][m][3] = t.w;
    }
#pragma unroll
    for (int x = 0; x < NX; ++x) {
      const u32x4* p = reinterpret_cast<const u32x4*>(row_addr(a.xsrc[x], stripe, off));
      u32x4 t = NTL ? __builtin_nontemporal_load(p) : *p;
      xx[u][x][0] = t.x; xx[u][x][1] = t.y; xx[u][x][2] = t.z; xx[u][x][3] = t.w;
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    uint32_t acc[R][4] = {};
#pragma unroll
    for (int m = 0; m + 1 < NM; m += 2) rows_mac2<R, 4>(acc, a.tab[m], a.tab[m + 1], xm[u][m], xm[u][m + 1]);
#pragma unroll
    for (int x = 0; x < NX; ++x) rows_xor<R, 4>(acc, a.xmask[x], xx[u][x]);
    const uint64_t off = (c0 + u * 256) * 16;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      u32x4* p = reinterpret_cast<u32x4*>(row_addr(a.dst[r], stripe, off));
      u32x4 t;
      t.x = acc[r][0]; t.y = acc[r][1]; t.z = acc[r][2]; t.w = acc[r][3];
      if (NTS) __builtin_nontemporal_store(t, p); else *p = t;
    }
  }
}

// TIMING-ONLY probe (wrong results): row m is read at a per-row rotated chunk
// of the block's 4 KiB tile (rotation SK chunks per row), so consecutive load
// instructions of a wave hit addresses that differ in bits 8-11.
template <int SK>
__global__ __launch_bounds__(256) void r1_skew(const RowsArgs<2, 12, 4, true> a) {
  const uint64_t gid = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (gid >= a.total) return;
  const uint64_t stripe = gid / a.chunks;
  const uint64_t c = gid - stripe * a.chunks;
  const uint64_t tile = c & ~255ull, t = c & 255;
  u32x4 s0 = {0, 0, 0, 0}, s1 = {0, 0, 0, 0};
#pragma unroll
  for (int m = 0; m < 12; ++m) {
    const uint64_t off = (tile + ((t + SK * m) & 255)) * 16;
    s0 ^= __builtin_nontemporal_load(reinterpret_cast<const gu32x4*>(row_addr(a.msrc[m], stripe, off)));
  }
#pragma unroll
  for (int x = 0; x < 4; ++x) {
    const uint64_t off = (tile + ((t + SK * (12 + x)) & 255)) * 16;
    s1 ^= __builtin_nontemporal_load(reinterpret_cast<const gu32x4*>(row_addr(a.xsrc[x], stripe, off)));
  }
  __builtin_nontemporal_store(s0, reinterpret_cast<gu32x4*>(row_addr(a.dst[0], stripe, c * 16)));
  __builtin_nontemporal_store(s1 ^ s0, reinterpret_cast<gu32x4*>(row_addr(a.dst[1], stripe, c * 16)));
}

// Encode variant with w-outer loops (table dwords for a column pair held in
// VGPRs, selectors computed per dword) and optional dwordx2 lanes (VB = 8).
template <int VB>
__global__ __launch_bounds__(256) void enc_wouter(const PairArgs<4, 12, true> a) {
  constexpr int P = 4, C = 12, W = VB / 4;
  const uint64_t gid = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
  const uint64_t chunks = a.half / VB;
  if (gid >= chunks * (a.total / a.chunks)) return;
  const uint64_t stripe = gid / chunks;
  const uint64_t off = (gid - stripe * chunks) * VB;
  uint32_t xa[C][W], xb[C][W];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const uint64_t s = row_addr(a.src[c], stripe, off);
    if constexpr (VB == 16) {
      u32x4 ta = __builtin_nontemporal_load(reinterpret_cast<const gu32x4*>(s));
      u32x4 tb = __builtin_nontemporal_load(reinterpret_cast<const gu32x4*>(s + a.half));
      xa[c][0] = ta.x; xa[c][1] = ta.y; xa[c][2] = ta.z; xa[c][3] = ta.w;
      xb[c][0] = tb.x; xb[c][1] = tb.y; xb[c][2] = tb.z; xb[c][3] = tb.w;
    } else {
      typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
      typedef __attribute__((address_space(1))) u32x2 gu32x2;
      u32x2 ta = __builtin_nontemporal_load(reinterpret_cast<const gu32x2*>(s));
      u32x2 tb = __builtin_nontemporal_load(reinterpret_cast<const gu32x2*>(s + a.half));
      xa[c][0] = ta.x; xa[c][1] = ta.y;
      xb[c][0] = tb.x; xb[c][1] = tb.y;
    }
  }
  uint32_t acc_a[P][W] = {}, acc_b[P][W] = {};
#pragma unroll
  for (int c = 0; c < C; c += 2) {
#pragma unroll
    for (int w = 0; w < W; ++w) {
      const Sel sa0 = sel_of(xa[c][w]), sb0 = sel_of(xb[c][w]);
      const Sel sa1 = sel_of(xa[c + 1][w]), sb1 = sel_of(xb[c + 1][w]);
#pragma unroll
      for (int r = 0; r < P; ++r) {
        acc_a[r][w] = x3(acc_a[r][w], gmul(a.tab[c][r], sa0), gmul(a.tab[c + 1][r], sa1));
        acc_b[r][w] = x3(acc_b[r][w], gmul(a.tab[c][r], sb0), gmul(a.tab[c + 1][r], sb1));
      }
    }
#pragma unroll
    for (int w = 0; w < W; ++w) {
      acc_b[1 + c % 3][w] ^= xa[c][w];
      acc_b[1 + (c + 1) % 3][w] ^= xa[c + 1][w];
    }
  }
#pragma unroll
  for (int r = 0; r < P; ++r) {
    const uint64_t d = row_addr(a.dst[r], stripe, off);
    if constexpr (VB == 16) {
      u32x4 ta, tb;
      ta.x = acc_a[r][0]; ta.y = acc_a[r][1]; ta.z = acc_a[r][2]; ta.w = acc_a[r][3];
      tb.x = acc_b[r][0]; tb.y = acc_b[r][1]; tb.z = acc_b[r][2]; tb.w = acc_b[r][3];
      __builtin_nontemporal_store(ta, reinterpret_cast<gu32x4*>(d));
      __builtin_nontemporal_store(tb, reinterpret_cast<gu32x4*>(d + a.half));
    } else {
      typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
      typedef __attribute__((address_space(1))) u32x2 gu32x2;
      u32x2 ta, tb;
      ta.x = acc_a[r][0]; ta.y = acc_a[r][1];
      tb.x = acc_b[r][0]; tb.y = acc_b[r][1];
      __builtin_nontemporal_store(ta, reinterpret_cast<gu32x2*>(d));
      __builtin_nontemporal_store(tb, reinterpret_cast<gu32x2*>(d + a.half));
    }
  }
}

// Read-ceiling probes: U independent 16-B nt loads per lane (one-shot grid),
// and an LDS-DMA (global_load_lds_dwordx4) stream into a per-wave LDS ring.
template <int U, bool NT>
__global__ __launch_bounds__(256) void read_u(const u32x4* __restrict__ a, uint64_t n, uint32_t* sink) {
  const uint64_t base = (static_cast<uint64_t>(blockIdx.x) * 256 * U) + threadIdx.x;
  u32x4 s = {0, 0, 0, 0};
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint64_t i = base + u * 256;
    if (i < n) {
      const gu32x4* p = (const gu32x4*)(a + i);
      s ^= NT ? __builtin_nontemporal_load(p) : *p;
    }
  }
  if ((s.x ^ s.y ^ s.z ^ s.w) == 0x12345678u) sink[0] = 1;
}

template <int U>
__global__ __launch_bounds__(256) void read_glds(const u32x4* __restrict__ a, uint64_t n, uint32_t* sink) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[4 * U * 1024];
  const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  const uint64_t base = (static_cast<uint64_t>(blockIdx.x) * 256 * U) + wave * 64 + lane;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint64_t i = base + u * 256;
    if (i < n)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(a + i),
                                       (__attribute__((address_space(3))) void*)(lds + (wave * U + u) * 1024),
                                       16, 0, 0);
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (lds[threadIdx.x * 16] == 0x5a && lds[threadIdx.x * 16 + 1] == 0x5a && sink[0] == 7) sink[1] = 1;
}

// ReconstOne / Encode address patterns split into their read and write parts.
template <bool READ, bool WRITE>
__global__ __launch_bounds__(256) void r1_rw(const RowsArgs<2, 12, 4, true> a, uint32_t* sink) {
  const uint64_t gid = logical_block(a.order) * 256 + threadIdx.x;
  if (gid >= a.total) return;
  const uint64_t stripe = gid / a.chunks;
  const uint64_t off = (gid - stripe * a.chunks) * 16;
  u32x4 s0 = {0, 0, 0, 0}, s1 = {1, 2, 3, 4};
  if (READ) {
#pragma unroll
    for (int m = 0; m < 12; ++m)
      s0 ^= __builtin_nontemporal_load(reinterpret_cast<const gu32x4*>(row_addr(a.msrc[m], stripe, off)));
#pragma unroll
    for (int x = 0; x < 4; ++x)
      s1 ^= __builtin_nontemporal_load(reinterpret_cast<const gu32x4*>(row_addr(a.xsrc[x], stripe, off)));
  }
  if (WRITE) {
    __builtin_nontemporal_store(s0, reinterpret_cast<gu32x4*>(row_addr(a.dst[0], stripe, off)));
    __builtin_nontemporal_store(s1 ^ s0, reinterpret_cast<gu32x4*>(row_addr(a.dst[1], stripe, off)));
  } else if ((s0.x ^ s1.y) == 0x12345678u) {
    sink[0] = 1;
  }
}

template <bool READ, bool WRITE>
__global__ __launch_bounds__(256) void enc_rw(const PairArgs<4, 12, true> a, uint32_t* sink) {
  const uint64_t gid = logical_block(a.order) * 256 + threadIdx.x;
  if (gid >= a.total) return;
  const uint64_t stripe = gid / a.chunks;
  const uint64_t off = (gid - stripe * a.chunks) * 16;
  u32x4 sa = {0, 0, 0, 0}, sb = {1, 2, 3, 4};
  if (READ) {
#pragma unroll
    for (int c = 0; c < 12; ++c) {
      const uint64_t s = row_addr(a.src[c], stripe, off);
      sa ^= __builtin_nontemporal_load(reinterpret_cast<const gu32x4*>(s));
      sb ^= __builtin_nontemporal_load(reinterpret_cast<const gu32x4*>(s + a.half));
    }
  }
  if (WRITE) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint64_t d = row_addr(a.dst[r], stripe, off);
      __builtin_nontemporal_store(sa + r, reinterpret_cast<gu32x4*>(d));
      __builtin_nontemporal_store(sb + r, reinterpret_cast<gu32x4*>(d + a.half));
    }
  } else if ((sa.x ^ sb.y) == 0x12345678u) {
    sink[0] = 1;
  }
}

// s_setprio probes: the product Encode / ReconstOne bodies with the wave's
// priority raised while it issues its loads (PR), dropped for the compute.
template <int PR>
__global__ __launch_bounds__(256) void enc_prio(const PairArgs<4, 12, true> a) {
  constexpr int P = 4, C = 12, W = 4;
  const uint64_t gid = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (gid >= a.total) return;
  const uint64_t stripe = gid / a.chunks;
  const uint64_t off = (gid - stripe * a.chunks) * 16;
  uint32_t acc_a[P][W] = {}, acc_b[P][W] = {};
  uint32_t xa[C][W], xb[C][W];
  if (PR) __builtin_amdgcn_s_setprio(PR);
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const uint64_t s = row_addr(a.src[c], stripe, off);
    ld<true>(xa[c], s, 16);
    ld<true>(xb[c], s + a.half, 16);
  }
  if (PR) __builtin_amdgcn_s_setprio(0);
#pragma unroll
  for (int c = 0; c + 1 < C; c += 2)
    pair_mac2<P, W>(acc_a, acc_b, a.tab[c], a.tab[c + 1], xa[c], xb[c], xa[c + 1], xb[c + 1]);
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int w = 0; w < W; ++w) acc_b[1 + c % (P - 1)][w] ^= xa[c][w];
#pragma unroll
  for (int r = 0; r < P; ++r) {
    const uint64_t d = row_addr(a.dst[r], stripe, off);
    st<true>(acc_a[r], d, 16);
    st<true>(acc_b[r], d + a.half, 16);
  }
}

template <int PR>
__global__ __launch_bounds__(256) void r1_prio(const RowsArgs<2, 12, 4, true> a) {
  constexpr int R = 2, NM = 12, NX = 4, W = 4;
  const uint64_t gid = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (gid >= a.total) return;
  const uint64_t stripe = gid / a.chunks;
  const uint64_t off = (gid - stripe * a.chunks) * 16;
  uint32_t acc[R][W] = {};
  uint32_t xm[NM][W], xx[NX][W];
  if (PR) __builtin_amdgcn_s_setprio(PR);
#pragma unroll
  for (int m = 0; m < NM; ++m) ld<true>(xm[m], row_addr(a.msrc[m], stripe, off), 16);
#pragma unroll
  for (int x = 0; x < NX; ++x) ld<true>(xx[x], row_addr(a.xsrc[x], stripe, off), 16);
  if (PR) __builtin_amdgcn_s_setprio(0);
#pragma unroll
  for (int m = 0; m + 1 < NM; m += 2) rows_mac2<R, W>(acc, a.tab[m], a.tab[m + 1], xm[m], xm[m + 1]);
#pragma unroll
  for (int x = 0; x < NX; ++x) rows_xor<R, W>(acc, a.xmask[x], xx[x]);
#pragma unroll
  for (int r = 0; r < R; ++r) st<true>(acc[r], row_addr(a.dst[r], stripe, off), 16);
}

// Grid-stride XOR-only probes (memory ceiling with a persistent-style grid).
__global__ __launch_bounds__(256) void r1_xor_gs(const RowsArgs<2, 12, 4, true> a) {
  for (uint64_t gid = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x; gid < a.total;
       gid += static_cast<uint64_t>(gridDim.x) * 256) {
    const uint64_t stripe = gid / a.chunks;
    const uint64_t off = (gid - stripe * a.chunks) * 16;
    u32x4 s0 = {0, 0, 0, 0}, s1 = {0, 0, 0, 0};
#pragma unroll
    for (int m = 0; m < 12; ++m)
      s0 ^= __builtin_nontemporal_load(reinterpret_cast<const gu32x4*>(row_addr(a.msrc[m], stripe, off)));
#pragma unroll
    for (int x = 0; x < 4; ++x)
      s1 ^= __builtin_nontemporal_load(reinterpret_cast<const gu32x4*>(row_addr(a.xsrc[x], stripe, off)));
    __builtin_nontemporal_store(s0, reinterpret_cast<gu32x4*>(row_addr(a.dst[0], stripe, off)));
    __builtin_nontemporal_store(s1 ^ s0, reinterpret_cast<gu32x4*>(row_addr(a.dst[1], stripe, off)));
  }
}

__global__ __launch_bounds__(256) void r1_xor_nt(const RowsArgs<2, 12, 4, true> a) {
  const uint64_t gid = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (gid >= a.total) return;
  const uint64_t stripe = gid / a.chunks;
  const uint64_t off = (gid - stripe * a.chunks) * 16;
  u32x4 s0 = {0, 0, 0, 0}, s1 = {0, 0, 0, 0};
#pragma unroll
  for (int m = 0; m < 12; ++m)
    s0 ^= __builtin_nontemporal_load(reinterpret_cast<const gu32x4*>(row_addr(a.msrc[m], stripe, off)));
#pragma unroll
  for (int x = 0; x < 4; ++x)
    s1 ^= __builtin_nontemporal_load(reinterpret_cast<const gu32x4*>(row_addr(a.xsrc[x], stripe, off)));
  __builtin_nontemporal_store(s0, reinterpret_cast<gu32x4*>(row_addr(a.dst[0], stripe, off)));
  __builtin_nontemporal_store(s1 ^ s0, reinterpret_cast<gu32x4*>(row_addr(a.dst[1], stripe, off)));
}

__global__ __launch_bounds__(256) void enc_xor_gs(const PairArgs<4, 12, true> a) {
  for (uint64_t gid = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x; gid < a.total;
       gid += static_cast<uint64_t>(gridDim.x) * 256) {
    const uint64_t stripe = gid / a.chunks;
    const uint64_t off = (gid - stripe * a.chunks) * 16;
    u32x4 sa = {0, 0, 0, 0}, sb = {0, 0, 0, 0};
#pragma unroll
    for (int c = 0; c < 12; ++c) {
      const uint64_t s = row_addr(a.src[c], stripe, off);
      sa ^= __builtin_nontemporal_load(reinterpret_cast<const gu32x4*>(s));
      sb ^= __builtin_nontemporal_load(reinterpret_cast<const gu32x4*>(s + a.half));
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint64_t d = row_addr(a.dst[r], stripe, off);
      __builtin_nontemporal_store(sa + r, reinterpret_cast<gu32x4*>(d));
      __builtin_nontemporal_store(sb + r, reinterpret_cast<gu32x4*>(d + a.half));
    }
  }
}

__global__ __launch_bounds__(256) void enc_xor_nt(const PairArgs<4, 12, true> a) {
  const uint64_t gid = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (gid >= a.total) return;
  const uint64_t stripe = gid / a.chunks;
  const uint64_t off = (gid - stripe * a.chunks) * 16;
  u32x4 sa = {0, 0, 0, 0}, sb = {0, 0, 0, 0};
#pragma unroll
  for (int c = 0; c < 12; ++c) {
    const uint64_t s = row_addr(a.src[c], stripe, off);
    sa ^= __builtin_nontemporal_load(reinterpret_cast<const gu32x4*>(s));
    sb ^= __builtin_nontemporal_load(reinterpret_cast<const gu32x4*>(s + a.half));
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const uint64_t d = row_addr(a.dst[r], stripe, off);
    __builtin_nontemporal_store(sa + r, reinterpret_cast<gu32x4*>(d));
    __builtin_nontemporal_store(sb + r, reinterpret_cast<gu32x4*>(d + a.half));
  }
}

// Same addresses, XOR only (memory ceiling of the ReconstOne pattern).
__global__ __launch_bounds__(256) void r1_xoronly(const RowsArgs<2, 12, 4, true> a) {
  const uint64_t gid = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (gid >= a.total) return;
  const uint64_t stripe = gid / a.chunks;
  const uint64_t off = (gid - stripe * a.chunks) * 16;
  u32x4 s0 = {0, 0, 0, 0}, s1 = {0, 0, 0, 0};
#pragma unroll
  for (int m = 0; m < 12; ++m) s0 ^= *reinterpret_cast<const u32x4*>(row_addr(a.msrc[m], stripe, off));
#pragma unroll
  for (int x = 0; x < 4; ++x) s1 ^= *reinterpret_cast<const u32x4*>(row_addr(a.xsrc[x], stripe, off));
  *reinterpret_cast<u32x4*>(row_addr(a.dst[0], stripe, off)) = s0;
  *reinterpret_cast<u32x4*>(row_addr(a.dst[1], stripe, off)) = s1 ^ s0;
}

// --------------------------------------------------- Encode-shaped variants
template <int WAVES, bool NTS, bool NTL = false>
__global__ __launch_bounds__(256, WAVES) void enc_var(const PairArgs<4, 12, true> a) {
  constexpr int P = 4, C = 12, W = 4;
  const uint64_t gid = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (gid >= a.total) return;
  const uint64_t stripe = gid / a.chunks;
  const uint64_t off = (gid - stripe * a.chunks) * 16;
  uint32_t acc_a[P][W] = {}, acc_b[P][W] = {};
  uint32_t xa[C][W], xb[C][W];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const uint64_t s = row_addr(a.src[c], stripe, off);
    if (NTL) {
      u32x4 ta = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(s));
      u32x4 tb = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(s + a.half));
      xa[c][0] = ta.x; xa[c][1] = ta.y; xa[c][2] = ta.z; xa[c][3] = ta.w;
      xb[c][0] = tb.x; xb[c][1] = tb.y; xb[c][2] = tb.z; xb[c][3] = tb.w;
    } else {
      ld<true>(xa[c], s, 16);
      ld<true>(xb[c], s + a.half, 16);
    }
  }
#pragma unroll
  for (int c = 0; c + 1 < C; c += 2)
    pair_mac2<P, W>(acc_a, acc_b, a.tab[c], a.tab[c + 1], xa[c], xb[c], xa[c + 1], xb[c + 1]);
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int w = 0; w < W; ++w) acc_b[1 + c % (P - 1)][w] ^= xa[c][w];
#pragma unroll
  for (int r = 0; r < P; ++r) {
    const uint64_t d = row_addr(a.dst[r], stripe, off);
    u32x4 ta, tb;
    ta.x = acc_a[r][0]; ta.y = acc_a[r][1]; ta.z = acc_a[r][2]; ta.w = acc_a[r][3];
    tb.x = acc_b[r][0]; tb.y = acc_b[r][1]; tb.z = acc_b[r][2]; tb.w = acc_b[r][3];
    if (NTS) {
      __builtin_nontemporal_store(ta, reinterpret_cast<u32x4*>(d));
      __builtin_nontemporal_store(tb, reinterpret_cast<u32x4*>(d + a.half));
    } else {
      *reinterpret_cast<u32x4*>(d) = ta;
      *reinterpret_cast<u32x4*>(d + a.half) = tb;
    }
  }
}

__global__ __launch_bounds__(256) void enc_xoronly(const PairArgs<4, 12, true> a) {
  const uint64_t gid = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (gid >= a.total) return;
  const uint64_t stripe = gid / a.chunks;
  const uint64_t off = (gid - stripe * a.chunks) * 16;
  u32x4 sa = {0, 0, 0, 0}, sb = {0, 0, 0, 0};
#pragma unroll
  for (int c = 0; c < 12; ++c) {
    const uint64_t s = row_addr(a.src[c], stripe, off);
    sa ^= *reinterpret_cast<const u32x4*>(s);
    sb ^= *reinterpret_cast<const u32x4*>(s + a.half);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const uint64_t d = row_addr(a.dst[r], stripe, off);
    *reinterpret_cast<u32x4*>(d) = sa + r;
    *reinterpret_cast<u32x4*>(d + a.half) = sb + r;
  }
}

}  // namespace
}  // namespace xrs

using namespace xrs;

struct Timer {
  hipEvent_t a, b;
  Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
  template <class F>
  double ms(F f, int reps = 10) {
    f();
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float t;
    CK(hipEventElapsedTime(&t, a, b));
    return t / reps;
  }
};

static void report(const char* name, double ms, double bytes) {
  std::printf("%-44s %9.3f ms  %8.1f GB/s  (%.1f%% of 8 TB/s)\n", name, ms, bytes / ms / 1e6,
              bytes / ms / 1e6 / 80.0);
  std::fflush(stdout);
}

// Product kernels (through the real launchers) on a [n][16][S + pad] batch.
static void sweep_one(Timer& tm, uint64_t S, uint64_t n, uint64_t pad) {
  const GF& gf = GF::get();
  const uint64_t shard = S + pad, stripe = 16 * shard, H = S / 2;
  uint8_t* buf;
  CK(hipMalloc(&buf, n * stripe));
  hipLaunchKernelGGL(fill_kernel, dim3(8192), dim3(256), 0, 0, (uint32_t*)buf, n * stripe / 4, 5u);
  const uint64_t base = reinterpret_cast<uint64_t>(buf);
  PairPlan pp;
  std::memset(&pp, 0, sizeof(pp));
  pp.P = 4; pp.C = 12; pp.encode12 = true; pp.half = H; pp.n_stripes = n;
  for (int c = 0; c < 12; ++c) {
    pp.src[c] = {base + c * shard, stripe};
    pp.pb[c] = 1 + c % 3;
    for (int r = 0; r < 4; ++r) pp.tab[c][r] = gf.tab(gf.inv(static_cast<uint8_t>((12 + r) ^ c)));
  }
  for (int r = 0; r < 4; ++r) pp.dst[r] = {base + (12 + r) * shard, stripe};
  char name[128];
  double t = tm.ms([&] { CK((hipError_t)launch_pair(pp, nullptr)); });
  std::snprintf(name, sizeof name, "encode S=%llu n=%llu pad=%llu", (unsigned long long)S,
                (unsigned long long)n, (unsigned long long)pad);
  report(name, t, 16.0 * S * n);
  RowsPlan rp;
  std::memset(&rp, 0, sizeof(rp));
  rp.R = 2; rp.NM = 12; rp.NX = 4; rp.len = H; rp.n_stripes = n;
  const int k = 0;
  for (int m = 0; m < 12; ++m) {
    rp.msrc[m] = {base + (m == k ? 12 : m) * shard + H, stripe};
    for (int r = 0; r < 2; ++r) rp.tab[m][r] = gf.tab(static_cast<uint8_t>(17 * m + 5 * r + 3));
  }
  rp.xsrc[0] = {base + 13 * shard + H, stripe};
  for (int x = 1; x < 4; ++x) rp.xsrc[x] = {base + 3 * x * shard, stripe};
  for (int x = 0; x < 4; ++x) rp.xmask[x] = 2;
  rp.dst[0] = {base + k * shard + H, stripe};
  rp.dst[1] = {base + k * shard, stripe};
  t = tm.ms([&] { CK((hipError_t)launch_rows(rp, nullptr)); });
  std::snprintf(name, sizeof name, "reconst1 S=%llu n=%llu pad=%llu", (unsigned long long)S,
                (unsigned long long)n, (unsigned long long)pad);
  report(name, t, 9.0 * S * n);
  CK(hipFree(buf));
}

// Interleaved A/B over shard paddings: all buffers allocated up front, R
// rounds alternating between them, median per variant (rule: one process,
// interleaved rounds).
static void pad_ab(Timer& tm, uint64_t S, std::vector<uint64_t> pads, int rounds) {
  const GF& gf = GF::get();
  const uint64_t n = (4ull << 30) / (16 * S), H = S / 2;
  struct V { uint64_t pad; uint8_t* buf; PairPlan pp; RowsPlan rp; std::vector<double> te, tr; };
  std::vector<V> vs(pads.size());
  for (size_t i = 0; i < pads.size(); ++i) {
    V& v = vs[i];
    v.pad = pads[i];
    const uint64_t shard = S + v.pad, stripe = 16 * shard;
    CK(hipMalloc(&v.buf, n * stripe));
    hipLaunchKernelGGL(fill_kernel, dim3(8192), dim3(256), 0, 0, (uint32_t*)v.buf, n * stripe / 4, 5u);
    const uint64_t base = reinterpret_cast<uint64_t>(v.buf);
    std::memset(&v.pp, 0, sizeof(v.pp));
    v.pp.P = 4; v.pp.C = 12; v.pp.encode12 = true; v.pp.half = H; v.pp.n_stripes = n;
    for (int c = 0; c < 12; ++c) {
      v.pp.src[c] = {base + c * shard, stripe};
      v.pp.pb[c] = 1 + c % 3;
      for (int r = 0; r < 4; ++r) v.pp.tab[c][r] = gf.tab(gf.inv(static_cast<uint8_t>((12 + r) ^ c)));
    }
    for (int r = 0; r < 4; ++r) v.pp.dst[r] = {base + (12 + r) * shard, stripe};
    std::memset(&v.rp, 0, sizeof(v.rp));
    v.rp.R = 2; v.rp.NM = 12; v.rp.NX = 4; v.rp.len = H; v.rp.n_stripes = n;
    for (int m = 0; m < 12; ++m) {
      v.rp.msrc[m] = {base + (m == 0 ? 12 : m) * shard + H, stripe};
      for (int r = 0; r < 2; ++r) v.rp.tab[m][r] = gf.tab(static_cast<uint8_t>(17 * m + 5 * r + 3));
    }
    v.rp.xsrc[0] = {base + 13 * shard + H, stripe};
    for (int x = 1; x < 4; ++x) v.rp.xsrc[x] = {base + 3 * x * shard, stripe};
    for (int x = 0; x < 4; ++x) v.rp.xmask[x] = 2;
    v.rp.dst[0] = {base + H, stripe};
    v.rp.dst[1] = {base, stripe};
  }
  for (int r = 0; r < rounds; ++r)
    for (V& v : vs) {
      v.te.push_back(tm.ms([&] { CK((hipError_t)launch_pair(v.pp, nullptr)); }, 5));
      v.tr.push_back(tm.ms([&] { CK((hipError_t)launch_rows(v.rp, nullptr)); }, 5));
    }
  for (V& v : vs) {
    std::sort(v.te.begin(), v.te.end());
    std::sort(v.tr.begin(), v.tr.end());
    char name[128];
    std::snprintf(name, sizeof name, "encode   S=%-8llu pad=%-5llu median", (unsigned long long)S,
                  (unsigned long long)v.pad);
    report(name, v.te[rounds / 2], 16.0 * S * n);
    std::snprintf(name, sizeof name, "reconst1 S=%-8llu pad=%-5llu median", (unsigned long long)S,
                  (unsigned long long)v.pad);
    report(name, v.tr[rounds / 2], 9.0 * S * n);
    CK(hipFree(v.buf));
  }
}

int main(int argc, char** argv) {
  const std::string which = argc > 1 ? argv[1] : "all";
  const GF& gf = GF::get();
  Timer tm;
  if (which == "gs") {
    // ReconstOne 1 MiB (pad 256) and Encode 4 KiB (pad 0), 4 GiB batches.
    const uint64_t S1 = 1 << 20, n1 = 256, H1 = S1 / 2, sh1 = S1 + 256, st1 = 16 * sh1;
    const uint64_t S2 = 4096, n2 = 65536, H2 = S2 / 2, st2 = 16 * S2;
    uint8_t *b1, *b2;
    CK(hipMalloc(&b1, n1 * st1));
    CK(hipMalloc(&b2, n2 * st2));
    hipLaunchKernelGGL(fill_kernel, dim3(8192), dim3(256), 0, 0, (uint32_t*)b1, n1 * st1 / 4, 5u);
    hipLaunchKernelGGL(fill_kernel, dim3(8192), dim3(256), 0, 0, (uint32_t*)b2, n2 * st2 / 4, 6u);
    const uint64_t base1 = reinterpret_cast<uint64_t>(b1), base2 = reinterpret_cast<uint64_t>(b2);
    RowsArgs<2, 12, 4, true> ra;
    std::memset(&ra, 0, sizeof(ra));
    for (int m = 0; m < 12; ++m) {
      ra.msrc[m] = {base1 + (m == 0 ? 12 : m) * sh1 + H1, st1};
      for (int r = 0; r < 2; ++r) ra.tab[m][r] = gf.tab(static_cast<uint8_t>(17 * m + 5 * r + 3));
    }
    ra.xsrc[0] = {base1 + 13 * sh1 + H1, st1};
    for (int x = 1; x < 4; ++x) ra.xsrc[x] = {base1 + 3 * x * sh1, st1};
    for (int x = 0; x < 4; ++x) ra.xmask[x] = 2;
    ra.dst[0] = {base1 + H1, st1};
    ra.dst[1] = {base1, st1};
    ra.nm = 12; ra.nx = 4; ra.len = H1; ra.chunks = H1 / 16; ra.total = ra.chunks * n1;
    PairArgs<4, 12, true> pa;
    std::memset(&pa, 0, sizeof(pa));
    for (int c = 0; c < 12; ++c) {
      pa.src[c] = {base2 + c * S2, st2};
      for (int r = 0; r < 4; ++r) pa.tab[c][r] = gf.tab(gf.inv(static_cast<uint8_t>((12 + r) ^ c)));
    }
    for (int r = 0; r < 4; ++r) pa.dst[r] = {base2 + (12 + r) * S2, st2};
    pa.n_src = 12; pa.half = H2; pa.chunks = H2 / 16; pa.total = pa.chunks * n2;
    const unsigned bl1 = (unsigned)(ra.total / 256), bl2 = (unsigned)(pa.total / 256);
    const unsigned grids[] = {1024, 2048, 4096, 8192, 16384};
    std::vector<double> tr[8], te[8];
    for (int round = 0; round < 7; ++round) {
      tr[0].push_back(tm.ms([&] { hipLaunchKernelGGL((rows_kernel<2, 12, 4, false, true>), dim3(bl1), dim3(256), 0, 0, ra); }, 5));
      tr[1].push_back(tm.ms([&] { hipLaunchKernelGGL(r1_xor_nt, dim3(bl1), dim3(256), 0, 0, ra); }, 5));
      te[0].push_back(tm.ms([&] { hipLaunchKernelGGL((pair_kernel<4, 12, false, true>), dim3(bl2), dim3(256), 0, 0, pa); }, 5));
      te[1].push_back(tm.ms([&] { hipLaunchKernelGGL(enc_xor_nt, dim3(bl2), dim3(256), 0, 0, pa); }, 5));
      for (int g = 0; g < 5; ++g) {
        tr[2 + g].push_back(tm.ms([&] { hipLaunchKernelGGL(r1_xor_gs, dim3(grids[g]), dim3(256), 0, 0, ra); }, 5));
        te[2 + g].push_back(tm.ms([&] { hipLaunchKernelGGL(enc_xor_gs, dim3(grids[g]), dim3(256), 0, 0, pa); }, 5));
      }
    }
    for (int i = 0; i < 7; ++i) {
      std::sort(tr[i].begin(), tr[i].end());
      std::sort(te[i].begin(), te[i].end());
      char name[128];
      if (i < 2) std::snprintf(name, sizeof name, "r1 1MiB pad256 %s", i ? "xor-only nt" : "product");
      else std::snprintf(name, sizeof name, "r1 1MiB pad256 xor grid-stride g=%u", grids[i - 2]);
      report(name, tr[i][3], 9.0 * S1 * n1);
      if (i < 2) std::snprintf(name, sizeof name, "enc 4KiB %s", i ? "xor-only nt" : "product");
      else std::snprintf(name, sizeof name, "enc 4KiB xor grid-stride g=%u", grids[i - 2]);
      report(name, te[i][3], 16.0 * S2 * n2);
    }
    return 0;
  }
  if (which == "encvar") {
    const uint64_t S2 = 4096, n2 = 65536, H2 = S2 / 2, st2 = 16 * S2;
    uint8_t* b2;
    CK(hipMalloc(&b2, n2 * st2));
    hipLaunchKernelGGL(fill_kernel, dim3(8192), dim3(256), 0, 0, (uint32_t*)b2, n2 * st2 / 4, 6u);
    const uint64_t base2 = reinterpret_cast<uint64_t>(b2);
    PairArgs<4, 12, true> pa;
    std::memset(&pa, 0, sizeof(pa));
    for (int c = 0; c < 12; ++c) {
      pa.src[c] = {base2 + c * S2, st2};
      for (int r = 0; r < 4; ++r) pa.tab[c][r] = gf.tab(gf.inv(static_cast<uint8_t>((12 + r) ^ c)));
    }
    for (int r = 0; r < 4; ++r) pa.dst[r] = {base2 + (12 + r) * S2, st2};
    pa.n_src = 12; pa.half = H2; pa.chunks = H2 / 16; pa.total = pa.chunks * n2;
    const unsigned bl = (unsigned)(pa.total / 256);
    hipLaunchKernelGGL((pair_kernel<4, 12, false, true>), dim3(bl), dim3(256), 0, 0, pa);
    const unsigned long long ref = checksum(b2, n2 * st2);
    std::vector<double> t[4];
    const char* nm[4] = {"product", "xor-only nt", "w-outer x4", "w-outer x2"};
    for (int round = 0; round < 7; ++round) {
      t[0].push_back(tm.ms([&] { hipLaunchKernelGGL((pair_kernel<4, 12, false, true>), dim3(bl), dim3(256), 0, 0, pa); }, 5));
      t[1].push_back(tm.ms([&] { hipLaunchKernelGGL(enc_xor_nt, dim3(bl), dim3(256), 0, 0, pa); }, 5));
      hipLaunchKernelGGL((pair_kernel<4, 12, false, true>), dim3(bl), dim3(256), 0, 0, pa);
      t[2].push_back(tm.ms([&] { hipLaunchKernelGGL((enc_wouter<16>), dim3(bl), dim3(256), 0, 0, pa); }, 5));
      if (round == 0 && checksum(b2, n2 * st2) != ref) std::printf("   !! w-outer x4 differs\n");
      t[3].push_back(tm.ms([&] { hipLaunchKernelGGL((enc_wouter<8>), dim3(2 * bl), dim3(256), 0, 0, pa); }, 5));
      if (round == 0 && checksum(b2, n2 * st2) != ref) std::printf("   !! w-outer x2 differs\n");
    }
    for (int i = 0; i < 4; ++i) {
      std::sort(t[i].begin(), t[i].end());
      char name[96];
      std::snprintf(name, sizeof name, "enc 4KiB %s", nm[i]);
      report(name, t[i][3], 16.0 * S2 * n2);
    }
    return 0;
  }
  if (which == "skew") {
    const uint64_t S = 1 << 20, n = 256, H = S / 2;
    for (uint64_t pad : {0ull, 256ull}) {
      const uint64_t shard = S + pad, stripe = 16 * shard;
      uint8_t* buf;
      CK(hipMalloc(&buf, n * stripe));
      hipLaunchKernelGGL(fill_kernel, dim3(8192), dim3(256), 0, 0, (uint32_t*)buf, n * stripe / 4, 5u);
      const uint64_t base = reinterpret_cast<uint64_t>(buf);
      RowsArgs<2, 12, 4, true> a;
      std::memset(&a, 0, sizeof(a));
      for (int m = 0; m < 12; ++m) a.msrc[m] = {base + (m == 0 ? 12 : m) * shard + H, stripe};
      a.xsrc[0] = {base + 13 * shard + H, stripe};
      for (int x = 1; x < 4; ++x) a.xsrc[x] = {base + 3 * x * shard, stripe};
      a.dst[0] = {base + H, stripe};
      a.dst[1] = {base, stripe};
      a.nm = 12; a.nx = 4; a.len = H; a.chunks = H / 16; a.total = a.chunks * n;
      const unsigned blocks = (unsigned)(a.total / 256);
      std::vector<double> t[5];
      for (int r = 0; r < 7; ++r) {
        t[0].push_back(tm.ms([&] { hipLaunchKernelGGL((rows_kernel<2, 12, 4, false, true>), dim3(blocks), dim3(256), 0, 0, a); }, 5));
        t[1].push_back(tm.ms([&] { hipLaunchKernelGGL((r1_skew<0>), dim3(blocks), dim3(256), 0, 0, a); }, 5));
        t[2].push_back(tm.ms([&] { hipLaunchKernelGGL((r1_skew<4>), dim3(blocks), dim3(256), 0, 0, a); }, 5));
        t[3].push_back(tm.ms([&] { hipLaunchKernelGGL((r1_skew<16>), dim3(blocks), dim3(256), 0, 0, a); }, 5));
        t[4].push_back(tm.ms([&] { hipLaunchKernelGGL((r1_skew<64>), dim3(blocks), dim3(256), 0, 0, a); }, 5));
      }
      const char* nm[5] = {"product", "skew0 (xor only)", "skew4 (64 B/row)", "skew16 (256 B/row)", "skew64 (1 KiB/row)"};
      for (int i = 0; i < 5; ++i) {
        std::sort(t[i].begin(), t[i].end());
        char name[128];
        std::snprintf(name, sizeof name, "r1 1MiB pad=%llu %s", (unsigned long long)pad, nm[i]);
        report(name, t[i][3], 9.0 * S * n);
      }
      CK(hipFree(buf));
    }
    return 0;
  }
  if (which == "padab") {
    for (uint64_t S : {4096ull, 65536ull, 1ull << 20, 8ull << 20})
      pad_ab(tm, S, {0, 128, 256, 512, 4096 + 256}, 7);
    return 0;
  }
  if (which == "rw") {
    // same setup as "gs": ReconstOne 1 MiB pad 256, Encode 4 KiB pad 0;
    // "rw xcd": ReconstOne 1 MiB unpadded, both in the product's XCD block order
    const bool xcd = argc > 2 && std::string(argv[2]) == "xcd";
    const uint64_t S1 = 1 << 20, n1 = 256, H1 = S1 / 2, sh1 = S1 + (xcd ? 0 : 256), st1 = 16 * sh1;
    const uint64_t S2 = 4096, n2 = 65536, H2 = S2 / 2, st2 = 16 * S2;
    uint8_t *b1, *b2;
    uint32_t* sink;
    CK(hipMalloc(&b1, n1 * st1));
    CK(hipMalloc(&b2, n2 * st2));
    CK(hipMalloc(&sink, 64));
    hipLaunchKernelGGL(fill_kernel, dim3(8192), dim3(256), 0, 0, (uint32_t*)b1, n1 * st1 / 4, 5u);
    hipLaunchKernelGGL(fill_kernel, dim3(8192), dim3(256), 0, 0, (uint32_t*)b2, n2 * st2 / 4, 6u);
    const uint64_t base1 = reinterpret_cast<uint64_t>(b1), base2 = reinterpret_cast<uint64_t>(b2);
    RowsArgs<2, 12, 4, true> ra;
    std::memset(&ra, 0, sizeof(ra));
    for (int m = 0; m < 12; ++m) {
      ra.msrc[m] = {base1 + (m == 0 ? 12 : m) * sh1 + H1, st1};
      for (int r = 0; r < 2; ++r) ra.tab[m][r] = gf.tab(static_cast<uint8_t>(17 * m + 5 * r + 3));
    }
    ra.xsrc[0] = {base1 + 13 * sh1 + H1, st1};
    for (int x = 1; x < 4; ++x) ra.xsrc[x] = {base1 + 3 * x * sh1, st1};
    for (int x = 0; x < 4; ++x) ra.xmask[x] = 2;
    ra.dst[0] = {base1 + H1, st1};
    ra.dst[1] = {base1, st1};
    ra.nm = 12; ra.nx = 4; ra.len = H1; ra.chunks = H1 / 16; ra.total = ra.chunks * n1;
    PairArgs<4, 12, true> pa;
    std::memset(&pa, 0, sizeof(pa));
    for (int c = 0; c < 12; ++c) {
      pa.src[c] = {base2 + c * S2, st2};
      for (int r = 0; r < 4; ++r) pa.tab[c][r] = gf.tab(gf.inv(static_cast<uint8_t>((12 + r) ^ c)));
    }
    for (int r = 0; r < 4; ++r) pa.dst[r] = {base2 + (12 + r) * S2, st2};
    pa.n_src = 12; pa.half = H2; pa.chunks = H2 / 16; pa.total = pa.chunks * n2;
    const unsigned bl1 = (unsigned)(ra.total / 256), bl2 = (unsigned)(pa.total / 256);
    if (xcd) {
      ra.order = {bl1, 128};
      pa.order = {bl2, 32};
    }
    std::vector<double> t[8];
    for (int round = 0; round < 5; ++round) {
      t[0].push_back(tm.ms([&] { hipLaunchKernelGGL((rows_kernel<2, 12, 4, false, true>), dim3(bl1), dim3(256), 0, 0, ra); }, 5));
      t[1].push_back(tm.ms([&] { hipLaunchKernelGGL((r1_rw<true, true>), dim3(bl1), dim3(256), 0, 0, ra, sink); }, 5));
      t[2].push_back(tm.ms([&] { hipLaunchKernelGGL((r1_rw<true, false>), dim3(bl1), dim3(256), 0, 0, ra, sink); }, 5));
      t[3].push_back(tm.ms([&] { hipLaunchKernelGGL((r1_rw<false, true>), dim3(bl1), dim3(256), 0, 0, ra, sink); }, 5));
      t[4].push_back(tm.ms([&] { hipLaunchKernelGGL((pair_kernel<4, 12, false, true>), dim3(bl2), dim3(256), 0, 0, pa); }, 5));
      t[5].push_back(tm.ms([&] { hipLaunchKernelGGL((enc_rw<true, true>), dim3(bl2), dim3(256), 0, 0, pa, sink); }, 5));
      t[6].push_back(tm.ms([&] { hipLaunchKernelGGL((enc_rw<true, false>), dim3(bl2), dim3(256), 0, 0, pa, sink); }, 5));
      t[7].push_back(tm.ms([&] { hipLaunchKernelGGL((enc_rw<false, true>), dim3(bl2), dim3(256), 0, 0, pa, sink); }, 5));
    }
    if (argc > 2 && std::string(argv[2]) == "prio") {
      std::vector<double> tq[2][4];
      for (int round = 0; round < 7; ++round) {
        tq[0][0].push_back(tm.ms([&] { hipLaunchKernelGGL((rows_kernel<2, 12, 4, false, true>), dim3(bl1), dim3(256), 0, 0, ra); }, 5));
        tq[0][1].push_back(tm.ms([&] { hipLaunchKernelGGL((r1_prio<0>), dim3(bl1), dim3(256), 0, 0, ra); }, 5));
        tq[0][2].push_back(tm.ms([&] { hipLaunchKernelGGL((r1_prio<1>), dim3(bl1), dim3(256), 0, 0, ra); }, 5));
        tq[0][3].push_back(tm.ms([&] { hipLaunchKernelGGL((r1_prio<3>), dim3(bl1), dim3(256), 0, 0, ra); }, 5));
        tq[1][0].push_back(tm.ms([&] { hipLaunchKernelGGL((pair_kernel<4, 12, false, true>), dim3(bl2), dim3(256), 0, 0, pa); }, 5));
        tq[1][1].push_back(tm.ms([&] { hipLaunchKernelGGL((enc_prio<0>), dim3(bl2), dim3(256), 0, 0, pa); }, 5));
        tq[1][2].push_back(tm.ms([&] { hipLaunchKernelGGL((enc_prio<1>), dim3(bl2), dim3(256), 0, 0, pa); }, 5));
        tq[1][3].push_back(tm.ms([&] { hipLaunchKernelGGL((enc_prio<3>), dim3(bl2), dim3(256), 0, 0, pa); }, 5));
      }
      const char* qn[4] = {"product", "copy, no setprio", "setprio 1 around loads", "setprio 3 around loads"};
      for (int k = 0; k < 2; ++k)
        for (int i = 0; i < 4; ++i) {
          std::sort(tq[k][i].begin(), tq[k][i].end());
          char name[96];
          std::snprintf(name, sizeof name, "%s %s", k ? "enc" : "r1 ", qn[i]);
          report(name, tq[k][i][3], k ? 16.0 * S2 * n2 : 9.0 * S1 * n1);
        }
      return 0;
    }
    const char* nm[8] = {"r1 product", "r1 read+write (xor)", "r1 read only (16 rows)", "r1 write only (2 rows)",
                         "enc product", "enc read+write (xor)", "enc read only (24 halves)", "enc write only (8 halves)"};
    const double by[8] = {9.0 * S1 * n1, 9.0 * S1 * n1, 8.0 * S1 * n1, 1.0 * S1 * n1,
                          16.0 * S2 * n2, 16.0 * S2 * n2, 12.0 * S2 * n2, 4.0 * S2 * n2};
    for (int i = 0; i < 8; ++i) {
      std::sort(t[i].begin(), t[i].end());
      report(nm[i], t[i][2], by[i]);
    }
    return 0;
  }
  if (which == "readceil") {
    const uint64_t bytes = 8ull << 30, n = bytes / 16;
    uint8_t* a;
    uint32_t* sink;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(sink, 0, 64));
    hipLaunchKernelGGL(fill_kernel, dim3(8192), dim3(256), 0, 0, (uint32_t*)a, bytes / 4, 1u);
    const u32x4* p = (const u32x4*)a;
    std::vector<double> t[9];
    const char* nm[9] = {"read U=1 plain", "read U=1 nt", "read U=4 nt", "read U=8 nt", "read U=4 plain",
                         "glds U=1", "glds U=4", "glds U=8", "copy float4 g=65536"};
    uint8_t* b;
    CK(hipMalloc(&b, bytes));
    for (int r = 0; r < 5; ++r) {
      t[0].push_back(tm.ms([&] { hipLaunchKernelGGL((read_u<1, false>), dim3(n / 256), dim3(256), 0, 0, p, n, sink); }, 5));
      t[1].push_back(tm.ms([&] { hipLaunchKernelGGL((read_u<1, true>), dim3(n / 256), dim3(256), 0, 0, p, n, sink); }, 5));
      t[2].push_back(tm.ms([&] { hipLaunchKernelGGL((read_u<4, true>), dim3(n / 1024), dim3(256), 0, 0, p, n, sink); }, 5));
      t[3].push_back(tm.ms([&] { hipLaunchKernelGGL((read_u<8, true>), dim3(n / 2048), dim3(256), 0, 0, p, n, sink); }, 5));
      t[4].push_back(tm.ms([&] { hipLaunchKernelGGL((read_u<4, false>), dim3(n / 1024), dim3(256), 0, 0, p, n, sink); }, 5));
      t[5].push_back(tm.ms([&] { hipLaunchKernelGGL((read_glds<1>), dim3(n / 256), dim3(256), 0, 0, p, n, sink); }, 5));
      t[6].push_back(tm.ms([&] { hipLaunchKernelGGL((read_glds<4>), dim3(n / 1024), dim3(256), 0, 0, p, n, sink); }, 5));
      t[7].push_back(tm.ms([&] { hipLaunchKernelGGL((read_glds<8>), dim3(n / 2048), dim3(256), 0, 0, p, n, sink); }, 5));
      t[8].push_back(tm.ms([&] { hipLaunchKernelGGL(copy_kernel, dim3(65536), dim3(256), 0, 0, p, (u32x4*)b, n); }, 5));
    }
    for (int i = 0; i < 9; ++i) {
      std::sort(t[i].begin(), t[i].end());
      report(nm[i], t[i][2], i == 8 ? 2.0 * bytes : 1.0 * bytes);
    }
    return 0;
  }
  if (which == "padfine") {  // 1 MiB vects, finer pad sweep
    pad_ab(tm, 1ull << 20, {192, 256, 320, 384, 640, 768}, 7);
    pad_ab(tm, 1ull << 20, {256, 1280, 1536, 2304, 3328, 6400}, 7);
    pad_ab(tm, 4096, {0, 64, 128, 192, 320}, 7);
    return 0;
  }
  if (which == "sweep") {
    for (uint64_t S : {4096ull, 65536ull, 1ull << 20, 8ull << 20})
      for (uint64_t pad : {0ull, 256ull}) sweep_one(tm, S, (8ull << 30) / (16 * S), pad);
    return 0;
  }
  // ---------------- ReconstOne pattern: 512 stripes x 16 x 1 MiB
  std::vector<unsigned long long> pads;
  for (int i = 2; i < argc; ++i) pads.push_back(std::strtoull(argv[i], nullptr, 0));
  if (pads.empty()) pads = {0ull, 4096ull, 256ull};
  if (which == "all" || which == "r1") {
    for (uint64_t pad : pads) {
      const uint64_t S = 1 << 20, shard = S + pad, stripe = 16 * shard, n = 512;
      uint8_t* buf;
      CK(hipMalloc(&buf, n * stripe));
      hipLaunchKernelGGL(fill_kernel, dim3(8192), dim3(256), 0, 0, (uint32_t*)buf, n * stripe / 4, 7u);
      CK(hipDeviceSynchronize());
      const uint64_t base = reinterpret_cast<uint64_t>(buf), H = S / 2;
      const int k = 0;
      RowsArgs<2, 12, 4, true> a;
      std::memset(&a, 0, sizeof(a));
      for (int m = 0; m < 12; ++m) {
        a.msrc[m] = {base + (m == k ? 12 : m) * shard + H, stripe};
        for (int r = 0; r < 2; ++r) a.tab[m][r] = gf.tab(static_cast<uint8_t>(17 * m + 5 * r + 3));
      }
      a.xsrc[0] = {base + 13 * shard + H, stripe};
      a.xsrc[1] = {base + 3 * shard, stripe};
      a.xsrc[2] = {base + 6 * shard, stripe};
      a.xsrc[3] = {base + 9 * shard, stripe};
      for (int x = 0; x < 4; ++x) a.xmask[x] = 2;
      a.dst[0] = {base + k * shard + H, stripe};
      a.dst[1] = {base + k * shard, stripe};
      a.nm = 12; a.nx = 4; a.len = H; a.chunks = H / 16; a.total = a.chunks * n;
      const double bytes = 9.0 * S * n;
      const unsigned blocks = (unsigned)(a.total / 256);
      char name[128];
      std::snprintf(name, sizeof name, "r1 product rows_kernel pad=%llu", (unsigned long long)pad);
      double t = tm.ms([&] { hipLaunchKernelGGL((rows_kernel<2, 12, 4, false, true>), dim3(blocks), dim3(256), 0, 0, a); });
      report(name, t, bytes);
      const unsigned long long ref = checksum(buf, n * stripe);
      auto chk = [&](const char* nm) {
        if (checksum(buf, n * stripe) != ref) std::printf("   !! %s output differs\n", nm);
      };
      std::snprintf(name, sizeof name, "r1 xor-only pad=%llu", (unsigned long long)pad);
      t = tm.ms([&] { hipLaunchKernelGGL(r1_xoronly, dim3(blocks), dim3(256), 0, 0, a); });
      report(name, t, bytes);
      // restore outputs
      hipLaunchKernelGGL((rows_kernel<2, 12, 4, false, true>), dim3(blocks), dim3(256), 0, 0, a);
#define R1V(U, NTL, NTS)                                                                        \
  t = tm.ms([&] { hipLaunchKernelGGL((r1_var<U, NTL, NTS>), dim3(blocks / U), dim3(256), 0, 0, a); }); \
  std::snprintf(name, sizeof name, "r1 var U=%d ntl=%d nts=%d pad=%llu", U, NTL, NTS, (unsigned long long)pad); \
  report(name, t, bytes);                                                                       \
  chk(name);
      R1V(1, true, true)
      R1V(2, true, true)
      CK(hipFree(buf));
    }
  }
  // ---------------- Encode pattern: 65536 stripes x 16 x 4 KiB
  if (which == "all" || which == "enc") for (uint64_t pad : pads) {
    const uint64_t S = 4096, n = 65536, shard = S + pad, stripe = 16 * shard;
    uint8_t* buf;
    CK(hipMalloc(&buf, n * stripe));
    hipLaunchKernelGGL(fill_kernel, dim3(8192), dim3(256), 0, 0, (uint32_t*)buf, n * stripe / 4, 9u);
    const uint64_t base = reinterpret_cast<uint64_t>(buf), H = S / 2;
    PairArgs<4, 12, true> a;
    std::memset(&a, 0, sizeof(a));
    for (int c = 0; c < 12; ++c) {
      a.src[c] = {base + c * shard, stripe};
      for (int r = 0; r < 4; ++r) a.tab[c][r] = gf.tab(gf.inv(static_cast<uint8_t>((12 + r) ^ c)));
    }
    for (int r = 0; r < 4; ++r) a.dst[r] = {base + (12 + r) * shard, stripe};
    std::printf("-- enc pad=%llu\n", (unsigned long long)pad);
    a.n_src = 12; a.half = H; a.chunks = H / 16; a.total = a.chunks * n;
    const unsigned blocks = (unsigned)(a.total / 256);
    const double bytes = 16.0 * S * n;
    double t = tm.ms([&] { hipLaunchKernelGGL((pair_kernel<4, 12, false, true>), dim3(blocks), dim3(256), 0, 0, a); });
    report("enc product pair_kernel", t, bytes);
    const unsigned long long ref = checksum(buf, n * stripe);
    t = tm.ms([&] { hipLaunchKernelGGL(enc_xoronly, dim3(blocks), dim3(256), 0, 0, a); });
    report("enc xor-only", t, bytes);
    char name[128];
#define ENCV(WV, NTS)                                                                             \
  t = tm.ms([&] { hipLaunchKernelGGL((enc_var<WV, NTS>), dim3(blocks), dim3(256), 0, 0, a); });    \
  std::snprintf(name, sizeof name, "enc var waves=%d nts=%d", WV, NTS);                           \
  report(name, t, bytes);                                                                         \
  if (checksum(buf, n * stripe) != ref) std::printf("   !! %s output differs\n", name);
    ENCV(2, false)
    ENCV(2, true)
    t = tm.ms([&] { hipLaunchKernelGGL((enc_var<2, true, true>), dim3(blocks), dim3(256), 0, 0, a); });
    report("enc var waves=2 nts=1 ntl=1", t, bytes);
    if (checksum(buf, n * stripe) != ref) std::printf("   !! ntl output differs\n");
    CK(hipFree(buf));
  }
  // ---------------- plain streaming ceilings (8 GiB)
  if (which == "all" || which == "copy") {
    const uint64_t bytes = 8ull << 30;
    uint8_t *a, *b;
    uint32_t* sink;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc(&sink, 4));
    hipLaunchKernelGGL(fill_kernel, dim3(8192), dim3(256), 0, 0, (uint32_t*)a, bytes / 4, 1u);
    const uint64_t n = bytes / 16;
    for (unsigned g : {2048u, 8192u, 65536u}) {
      double t = tm.ms([&] { hipLaunchKernelGGL(copy_kernel, dim3(g), dim3(256), 0, 0, (const u32x4*)a, (u32x4*)b, n); });
      char name[96];
      std::snprintf(name, sizeof name, "copy float4 8 GiB grid=%u", g);
      report(name, t, 2.0 * bytes);
      t = tm.ms([&] { hipLaunchKernelGGL(read_kernel, dim3(g), dim3(256), 0, 0, (const u32x4*)a, n, sink); });
      std::snprintf(name, sizeof name, "read-only 8 GiB grid=%u", g);
      report(name, t, 1.0 * bytes);
    }
    CK(hipFree(a));
    CK(hipFree(b));
  }
  return 0;
}
