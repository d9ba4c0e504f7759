// mapprobe.hip -- probe: does the block -> (stripe, offset) mapping change the
// HBM rate of the ReconstOne / Encode patterns on unpadded power-of-two
// layouts?  Not part of the product.
//
// The product kernels map consecutive blocks to consecutive 4 KiB pieces of a
// stripe.  With 1 MiB vects back to back (shard stride 2^20), ReconstOne runs
// at 4.9 TB/s against 5.6 TB/s with a 256 B pad per shard.
// Variants here only reorder which blocks run together:
//   seq   : the product order;
//   xcd   : block i runs on XCD i % 8; give each XCD a contiguous range;
//   rot   : within a stripe, rotate the chunk order by stripe * 37 blocks;
//   inter : stripe-interleaved (block i -> stripe i % n, chunk i / n).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I xrs_amd/csrc tools/mapprobe.hip xrs_amd/csrc/gf256.cpp -o tools/mapprobe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../xrs_amd/csrc/kernels.hip"
#include "gf256.h"

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));  \
      std::exit(2);                                                                            \
    }                                                                                          \
  } while (0)

namespace xrs {
namespace {

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

__constant__ uint64_t kChunk;

// Block index -> logical block (a bijection on [0, nblk)); bps = blocks per stripe.
template <int MAP>
__device__ __forceinline__ uint64_t remap(uint64_t b, uint64_t nblk, uint64_t bps) {
  if constexpr (MAP == 1) {  // xcd: contiguous range per XCD
    const uint64_t per = nblk / 8;
    if (b < per * 8) return (b % 8) * per + b / 8;
    return b;
  } else if constexpr (MAP == 2) {  // rot
    const uint64_t s = b / bps, c = b - s * bps;
    return s * bps + (c + s * 37) % bps;
  } else if constexpr (MAP == 3) {  // inter
    const uint64_t ns = nblk / bps;
    return (b % ns) * bps + b / ns;
  } else if constexpr (MAP == 4) {  // xcd chunks: groups of 8*K blocks, K consecutive per XCD
    const uint64_t K = kChunk, q = b / 8, g = q / K;
    if ((g + 1) * 8 * K <= nblk) return g * 8 * K + (b % 8) * K + q % K;
    return b;  // tail past the last whole group: identity
  } else if constexpr (MAP == 5) {  // xcd then rot
    return remap<2>(remap<1>(b, nblk, bps), nblk, bps);
  }
  return b;
}

template <int MAP>
__global__ __launch_bounds__(256) void r1_map(const RowsArgs<2, 12, 4, true> a, uint64_t nblk, uint64_t bps) {
  constexpr int R = 2, NM = 12, NX = 4, W = 4;
  const uint64_t lb = remap<MAP>(blockIdx.x, nblk, bps);
  const uint64_t gid = lb * 256 + threadIdx.x;
  const uint64_t stripe = gid / a.chunks;
  const uint64_t off = (gid - stripe * a.chunks) * 16;
  uint32_t acc[R][W] = {};
  uint32_t xm[NM][W], xx[NX][W];
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int m = 0; m < NM; ++m) ld<true>(xm[m], row_addr(a.msrc[m], stripe, off), 16);
#pragma unroll
  for (int x = 0; x < NX; ++x) ld<true>(xx[x], row_addr(a.xsrc[x], stripe, off), 16);
  __builtin_amdgcn_s_setprio(0);
#pragma unroll
  for (int m = 0; m + 1 < NM; m += 2) rows_mac2<R, W>(acc, a.tab[m], a.tab[m + 1], xm[m], xm[m + 1]);
#pragma unroll
  for (int x = 0; x < NX; ++x) rows_xor<R, W>(acc, a.xmask[x], xx[x]);
#pragma unroll
  for (int r = 0; r < R; ++r) st<true>(acc[r], row_addr(a.dst[r], stripe, off), 16);
}

template <int MAP>
__global__ __launch_bounds__(256) void enc_map(const PairArgs<4, 12, true> a, uint64_t nblk, uint64_t bps) {
  constexpr int P = 4, C = 12, W = 4;
  const uint64_t lb = remap<MAP>(blockIdx.x, nblk, bps);
  const uint64_t gid = lb * 256 + threadIdx.x;
  const uint64_t stripe = gid / a.chunks;
  const uint64_t off = (gid - stripe * a.chunks) * 16;
  uint32_t acc_a[P][W] = {}, acc_b[P][W] = {};
  uint32_t xa[C][W], xb[C][W];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const uint64_t s = row_addr(a.src[c], stripe, off);
    ld<true>(xa[c], s, 16);
    ld<true>(xb[c], s + a.half, 16);
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
    st<true>(acc_a[r], d, 16);
    st<true>(acc_b[r], d + a.half, 16);
  }
}

struct Timer {
  hipEvent_t a, b;
  Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
  template <class F>
  double ms(F f, int reps = 5) {
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

void report(const char* name, double ms, double bytes) {
  std::printf("%-48s %8.3f ms  %8.1f GB/s  (%.1f%%)\n", name, ms, bytes / ms / 1e6, bytes / ms / 1e6 / 80.0);
  std::fflush(stdout);
}

}  // namespace
}  // namespace xrs

using namespace xrs;

static const char* kMapName[6] = {"seq", "xcd", "rot", "inter", "xcdK", "xcd+rot"};

// Interleaved rounds over: seq, xcd, xcdK for K in kKs, and (whole blocks
// per stripe only) rot and xcd+rot; median of 5.
static const uint64_t kKs[] = {16, 32, 64, 128, 256, 1024};
template <class L>
static void run_variants(Timer& tm, const char* op, uint64_t S, uint64_t pad, double bytes, L launch, bool rot) {
  struct V { int map; uint64_t K; std::vector<double> t; };
  std::vector<V> vs = {{0, 0, {}}, {1, 0, {}}};
  for (uint64_t K : kKs) vs.push_back({4, K, {}});
  (void)rot;
  for (int r = 0; r < 9; ++r)
    for (V& v : vs) {
      CK(hipMemcpyToSymbol(HIP_SYMBOL(kChunk), &v.K, sizeof(v.K)));
      v.t.push_back(tm.ms([&] { launch(v.map, v.K); }));
    }
  for (V& v : vs) {
    std::sort(v.t.begin(), v.t.end());
    char name[128];
    std::snprintf(name, sizeof name, "%s S=%llu pad=%llu %s K=%llu", op, (unsigned long long)S,
                  (unsigned long long)pad, kMapName[v.map], (unsigned long long)v.K);
    report(name, v.t[4], bytes);
  }
}

static void r1_case(Timer& tm, uint64_t S, uint64_t n, uint64_t pad) {
  const GF& gf = GF::get();
  const uint64_t H = S / 2, shard = S + pad, stripe = 16 * shard;
  uint8_t* buf;
  CK(hipMalloc(&buf, n * stripe));
  hipLaunchKernelGGL(fill_kernel, dim3(8192), dim3(256), 0, 0, (uint32_t*)buf, n * stripe / 4, 5u);
  const uint64_t base = reinterpret_cast<uint64_t>(buf);
  RowsArgs<2, 12, 4, true> a;
  std::memset(&a, 0, sizeof(a));
  for (int m = 0; m < 12; ++m) {
    a.msrc[m] = {base + (m == 0 ? 12 : m) * shard + H, stripe};
    for (int r = 0; r < 2; ++r) a.tab[m][r] = gf.tab(static_cast<uint8_t>(17 * m + 5 * r + 3));
  }
  a.xsrc[0] = {base + 13 * shard + H, stripe};
  for (int x = 1; x < 4; ++x) a.xsrc[x] = {base + 3 * x * shard, stripe};
  for (int x = 0; x < 4; ++x) a.xmask[x] = 2;
  a.dst[0] = {base + H, stripe};
  a.dst[1] = {base, stripe};
  a.nm = 12; a.nx = 4; a.len = H; a.chunks = H / 16; a.total = a.chunks * n;
  const uint64_t nblk = a.total / 256, bps = std::max<uint64_t>(1, a.chunks / 256);
  void (*ks[6])(const RowsArgs<2, 12, 4, true>, uint64_t, uint64_t) = {r1_map<0>, r1_map<1>, r1_map<2>,
                                                                        r1_map<3>, r1_map<4>, r1_map<5>};
  hipLaunchKernelGGL(ks[0], dim3(nblk), dim3(256), 0, 0, a, nblk, bps);
  const unsigned long long ref = checksum(buf, n * stripe);
  run_variants(tm, "r1 ", S, pad, 9.0 * S * n, [&](int v, uint64_t K) {
    hipLaunchKernelGGL(ks[v], dim3(nblk), dim3(256), 0, 0, a, nblk, bps);
  }, a.chunks >= 256);
  if (checksum(buf, n * stripe) != ref) std::printf("   !! output differs\n");
  CK(hipFree(buf));
}

static void enc_case(Timer& tm, uint64_t S, uint64_t n, uint64_t pad) {
  const GF& gf = GF::get();
  const uint64_t H = S / 2, shard = S + pad, stripe = 16 * shard;
  uint8_t* buf;
  CK(hipMalloc(&buf, n * stripe));
  hipLaunchKernelGGL(fill_kernel, dim3(8192), dim3(256), 0, 0, (uint32_t*)buf, n * stripe / 4, 9u);
  const uint64_t base = reinterpret_cast<uint64_t>(buf);
  PairArgs<4, 12, true> a;
  std::memset(&a, 0, sizeof(a));
  for (int c = 0; c < 12; ++c) {
    a.src[c] = {base + c * shard, stripe};
    for (int r = 0; r < 4; ++r) a.tab[c][r] = gf.tab(gf.inv(static_cast<uint8_t>((12 + r) ^ c)));
  }
  for (int r = 0; r < 4; ++r) a.dst[r] = {base + (12 + r) * shard, stripe};
  a.n_src = 12; a.half = H; a.chunks = H / 16; a.total = a.chunks * n;
  const uint64_t nblk = a.total / 256, bps = std::max<uint64_t>(1, a.chunks / 256);
  void (*ks[6])(const PairArgs<4, 12, true>, uint64_t, uint64_t) = {enc_map<0>, enc_map<1>, enc_map<2>,
                                                                     enc_map<3>, enc_map<4>, enc_map<5>};
  hipLaunchKernelGGL(ks[0], dim3(nblk), dim3(256), 0, 0, a, nblk, bps);
  const unsigned long long ref = checksum(buf, n * stripe);
  run_variants(tm, "enc", S, pad, 16.0 * S * n, [&](int v, uint64_t K) {
    hipLaunchKernelGGL(ks[v], dim3(nblk), dim3(256), 0, 0, a, nblk, bps);
  }, a.chunks >= 256);
  if (checksum(buf, n * stripe) != ref) std::printf("   !! output differs\n");
  CK(hipFree(buf));
}

int main() {
  Timer tm;
  enc_case(tm, 4096, 65536, 0);
  r1_case(tm, 4096, 65536, 0);
  enc_case(tm, 1 << 20, 512, 0);
  r1_case(tm, 1 << 20, 512, 0);
  r1_case(tm, 1 << 20, 512, 256);
  r1_case(tm, 65536, 4096, 0);
  enc_case(tm, 65536, 4096, 0);
  r1_case(tm, 8 << 20, 64, 0);
  enc_case(tm, 8 << 20, 64, 0);
  enc_case(tm, 16384, 16384, 0);
  r1_case(tm, 16384, 16384, 0);
  return 0;
}
