// rmw_probe.hip -- the ceiling of config 4's access pattern (Update @ 8 MiB,
// 64 stripes, xrs_batch_layout strides): six rows read per stripe (four
// parity rows, old, new; both halves), four written back in place.  XOR only,
// no GF work, the product's 16-B nontemporal lanes, 256-thread blocks and
// XCD block order K = 32, so the product kernel (update_rows_kernel<4, true>)
// can be compared with the bare pattern:
//   inplace  -- the Update pattern (12 loads, 8 stores in place per lane)
//   outplace -- the same, stores to a second buffer
//   split    -- in place, a- and b-halves in different lanes (6 loads, 4 stores)
//   readonly -- the 12 loads alone
// Prints one JSON line per kernel: median GB/s of 10 * 8 MiB * 64 bytes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 gu32x4;

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      std::exit(1);                                                         \
    }                                                                       \
  } while (0)

constexpr uint64_t kS = 8u << 20, kH = kS / 2, kShard = kS + 4096 + 256, kRows = 6, kStripe = kRows * kShard;
constexpr uint64_t kN = 64, kK = 32;

__device__ __forceinline__ uint64_t logical(uint32_t b, uint64_t nblk) {
  const uint32_t q = b >> 3, g = q / kK;
  const uint64_t span = 8ull * kK;
  if ((g + 1) * span > nblk) return b;
  return g * span + (b & 7u) * kK + (q - g * kK);
}
__device__ __forceinline__ u32x4 ldn(uint64_t a) { return __builtin_nontemporal_load(reinterpret_cast<const gu32x4*>(a)); }
__device__ __forceinline__ void stn(u32x4 v, uint64_t a) { __builtin_nontemporal_store(v, reinterpret_cast<gu32x4*>(a)); }

template <int MODE>  // 0 inplace, 1 outplace, 3 readonly
__global__ __launch_bounds__(256) void pair_rmw(uint64_t base, uint64_t out, uint64_t nblk) {
  const uint64_t chunks = kH / 16;
  const uint64_t gid = logical(blockIdx.x, nblk) * 256 + threadIdx.x;
  if (gid >= chunks * kN) return;
  const uint64_t s = gid / chunks, off = (gid - s * chunks) * 16;
  const uint64_t row0 = base + s * kStripe + off;
  const u32x4 oa = ldn(row0 + 4 * kShard), ob = ldn(row0 + 4 * kShard + kH);
  const u32x4 na = ldn(row0 + 5 * kShard), nb = ldn(row0 + 5 * kShard + kH);
  u32x4 pa[4], pb[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    pa[q] = ldn(row0 + q * kShard);
    pb[q] = ldn(row0 + q * kShard + kH);
  }
  const u32x4 da = oa ^ na, db = ob ^ nb;
  const uint64_t w0 = MODE == 1 ? out + s * kStripe + off : row0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    pa[q] ^= da;
    pb[q] ^= db;
    if (MODE == 3) {
      if (pa[q].x == 0x9e3779b9u && pb[q].y == 0x7f4a7c15u) stn(pa[q], w0 + q * kShard);
    } else {
      stn(pa[q], w0 + q * kShard);
      stn(pb[q], w0 + q * kShard + kH);
    }
  }
}

__global__ __launch_bounds__(256) void split_rmw(uint64_t base, uint64_t nblk) {
  const uint64_t chunks = kS / 16;  // both halves as one row of S bytes
  const uint64_t gid = logical(blockIdx.x, nblk) * 256 + threadIdx.x;
  if (gid >= chunks * kN) return;
  const uint64_t s = gid / chunks, off = (gid - s * chunks) * 16;
  const uint64_t row0 = base + s * kStripe + off;
  const u32x4 d = ldn(row0 + 4 * kShard) ^ ldn(row0 + 5 * kShard);
  u32x4 p[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) p[q] = ldn(row0 + q * kShard);
#pragma unroll
  for (int q = 0; q < 4; ++q) stn(p[q] ^ d, row0 + q * kShard);
}

int main() {
  const uint64_t bytes = kStripe * kN;
  uint8_t *a, *b;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMemset(a, 0x5a, bytes));
  CK(hipMemset(b, 0x00, bytes));
  const uint64_t nb_pair = (kH / 16 * kN + 255) / 256, nb_split = (kS / 16 * kN + 255) / 256;
  const uint64_t A = reinterpret_cast<uint64_t>(a), B = reinterpret_cast<uint64_t>(b);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* names[4] = {"inplace", "outplace", "split", "readonly"};
  auto launch = [&](int k) {
    switch (k) {
      case 0: pair_rmw<0><<<dim3(nb_pair), dim3(256)>>>(A, B, nb_pair); break;
      case 1: pair_rmw<1><<<dim3(nb_pair), dim3(256)>>>(A, B, nb_pair); break;
      case 2: split_rmw<<<dim3(nb_split), dim3(256)>>>(A, nb_split); break;
      default: pair_rmw<3><<<dim3(nb_pair), dim3(256)>>>(A, B, nb_pair); break;
    }
  };
  std::vector<std::vector<float>> t(4);
  for (int k = 0; k < 4; ++k)
    for (int w = 0; w < 3; ++w) launch(k);
  CK(hipDeviceSynchronize());
  for (int round = 0; round < 15; ++round)
    for (int k = 0; k < 4; ++k) {
      CK(hipEventRecord(e0));
      launch(k);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[k].push_back(ms);
    }
  const double moved = 10.0 * kS * kN;
  for (int k = 0; k < 4; ++k) {
    std::sort(t[k].begin(), t[k].end());
    const double ms = t[k][t[k].size() / 2];
    const double m = k == 3 ? 6.0 * kS * kN : moved;
    std::printf("{\"kernel\": \"%s\", \"ms\": %.4f, \"gbs\": %.1f, \"frac\": %.4f}\n", names[k], ms,
                m / ms / 1e6, m / ms / 1e6 / 8000.0);
  }
  CK(hipFree(a));
  CK(hipFree(b));
  return 0;
}
