// zcprobe.hip -- probe: latency of one small Encode whose stripe lives in
// pinned, device-mapped host memory (the sync API's zero-copy path).  Not
// part of the product.  Variants spread the same bytes over more CUs: W
// dwords per lane (4 or 1) and BS threads per block (256 or 64).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I xrs_amd/csrc tools/zcprobe.hip xrs_amd/csrc/gf256.cpp -o tools/zcprobe
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

typedef __attribute__((address_space(1))) uint32_t gu32;

template <int W>
__device__ __forceinline__ void ldq(uint32_t* v, uint64_t addr) {
  if constexpr (W == 4) {
    ld<true>(v, addr, 16);
  } else {
    v[0] = __builtin_nontemporal_load(reinterpret_cast<const gu32*>(addr));
  }
}
template <int W>
__device__ __forceinline__ void stq(const uint32_t* v, uint64_t addr) {
  if constexpr (W == 4) {
    st<true>(v, addr, 16);
  } else {
    __builtin_nontemporal_store(v[0], reinterpret_cast<gu32*>(addr));
  }
}

template <int W, int BS>
__global__ __launch_bounds__(BS) void enc_zc(const PairArgs<4, 12, true> a, uint64_t chunks) {
  constexpr int P = 4, C = 12;
  const uint64_t gid = static_cast<uint64_t>(blockIdx.x) * BS + threadIdx.x;
  const uint64_t total = chunks * (a.total / a.chunks);
  if (gid >= total) return;
  const uint64_t stripe = gid / chunks;
  const uint64_t off = (gid - stripe * chunks) * (4 * W);
  uint32_t acc_a[P][W] = {}, acc_b[P][W] = {};
  uint32_t xa[C][W], xb[C][W];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const uint64_t s = row_addr(a.src[c], stripe, off);
    ldq<W>(xa[c], s);
    ldq<W>(xb[c], s + a.half);
  }
#pragma unroll
  for (int c = 0; c < C; ++c) pair_mac1<P, W>(acc_a, acc_b, a.tab[c], xa[c], xb[c]);
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int w = 0; w < W; ++w) acc_b[1 + c % (P - 1)][w] ^= xa[c][w];
#pragma unroll
  for (int r = 0; r < P; ++r) {
    const uint64_t d = row_addr(a.dst[r], stripe, off);
    stq<W>(acc_a[r], d);
    stq<W>(acc_b[r], d + a.half);
  }
}

__global__ void empty_kernel() {}

}  // namespace
}  // namespace xrs

using namespace xrs;

int main() {
  const GF& gf = GF::get();
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto host_ms = [&](auto&& f, int reps) {
    for (int i = 0; i < 20; ++i) f();
    CK(hipStreamSynchronize(s));
    std::vector<double> t;
    for (int i = 0; i < reps; ++i) {
      CK(hipEventRecord(e0, s));
      f();
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t.push_back(ms * 1e3);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
  };
  std::printf("empty kernel: %.1f us (event to event)\n",
              host_ms([&] { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s); }, 200));
  for (uint64_t S : {4096ull, 16384ull, 65536ull}) {
    for (int n : {1, 8}) {
      const uint64_t stripe = 16 * S, H = S / 2;
      uint8_t* h;
      CK(hipHostMalloc(&h, n * stripe, hipHostMallocMapped));
      for (uint64_t i = 0; i < n * stripe; ++i) h[i] = static_cast<uint8_t>(i * 131 + 7);
      void* dp;
      CK(hipHostGetDevicePointer(&dp, h, 0));
      const uint64_t base = reinterpret_cast<uint64_t>(dp);
      PairArgs<4, 12, true> a;
      std::memset(&a, 0, sizeof(a));
      for (int c = 0; c < 12; ++c) {
        a.src[c] = {base + c * S, stripe};
        for (int r = 0; r < 4; ++r) a.tab[c][r] = gf.tab(gf.inv(static_cast<uint8_t>((12 + r) ^ c)));
      }
      for (int r = 0; r < 4; ++r) a.dst[r] = {base + (12 + r) * S, stripe};
      a.n_src = 12; a.half = H; a.chunks = H / 16; a.total = a.chunks * n;
      a.order = {static_cast<uint32_t>((a.total + 255) / 256), 0};
      std::vector<uint8_t> ref;
      auto run = [&](int W, int BS) {
        const uint64_t chunks = H / (4 * W), total = chunks * n;
        const unsigned blocks = static_cast<unsigned>((total + BS - 1) / BS);
        if (W == 4 && BS == 256) hipLaunchKernelGGL((enc_zc<4, 256>), dim3(blocks), dim3(256), 0, s, a, chunks);
        if (W == 4 && BS == 64) hipLaunchKernelGGL((enc_zc<4, 64>), dim3(blocks), dim3(64), 0, s, a, chunks);
        if (W == 1 && BS == 256) hipLaunchKernelGGL((enc_zc<1, 256>), dim3(blocks), dim3(256), 0, s, a, chunks);
        if (W == 1 && BS == 64) hipLaunchKernelGGL((enc_zc<1, 64>), dim3(blocks), dim3(64), 0, s, a, chunks);
      };
      const double tp = host_ms([&] { hipLaunchKernelGGL((pair_kernel<4, 12, false, true>), dim3(a.order.nblk), dim3(256), 0, s, a); }, 200);
      CK(hipStreamSynchronize(s));
      ref.assign(h, h + n * stripe);
      std::printf("S=%-6llu n=%d product pair_kernel: %.1f us\n", (unsigned long long)S, n, tp);
      for (int W : {4, 1})
        for (int BS : {256, 64}) {
          const double t = host_ms([&] { run(W, BS); }, 200);
          CK(hipStreamSynchronize(s));
          const bool same = std::memcmp(ref.data(), h, n * stripe) == 0;
          std::printf("S=%-6llu n=%d W=%d BS=%-3d: %.1f us%s\n", (unsigned long long)S, n, W, BS, t,
                      same ? "" : "  !! differs");
        }
      CK(hipHostFree(h));
    }
  }
  return 0;
}
