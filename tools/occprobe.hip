// occprobe.hip -- probe: does capping waves per CU (unused dynamic LDS limits
// resident blocks) change the HBM rate of the product kernels?  Not part of
// the product.  ReconstOne (96 VGPRs) runs up to 20 waves/CU by registers,
// Encode (170 VGPRs) 8.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I xrs_amd/csrc tools/occprobe.hip xrs_amd/csrc/gf256.cpp -o tools/occprobe
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
}  // namespace
}  // namespace xrs

using namespace xrs;

int main() {
  const GF& gf = GF::get();
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto ms = [&](auto&& f) {
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < 5; ++i) f();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float t;
    CK(hipEventElapsedTime(&t, e0, e1));
    return t / 5;
  };
  const size_t lds[] = {0, 16 << 10, 20 << 10, 27 << 10, 33 << 10, 40 << 10, 54 << 10, 80 << 10};
  for (uint64_t S : {4096ull, 1ull << 20}) {
    const uint64_t n = (4ull << 30) / (16 * S), H = S / 2, stripe = 16 * S;
    uint8_t* buf;
    CK(hipMalloc(&buf, n * stripe));
    hipLaunchKernelGGL(fill_kernel, dim3(8192), dim3(256), 0, 0, (uint32_t*)buf, n * stripe / 4, 9u);
    const uint64_t base = reinterpret_cast<uint64_t>(buf);
    PairArgs<4, 12, true> a;
    std::memset(&a, 0, sizeof(a));
    for (int c = 0; c < 12; ++c) {
      a.src[c] = {base + c * S, stripe};
      for (int r = 0; r < 4; ++r) a.tab[c][r] = gf.tab(gf.inv(static_cast<uint8_t>((12 + r) ^ c)));
    }
    for (int r = 0; r < 4; ++r) a.dst[r] = {base + (12 + r) * S, stripe};
    a.n_src = 12; a.half = H; a.chunks = H / 16; a.total = a.chunks * n;
    const uint32_t nb = static_cast<uint32_t>(a.total / 256);
    a.order = {nb, 32};
    RowsArgs<2, 12, 4, true> r;
    std::memset(&r, 0, sizeof(r));
    for (int m = 0; m < 12; ++m) {
      r.msrc[m] = {base + (m == 0 ? 12 : m) * S + H, stripe};
      for (int q = 0; q < 2; ++q) r.tab[m][q] = gf.tab(static_cast<uint8_t>(17 * m + 5 * q + 3));
    }
    r.xsrc[0] = {base + 13 * S + H, stripe};
    for (int x = 1; x < 4; ++x) r.xsrc[x] = {base + 3 * x * S, stripe};
    for (int x = 0; x < 4; ++x) r.xmask[x] = 2;
    r.dst[0] = {base + H, stripe};
    r.dst[1] = {base, stripe};
    r.nm = 12; r.nx = 4; r.len = H; r.chunks = H / 16; r.total = r.chunks * n;
    const uint32_t nr = static_cast<uint32_t>(r.total / 256);
    r.order = {nr, S <= 4096 ? nr / 8 : 64u};
    std::vector<double> te[8], tr[8];
    for (int round = 0; round < 7; ++round)
      for (int i = 0; i < 8; ++i) {
        te[i].push_back(ms([&] { hipLaunchKernelGGL((pair_kernel<4, 12, false, true>), dim3(nb), dim3(256), lds[i], 0, a); }));
        tr[i].push_back(ms([&] { hipLaunchKernelGGL((rows_kernel<2, 12, 4, false, true>), dim3(nr), dim3(256), lds[i], 0, r); }));
      }
    for (int i = 0; i < 8; ++i) {
      int be = 0, br = 0;
      CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&be, (pair_kernel<4, 12, false, true>), 256, lds[i]));
      CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&br, (rows_kernel<2, 12, 4, false, true>), 256, lds[i]));
      std::sort(te[i].begin(), te[i].end());
      std::sort(tr[i].begin(), tr[i].end());
      std::printf("S=%-8llu lds=%3zuK  enc %2d waves/CU %8.1f GB/s   r1 %2d waves/CU %8.1f GB/s\n",
                  (unsigned long long)S, lds[i] >> 10, 4 * be, 16.0 * S * n / te[i][3] / 1e6, 4 * br,
                  9.0 * S * n / tr[i][3] / 1e6);
    }
    std::fflush(stdout);
    CK(hipFree(buf));
  }
  return 0;
}
