// tdm.hip -- probe: time-division multiplexing of HBM between reads and writes.
// Not part of the product.
//
// Question: Encode loses 14-22% to reads and writes sharing the HBM channels
// (profiles/r01_kbench10.log: reads alone 7.18 TB/s, writes alone 6.0 TB/s,
// mixed 6.0 TB/s).  Can a persistent kernel separate them in time across the
// whole chip?  Every wave reads and computes M work units into registers, then
// stores them only inside a chip-wide write slot of a fixed period measured
// on the constant-rate clock (s_memrealtime), so all CUs switch together
// without any inter-wave communication.  Every wave waits at most one period
// per unit batch, so the grid always drains.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I xrs_amd/csrc tools/tdm.hip -o tools/tdm
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

__device__ __forceinline__ uint64_t now() { return __builtin_amdgcn_s_memrealtime(); }

// Encode 12+4, one work unit = 64 lanes x 16 B of the a-half (and the b-half)
// of one stripe.  GFM: the product arithmetic; else XOR only (memory probe).
// SYNC: store only inside the write slot [rslot, period) of the clock.
template <int M, bool GFM, bool SYNC>
__global__ __launch_bounds__(256) void enc_tdm(const PairArgs<4, 12, true> a, uint64_t pmask,
                                               uint64_t rslot) {
  constexpr int P = 4, C = 12, W = 4;
  const uint64_t lane = threadIdx.x & 63;
  const uint64_t wave = (static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x) >> 6;
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * 4;
  const uint64_t units = a.total >> 6;
  if (SYNC)
    while ((now() & pmask) >= rslot) __builtin_amdgcn_s_sleep(2);
  for (uint64_t u0 = wave * M; u0 < units; u0 += nw * M) {
    uint32_t oa[M][P][W], ob[M][P][W];
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const uint64_t u = u0 + m;
      if (u >= units) break;
      const uint64_t gid = u * 64 + lane;
      const uint64_t stripe = gid / a.chunks;
      const uint64_t off = (gid - stripe * a.chunks) * 16;
      uint32_t xa[C][W], xb[C][W];
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const uint64_t s = row_addr(a.src[c], stripe, off);
        ld<true>(xa[c], s, 16);
        ld<true>(xb[c], s + a.half, 16);
      }
#pragma unroll
      for (int r = 0; r < P; ++r)
#pragma unroll
        for (int w = 0; w < W; ++w) oa[m][r][w] = ob[m][r][w] = 0u;
      if constexpr (GFM) {
#pragma unroll
        for (int c = 0; c + 1 < C; c += 2)
          pair_mac2<P, W>(oa[m], ob[m], a.tab[c], a.tab[c + 1], xa[c], xb[c], xa[c + 1], xb[c + 1]);
      } else {
#pragma unroll
        for (int c = 0; c < C; ++c)
#pragma unroll
          for (int w = 0; w < W; ++w) {
            oa[m][c & 3][w] ^= xa[c][w];
            ob[m][c & 3][w] ^= xb[c][w];
          }
      }
#pragma unroll
      for (int c = 0; c < C; ++c)
#pragma unroll
        for (int w = 0; w < W; ++w) ob[m][1 + c % (P - 1)][w] ^= xa[c][w];
    }
    if (SYNC)
      while ((now() & pmask) < rslot) __builtin_amdgcn_s_sleep(2);
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const uint64_t u = u0 + m;
      if (u >= units) break;
      const uint64_t gid = u * 64 + lane;
      const uint64_t stripe = gid / a.chunks;
      const uint64_t off = (gid - stripe * a.chunks) * 16;
#pragma unroll
      for (int r = 0; r < P; ++r) {
        const uint64_t d = row_addr(a.dst[r], stripe, off);
        st<true>(oa[m][r], d, 16);
        st<true>(ob[m][r], d + a.half, 16);
      }
    }
    if (SYNC)
      while ((now() & pmask) >= rslot) __builtin_amdgcn_s_sleep(2);
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

template <class K>
int resident_blocks(K kern) {
  int per_cu = 0, cus = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 256, 0));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  return per_cu * cus;
}

}  // namespace
}  // namespace xrs

using namespace xrs;

int main(int argc, char** argv) {
  const GF& gf = GF::get();
  int clk_khz = 0;
  CK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeWallClockRate, 0));
  std::printf("wall clock %d kHz\n", clk_khz);
  // Encode 12+4 @ 4 KiB, 65,536 stripes (4 GiB), contiguous.
  const uint64_t S = 4096, n = 65536, H = S / 2, stripe = 16 * S;
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
  const unsigned blocks = (unsigned)(a.total / 256);
  const double bytes = 16.0 * S * n;
  Timer tm;
  hipLaunchKernelGGL((pair_kernel<4, 12, false, true>), dim3(blocks), dim3(256), 0, 0, a);
  const unsigned long long ref = checksum(buf, n * stripe);

  struct Var { const char* name; void (*k)(const PairArgs<4, 12, true>, uint64_t, uint64_t); bool gfm; };
  const Var vars[] = {
      {"xor M=1 free", enc_tdm<1, false, false>, false}, {"xor M=2 free", enc_tdm<2, false, false>, false},
      {"xor M=4 free", enc_tdm<4, false, false>, false}, {"xor M=1 tdm", enc_tdm<1, false, true>, false},
      {"xor M=2 tdm", enc_tdm<2, false, true>, false},   {"xor M=4 tdm", enc_tdm<4, false, true>, false},
      {"gf  M=2 tdm", enc_tdm<2, true, true>, true},     {"gf  M=4 tdm", enc_tdm<4, true, true>, true},
  };
  for (const Var& v : vars) {
    int rb = resident_blocks(v.k);
    hipFuncAttributes fa;
    CK(hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(v.k)));
    std::printf("%-16s regs=%d resident blocks=%d\n", v.name, fa.numRegs, rb);
  }
  auto report = [&](const char* name, double ms) {
    std::printf("%-44s %8.3f ms  %8.1f GB/s  (%.1f%%)\n", name, ms, bytes / ms / 1e6, bytes / ms / 1e6 / 80.0);
    std::fflush(stdout);
  };
  std::vector<double> tp;
  for (int r = 0; r < 3; ++r)
    tp.push_back(tm.ms([&] { hipLaunchKernelGGL((pair_kernel<4, 12, false, true>), dim3(blocks), dim3(256), 0, 0, a); }));
  std::sort(tp.begin(), tp.end());
  report("product pair_kernel", tp[1]);
  const uint64_t periods[] = {1024, 2048, 4096, 8192};
  const double rfr[] = {0.68, 0.74, 0.80};
  for (const Var& v : vars) {
    const int rb = resident_blocks(v.k);
    const bool sync = std::strstr(v.name, "tdm") != nullptr;
    for (int gm : {1, 2}) {
      const unsigned g = static_cast<unsigned>(rb * gm);
      for (uint64_t per : periods) {
        for (double fr : rfr) {
          if (!sync && (per != 1024 || fr != 0.68)) continue;
          const uint64_t rs = static_cast<uint64_t>(per * fr);
          std::vector<double> t;
          for (int r = 0; r < 3; ++r)
            t.push_back(tm.ms([&] { hipLaunchKernelGGL(v.k, dim3(g), dim3(256), 0, 0, a, per - 1, rs); }));
          std::sort(t.begin(), t.end());
          char name[128];
          if (sync)
            std::snprintf(name, sizeof name, "%s grid=%ux per=%llu r=%.2f", v.name, gm, (unsigned long long)per, fr);
          else
            std::snprintf(name, sizeof name, "%s grid=%ux", v.name, gm);
          report(name, t[1]);
          if (v.gfm && checksum(buf, n * stripe) != ref) std::printf("   !! output differs\n");
        }
      }
    }
    if (!v.gfm) hipLaunchKernelGGL((pair_kernel<4, 12, false, true>), dim3(blocks), dim3(256), 0, 0, a);
  }
  CK(hipFree(buf));
  return 0;
}
