// storeprobe.hip -- probe: store cache policy in the XCD block order.  Not part
// of the product.  The product stores are nontemporal (global_store ... nt);
// this compares plain stores and relaxed atomic dword stores at agent and
// system scope (the compiler sets the gfx950 sc0/sc1 bits; no inline asm), and
// plain vs nontemporal loads, on the Encode 4 KiB / 1 MiB and ReconstOne 1 MiB
// patterns.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I xrs_amd/csrc tools/storeprobe.hip xrs_amd/csrc/gf256.cpp -o tools/storeprobe
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

// SM: 0 nt store, 1 plain store, 2 relaxed atomic dwords (agent), 3 (system).
template <int SM>
__device__ __forceinline__ void st4(const uint32_t* v, uint64_t addr) {
  if constexpr (SM == 0) {
    st<true>(v, addr, 16);
  } else if constexpr (SM == 1) {
    u32x4 t = {v[0], v[1], v[2], v[3]};
    *reinterpret_cast<gu32x4*>(addr) = t;
  } else {
    __attribute__((address_space(1))) uint32_t* p = reinterpret_cast<__attribute__((address_space(1))) uint32_t*>(addr);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __hip_atomic_store(p + i, v[i], __ATOMIC_RELAXED,
                         SM == 2 ? __HIP_MEMORY_SCOPE_AGENT : __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

template <bool NTL>
__device__ __forceinline__ void ld4(uint32_t* v, uint64_t addr) {
  if constexpr (NTL) {
    ld<true>(v, addr, 16);
  } else {
    const u32x4 t = *reinterpret_cast<const gu32x4*>(addr);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  }
}

template <int SM, bool NTL>
__global__ __launch_bounds__(256) void enc_sp(const PairArgs<4, 12, true> a) {
  constexpr int P = 4, C = 12, W = 4;
  const uint64_t gid = logical_block(a.order) * 256 + threadIdx.x;
  if (gid >= a.total) return;
  const uint64_t stripe = gid / a.chunks;
  const uint64_t off = (gid - stripe * a.chunks) * 16;
  uint32_t acc_a[P][W] = {}, acc_b[P][W] = {};
  uint32_t xa[C][W], xb[C][W];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const uint64_t s = row_addr(a.src[c], stripe, off);
    ld4<NTL>(xa[c], s);
    ld4<NTL>(xb[c], s + a.half);
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
    st4<SM>(acc_a[r], d);
    st4<SM>(acc_b[r], d + a.half);
  }
}

template <int SM, bool NTL>
__global__ __launch_bounds__(256) void r1_sp(const RowsArgs<2, 12, 4, true> a) {
  constexpr int R = 2, NM = 12, NX = 4, W = 4;
  const uint64_t gid = logical_block(a.order) * 256 + threadIdx.x;
  if (gid >= a.total) return;
  const uint64_t stripe = gid / a.chunks;
  const uint64_t off = (gid - stripe * a.chunks) * 16;
  uint32_t acc[R][W] = {};
  uint32_t xm[NM][W], xx[NX][W];
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int m = 0; m < NM; ++m) ld4<NTL>(xm[m], row_addr(a.msrc[m], stripe, off));
#pragma unroll
  for (int x = 0; x < NX; ++x) ld4<NTL>(xx[x], row_addr(a.xsrc[x], stripe, off));
  __builtin_amdgcn_s_setprio(0);
#pragma unroll
  for (int m = 0; m + 1 < NM; m += 2) rows_mac2<R, W>(acc, a.tab[m], a.tab[m + 1], xm[m], xm[m + 1]);
#pragma unroll
  for (int x = 0; x < NX; ++x) rows_xor<R, W>(acc, a.xmask[x], xx[x]);
#pragma unroll
  for (int r = 0; r < R; ++r) st4<SM>(acc[r], row_addr(a.dst[r], stripe, off));
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

const char* kName[] = {"nt store", "plain store", "atomic agent", "atomic system"};

template <class A, class K>
void run(Timer& tm, const char* op, uint64_t S, const A& a, uint64_t nblk, uint8_t* buf, uint64_t bytes_buf,
         double bytes, K (&ks)[2][4]) {
  hipLaunchKernelGGL(ks[1][0], dim3(nblk), dim3(256), 0, 0, a);
  const unsigned long long ref = checksum(buf, bytes_buf);
  std::vector<double> t[2][4];
  for (int r = 0; r < 7; ++r)
    for (int l = 0; l < 2; ++l)
      for (int m = 0; m < 4; ++m) t[l][m].push_back(tm.ms([&] { hipLaunchKernelGGL(ks[l][m], dim3(nblk), dim3(256), 0, 0, a); }));
  for (int l = 0; l < 2; ++l)
    for (int m = 0; m < 4; ++m) {
      std::sort(t[l][m].begin(), t[l][m].end());
      const double ms = t[l][m][3];
      std::printf("%s S=%-8llu %s loads, %-14s %8.3f ms  %8.1f GB/s\n", op, (unsigned long long)S,
                  l ? "nt   " : "plain", kName[m], ms, bytes / ms / 1e6);
    }
  if (checksum(buf, bytes_buf) != ref) std::printf("   !! output differs\n");
  std::fflush(stdout);
}

}  // namespace
}  // namespace xrs

using namespace xrs;

int main() {
  const GF& gf = GF::get();
  Timer tm;
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
    const uint64_t nblk = a.total / 256;
    a.order = {static_cast<uint32_t>(nblk), 32};
    void (*ke[2][4])(const PairArgs<4, 12, true>) = {{enc_sp<0, false>, enc_sp<1, false>, enc_sp<2, false>, enc_sp<3, false>},
                                                     {enc_sp<0, true>, enc_sp<1, true>, enc_sp<2, true>, enc_sp<3, true>}};
    run(tm, "enc", S, a, nblk, buf, n * stripe, 16.0 * S * n, ke);

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
    const uint64_t nb1 = r.total / 256;
    r.order = {static_cast<uint32_t>(nb1), S <= 4096 ? static_cast<uint32_t>(nb1 / 8) : 128u};
    void (*kr[2][4])(const RowsArgs<2, 12, 4, true>) = {{r1_sp<0, false>, r1_sp<1, false>, r1_sp<2, false>, r1_sp<3, false>},
                                                        {r1_sp<0, true>, r1_sp<1, true>, r1_sp<2, true>, r1_sp<3, true>}};
    run(tm, "r1 ", S, r, nb1, buf, n * stripe, 9.0 * S * n, kr);
    CK(hipFree(buf));
  }
  return 0;
}
