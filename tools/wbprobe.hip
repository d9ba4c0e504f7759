// wbprobe.hip -- does buffering outputs in registers (write-behind: a wave
// stores the outputs of T consecutive tiles in one burst, after all their
// loads) help HBM mix reads and writes?  Encode's memory pattern (12 source
// rows x 2 halves in, 4 parity rows x 2 halves out, 16 B per lane per row,
// nontemporal), XOR-only arithmetic, XCD block order K = 32 like the
// product.  Variants: T tiles per block, outputs stored per tile ("now") or
// after the last tile ("late").  Timing only; every index bounded by n.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 gu32x4;

__device__ __forceinline__ u32x4 ldv(uint64_t a) {
  return __builtin_nontemporal_load(reinterpret_cast<const gu32x4*>(a));
}
__device__ __forceinline__ void stv(uint64_t a, u32x4 v) {
  __builtin_nontemporal_store(v, reinterpret_cast<gu32x4*>(a));
}

struct Args {
  uint64_t base, S, H, stripe, chunks, total;  // total = lanes (16 B each) over all stripes
  uint32_t nsuper, k;                          // super-blocks in the grid, XCD order K
};

__device__ __forceinline__ uint32_t logical(uint32_t b, uint32_t nblk, uint32_t k) {
  const uint32_t q = b >> 3, g = q / k;
  if ((g + 1) * 8ull * k > nblk) return b;
  return g * 8 * k + (b & 7u) * k + (q - g * k);
}

template <int T, bool LATE>
__global__ __launch_bounds__(256) void wb(const Args a) {
  const uint32_t sb = logical(blockIdx.x, a.nsuper, a.k);
  u32x4 out[LATE ? T : 1][8];
  uint64_t addr[T];
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const uint64_t gid = (static_cast<uint64_t>(sb) * T + t) * 256 + threadIdx.x;
    addr[t] = ~0ull;
    if (gid >= a.total) continue;
    const uint64_t s = gid / a.chunks, off = (gid - s * a.chunks) * 16;
    const uint64_t st = a.base + s * a.stripe + off;
    addr[t] = st;
    u32x4 x[24];
#pragma unroll
    for (int c = 0; c < 12; ++c) {
      x[2 * c] = ldv(st + c * a.S);
      x[2 * c + 1] = ldv(st + c * a.S + a.H);
    }
    u32x4 o[8];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      o[2 * r] = x[2 * r] ^ x[2 * r + 8] ^ x[2 * r + 16];
      o[2 * r + 1] = x[2 * r + 1] ^ x[2 * r + 9] ^ x[2 * r + 17] ^ x[(2 * r + 6) % 24];
    }
    if constexpr (LATE) {
#pragma unroll
      for (int j = 0; j < 8; ++j) out[t][j] = o[j];
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        stv(st + (12 + r) * a.S, o[2 * r]);
        stv(st + (12 + r) * a.S + a.H, o[2 * r + 1]);
      }
    }
  }
  if constexpr (LATE) {
#pragma unroll
    for (int t = 0; t < T; ++t) {
      if (addr[t] == ~0ull) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        stv(addr[t] + (12 + r) * a.S, out[t][2 * r]);
        stv(addr[t] + (12 + r) * a.S + a.H, out[t][2 * r + 1]);
      }
    }
  }
}

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      std::exit(1);                                                         \
    }                                                                       \
  } while (0)

template <int T, bool LATE>
float run(const Args& a0, int reps) {
  Args a = a0;
  const uint64_t blocks = (a.total + 256 * T - 1) / (256 * T);
  a.nsuper = static_cast<uint32_t>(blocks);
  a.k = 32 / T > 0 ? 32 / T : 1;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) wb<T, LATE><<<blocks, 256>>>(a);
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) wb<T, LATE><<<blocks, 256>>>(a);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return ms / reps;
}

int main() {
  for (uint64_t S : {4096ull, 1ull << 20}) {
    const uint64_t n = (4ull << 30) / (16 * S);
    uint8_t* buf;
    CK(hipMalloc(&buf, n * 16 * S));
    CK(hipMemset(buf, 1, n * 16 * S));
    Args a{reinterpret_cast<uint64_t>(buf), S, S / 2, 16 * S, S / 32, n * (S / 32), 0, 0};
    const double bytes = 16.0 * S * n;
    // clock ramp
    for (int i = 0; i < 60; ++i) run<1, false>(a, 1);
    for (int round = 0; round < 3; ++round) {
      const float t1 = run<1, false>(a, 10), t2n = run<2, false>(a, 10), t2l = run<2, true>(a, 10),
                  t3l = run<3, true>(a, 10), t4l = run<4, true>(a, 10);
      std::printf("{\"S\": %llu, \"round\": %d, \"T1\": %.1f, \"T2_now\": %.1f, \"T2_late\": %.1f, "
                  "\"T3_late\": %.1f, \"T4_late\": %.1f}\n",
                  static_cast<unsigned long long>(S), round, bytes / t1 / 1e6, bytes / t2n / 1e6,
                  bytes / t2l / 1e6, bytes / t3l / 1e6, bytes / t4l / 1e6);
      std::fflush(stdout);
    }
    CK(hipFree(buf));
  }
  return 0;
}
