// oddprobe.hip -- why do vect sizes that are not a multiple of 128 B run
// slower?  Encode's access pattern (12 source rows, both halves, 4 output
// rows) with XOR in place of the GF arithmetic, at shard strides 4096 / 4100 /
// 4128 / 1 MiB / 1 MiB + 2, with nontemporal or plain loads and stores.
// Timing only (plus a bounded-index check on the host); not part of the product.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/oddprobe.hip -o tools/oddprobe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 gu32x4;

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);         \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

template <bool NT>
__device__ __forceinline__ u32x4 ld(uint64_t a) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const gu32x4*>(a));
  else return *reinterpret_cast<const gu32x4*>(a);
}
template <bool NT>
__device__ __forceinline__ void st(u32x4 v, uint64_t a) {
  if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<gu32x4*>(a));
  else *reinterpret_cast<gu32x4*>(a) = v;
}

// One lane: 16 B at offset `off` of both halves of 12 source rows and 4 output
// rows of one stripe.  XCD-aware order as in the product (K = 32).
// chunks: lanes per stripe-half (>= ceil(half/16); rounded up to a multiple of
// 64 = one wave never spans two stripes, the extra lanes exit).
template <bool NTL, bool NTS>
__global__ __launch_bounds__(256) void enc_xor(uint64_t base, uint64_t shard, uint64_t half,
                                              uint64_t chunks, uint64_t total, uint32_t nblk) {
  const uint32_t b = blockIdx.x, q = b >> 3, k = 32, g = q / k;
  uint64_t lb = b;
  if ((uint64_t)(g + 1) * 8 * k <= nblk) lb = (uint64_t)g * 8 * k + (b & 7u) * k + (q - g * k);
  const uint64_t gid = lb * 256 + threadIdx.x;
  if (gid >= total) return;
  const uint64_t stripe = gid / chunks;
  uint64_t off = (gid - stripe * chunks) * 16;
  if (off >= half) return;               // wave-aligned padding lanes
  if (off > half - 16) off = half - 16;  // ragged end: overlapping last chunk
  const uint64_t s0 = base + stripe * 16 * shard;
  u32x4 a[12], bb[12];
#pragma unroll
  for (int c = 0; c < 12; ++c) {
    a[c] = ld<NTL>(s0 + c * shard + off);
    bb[c] = ld<NTL>(s0 + c * shard + half + off);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    u32x4 xa = a[r] ^ a[r + 4] ^ a[r + 8], xb = bb[r] ^ bb[r + 4] ^ bb[r + 8];
    if (r) xb ^= a[r - 1];
    st<NTS>(xa, s0 + (12 + r) * shard + off);
    st<NTS>(xb, s0 + (12 + r) * shard + half + off);
  }
}

// ReconstOne's access pattern (k = 0 at 12+4): b-halves of shards 1..13,
// a-halves of shards 3, 6, 9 read; both halves of shard 0 written.
__global__ __launch_bounds__(256) void rec_xor(uint64_t base, uint64_t shard, uint64_t half,
                                              uint64_t chunks, uint64_t total, uint32_t nblk) {
  const uint32_t b = blockIdx.x;
  const uint64_t lb = (nblk >= 8) ? (uint64_t)(b & 7u) * (nblk / 8) + (b >> 3) : b;  // one range per XCD
  if ((nblk & 7u) != 0 && b >= nblk / 8 * 8) return;  // (probe: whole groups only)
  const uint64_t gid = lb * 256 + threadIdx.x;
  if (gid >= total) return;
  const uint64_t stripe = gid / chunks;
  uint64_t off = (gid - stripe * chunks) * 16;
  if (off > half - 16) off = half - 16;
  const uint64_t s0 = base + stripe * 16 * shard;
  u32x4 v[16];
#pragma unroll
  for (int c = 0; c < 13; ++c) v[c] = ld<true>(s0 + (1 + c) * shard + half + off);
  v[13] = ld<true>(s0 + 3 * shard + off);
  v[14] = ld<true>(s0 + 6 * shard + off);
  v[15] = ld<true>(s0 + 9 * shard + off);
  u32x4 x0 = v[0], x1 = v[1];
#pragma unroll
  for (int c = 2; c < 16; c += 2) {
    x0 ^= v[c];
    x1 ^= v[c + 1];
  }
  st<true>(x0, s0 + half + off);
  st<true>(x1, s0 + off);
}

double run_rec(uint8_t* buf, uint64_t shard, uint64_t size, uint64_t n) {
  const uint64_t half = size / 2, chunks = (half + 15) / 16, total = chunks * n;
  const uint32_t nblk = (uint32_t)((total + 255) / 256);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 30; ++i) rec_xor<<<nblk, 256>>>((uint64_t)buf, shard, half, chunks, total, nblk);
  CK(hipEventRecord(e0));
  const int reps = 20;
  for (int i = 0; i < reps; ++i) rec_xor<<<nblk, 256>>>((uint64_t)buf, shard, half, chunks, total, nblk);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return (double)n * 9 * size * reps / (ms / 1e3) / 1e9;
}

template <bool NTL, bool NTS>
double run(uint8_t* buf, uint64_t shard, uint64_t size, uint64_t n, bool wave_align = false) {
  const uint64_t half = size / 2;
  uint64_t chunks = (half + 15) / 16;
  if (wave_align) chunks = (chunks + 63) / 64 * 64;
  const uint64_t total = chunks * n;
  const uint32_t nblk = (uint32_t)((total + 255) / 256);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 30; ++i)
    enc_xor<NTL, NTS><<<nblk, 256>>>((uint64_t)buf, shard, half, chunks, total, nblk);
  CK(hipEventRecord(e0));
  const int reps = 20;
  for (int i = 0; i < reps; ++i)
    enc_xor<NTL, NTS><<<nblk, 256>>>((uint64_t)buf, shard, half, chunks, total, nblk);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return (double)n * 16 * size * reps / (ms / 1e3) / 1e9;
}

int main() {
  const uint64_t budget = 4ull << 30;
  uint8_t* buf;
  CK(hipMalloc(&buf, budget + (1 << 20)));
  CK(hipMemset(buf, 0x3c, budget + (1 << 20)));
  // Shard-stride sweep: vect size -> strides tried (stripe stride = 16 shards).
  struct Case {
    uint64_t size;
    int nstrides;
    uint64_t strides[14];
  };
  const Case cases[] = {
      {4096, 3, {4096, 4112, 4224}},
      {4100, 5, {4100, 4108, 4112, 4116, 4224}},
      {4128, 1, {4128}},
      {1 << 20, 9, {1 << 20, (1 << 20) + 16, (1 << 20) + 32, (1 << 20) + 64, (1 << 20) + 128,
                    (1 << 20) + 256, (1 << 20) + 1024, (1 << 20) + 4096, (1 << 20) + 4352}},
      {(1 << 20) + 2, 9, {(1 << 20) + 2, (1 << 20) + 16, (1 << 20) + 32, (1 << 20) + 64,
                          (1 << 20) + 128, (1 << 20) + 256, (1 << 20) + 1024, (1 << 20) + 4096,
                          (1 << 20) + 4352}},
  };
  for (int rep = 0; rep < 2; ++rep)
    for (const Case& c : cases)
      for (int i = 0; i < c.nstrides; ++i) {
        const uint64_t shard = c.strides[i], n = budget / (16 * shard);
        const double g0 = run<true, true>(buf, shard, c.size, n);
        const double g1 = run_rec(buf, shard, c.size, n / 8 * 8);
        std::printf("{\"round\": %d, \"vect_bytes\": %llu, \"shard_stride\": %llu, "
                    "\"gbs_encode\": %.1f, \"gbs_reconst_one\": %.1f}\n",
                    rep, (unsigned long long)c.size, (unsigned long long)shard, g0, g1);
        std::fflush(stdout);
      }
  CK(hipFree(buf));
  return 0;
}
