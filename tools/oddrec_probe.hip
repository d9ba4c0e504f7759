// oddrec_probe.hip -- ReconstOne's access pattern at an odd vect size, with
// the product's lane mapping, under four ways of reading misaligned rows.
//
// Layout: the bench's (stripes back to back, shards back to back), vect size
// S (4,100 by default, 4,096 as the aligned control): H = S/2-byte rows, lane
// = 16 B of a row, ceil(H/16) chunks per stripe, the last one overlapping
// (the product's ragged end).  Each lane reads the 16 rows ReconstOne(0)
// reads (11 data b-halves, P12 and P13 b-halves, a-halves of 3, 6, 9) and
// writes shard 0's two halves; the arithmetic is a stand-in of similar VALU
// weight (three v_perm + two XOR per output dword per row).
//   mode 0  direct dwordx4 loads at any alignment, nontemporal (the product)
//   mode 1  direct dwordx4 loads, temporal (may share a line between waves in L2)
//   mode 2  4-B-aligned dwordx4 + the next lane's first dword through DPP
//           (a one-dword spill load where the next lane is not contiguous),
//           v_alignbyte by the 0..3-byte remainder
//   mode 3  mode 2 for loads, temporal
//   mode 4  mode 0 with floor(H/16) lanes per stripe: no wave straddles a
//           stripe's ragged end; the last lane of each stripe also does the
//           overlapping tail chunk
// Not part of the product.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/oddrec_probe.hip -o tools/oddrec_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 gu32x4;
typedef __attribute__((address_space(1))) uint32_t gu32;

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      std::exit(1);                                                         \
    }                                                                       \
  } while (0)

template <bool NT>
__device__ __forceinline__ u32x4 ld16(uint64_t a) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const gu32x4*>(a));
  return *reinterpret_cast<const gu32x4*>(a);
}

__device__ __forceinline__ uint32_t next_lane(uint32_t v) {
  return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x130, 0xf, 0xf, false));
}

__device__ __forceinline__ int lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

// Phase 1 of a realigned read: the 4-B-aligned chunk under the lane's bytes.
template <bool NT>
__device__ __forceinline__ u32x4 ld_al4(uint64_t a) {
  return ld16<NT>(a & ~uint64_t(3));
}

// Phase 2: the 16 bytes at a, from the chunk c (loaded at a & ~3) and the
// next 4-B-aligned dword (the next lane's first dword when that lane's chunk
// follows on; else a one-dword load).
__device__ __forceinline__ u32x4 fix_al4(u32x4 c, uint64_t a) {
  const uint32_t r = static_cast<uint32_t>(a) & 3u;
  const uint32_t a4 = static_cast<uint32_t>(a) & ~3u;
  const uint32_t na4 = next_lane(a4);
  uint32_t nx = next_lane(c.x);
  if (r != 0 && (lane_id() == 63 || na4 != a4 + 16))
    nx = *reinterpret_cast<const gu32*>((a & ~uint64_t(3)) + 16);
  u32x4 o;
  o.x = __builtin_amdgcn_alignbyte(c.y, c.x, r);
  o.y = __builtin_amdgcn_alignbyte(c.z, c.y, r);
  o.z = __builtin_amdgcn_alignbyte(c.w, c.z, r);
  o.w = __builtin_amdgcn_alignbyte(nx, c.w, r);
  return o;
}

__device__ __forceinline__ uint32_t fake_gf(uint32_t x, uint32_t t0, uint32_t t1) {
  const uint32_t s0 = x & 0x07070707u, s1 = (x >> 3) & 0x07070707u, s2 = (x >> 6) & 0x03030303u;
  return __builtin_amdgcn_perm(t1, t0, s0) ^ __builtin_amdgcn_perm(t0, t1, s1) ^
         __builtin_amdgcn_perm(0u, t0, s2);
}

struct Rows {
  uint64_t src[16];  // stripe-0 address of each row read
  uint64_t dst[2];   // shard 0's b-half, a-half
};

template <int MODE>
__device__ __forceinline__ void rec_body(const Rows& r, uint64_t base, uint32_t t0, uint32_t t1);

template <int MODE>
__global__ __launch_bounds__(256) void rec_mix(const Rows r, uint64_t stride, uint64_t len,
                                              uint64_t chunks, uint64_t total, uint32_t t0,
                                              uint32_t t1) {
  const uint64_t gid = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (gid >= total) return;
  const uint64_t st = gid / chunks;
  uint64_t off = (gid - st * chunks) * 16;
  if constexpr (MODE == 4) {
    // floor(len/16) lanes per stripe (no lane straddles the ragged end); the
    // last lane of each stripe also does the overlapping tail chunk
    rec_body<0>(r, st * stride + off, t0, t1);
    if (off + 16 == chunks * 16 && len % 16) rec_body<0>(r, st * stride + len - 16, t0, t1);
    return;
  }
  if (off > len - 16) off = len - 16;
  rec_body<MODE>(r, st * stride + off, t0, t1);
}

template <int MODE>
__device__ __forceinline__ void rec_body(const Rows& r, uint64_t base, uint32_t t0, uint32_t t1) {
  constexpr bool NT = MODE == 0 || MODE == 2;
  constexpr bool AL4 = MODE == 2 || MODE == 3;
  u32x4 x[16];
#pragma unroll
  for (int m = 0; m < 16; ++m) x[m] = AL4 ? ld_al4<NT>(r.src[m] + base) : ld16<NT>(r.src[m] + base);
  if constexpr (AL4) {
#pragma unroll
    for (int m = 0; m < 16; ++m) x[m] = fix_al4(x[m], r.src[m] + base);
  }
  u32x4 b = {0, 0, 0, 0}, a = {0, 0, 0, 0};
#pragma unroll
  for (int m = 0; m < 12; ++m) {
    b.x ^= fake_gf(x[m].x, t0 + m, t1);
    b.y ^= fake_gf(x[m].y, t0 + m, t1);
    b.z ^= fake_gf(x[m].z, t0 + m, t1);
    b.w ^= fake_gf(x[m].w, t0 + m, t1);
    a.x ^= fake_gf(x[m].x, t1 + m, t0);
    a.y ^= fake_gf(x[m].y, t1 + m, t0);
    a.z ^= fake_gf(x[m].z, t1 + m, t0);
    a.w ^= fake_gf(x[m].w, t1 + m, t0);
  }
#pragma unroll
  for (int m = 12; m < 16; ++m) a ^= x[m];
  __builtin_nontemporal_store(b, reinterpret_cast<gu32x4*>(r.dst[0] + base));
  __builtin_nontemporal_store(a, reinterpret_cast<gu32x4*>(r.dst[1] + base));
}

// Correctness of the realigned read: gather 16 B at every offset of a row
// through fix_al4 and compare with the bytes.
__global__ void al4_copy(uint64_t src, uint64_t dst, uint64_t n, uint64_t len, uint64_t chunks) {
  const uint64_t gid = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (gid >= n) return;
  const uint64_t st = gid / chunks;
  uint64_t off = (gid - st * chunks) * 16;
  if (off > len - 16) off = len - 16;
  const uint64_t a = src + st * (len + 6) + off;  // rows len + 6 apart: every remainder
  const u32x4 c = ld_al4<true>(a);
  const u32x4 v = fix_al4(c, a);
  *reinterpret_cast<gu32x4*>(dst + st * len + off) = v;
}

template <int MODE>
double run(const Rows& r, uint64_t stride, uint64_t len, uint64_t n) {
  const uint64_t chunks = MODE == 4 ? len / 16 : (len + 15) / 16, total = chunks * n;
  const uint32_t nblk = static_cast<uint32_t>((total + 255) / 256);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 5; ++i) rec_mix<MODE><<<nblk, 256>>>(r, stride, len, chunks, total, 0x1234u, 0x5678u);
  CK(hipEventRecord(e0));
  const int reps = 20;
  for (int i = 0; i < reps; ++i)
    rec_mix<MODE><<<nblk, 256>>>(r, stride, len, chunks, total, 0x1234u, 0x5678u);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return static_cast<double>(n) * 18 * len * reps / (ms / 1e3) / 1e9;  // 9*S per stripe
}

int main(int argc, char** argv) {
  {  // correctness of fix_al4 at every remainder, across stripe ends
    const uint64_t len = 2050, n = 4096, chunks = (len + 15) / 16;
    const uint64_t sb = n * (len + 6) + 64;
    std::vector<uint8_t> h(sb), g(n * len);
    for (uint64_t i = 0; i < sb; ++i) h[i] = static_cast<uint8_t>(i * 131 + (i >> 8) * 7 + 1);
    uint8_t *src, *dst;
    CK(hipMalloc(&src, sb));
    CK(hipMalloc(&dst, n * len));
    CK(hipMemcpy(src, h.data(), sb, hipMemcpyHostToDevice));
    for (uint64_t mis = 0; mis < 4; ++mis) {
      const uint64_t tot = chunks * n;
      al4_copy<<<static_cast<unsigned>((tot + 255) / 256), 256>>>((uint64_t)src + mis, (uint64_t)dst, tot,
                                                                 len, chunks);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(g.data(), dst, n * len, hipMemcpyDeviceToHost));
      bool ok = true;
      for (uint64_t s = 0; s < n && ok; ++s)
        ok = std::memcmp(g.data() + s * len, h.data() + mis + s * (len + 6), len) == 0;
      std::printf("{\"check\": \"al4\", \"mis\": %lu, \"exact\": %s}\n", (unsigned long)mis,
                  ok ? "true" : "false");
      if (!ok) return 1;
    }
    CK(hipFree(src));
    CK(hipFree(dst));
  }
  const int sizes[] = {4100, 4096, 4104, 4098};
  const uint64_t bytes = 4300ull << 20;
  uint8_t* buf;
  CK(hipMalloc(&buf, bytes + 4096));
  CK(hipMemset(buf, 0x3c, bytes + 4096));
  for (int rep = 0; rep < 3; ++rep)
    for (int S : sizes) {
      const uint64_t len = S / 2, stride = 16ull * S, n = bytes / stride;
      Rows r;
      const uint64_t b = (uint64_t)buf;
      for (int m = 0; m < 11; ++m) r.src[m] = b + (m + 1) * S + len;  // data 1..11 b-halves
      r.src[11] = b + 12ull * S + len;                                // P12 b-half
      r.src[12] = b + 13ull * S + len;                                // P13 b-half
      r.src[13] = b + 3ull * S;                                       // a-halves 3, 6, 9
      r.src[14] = b + 6ull * S;
      r.src[15] = b + 9ull * S;
      r.dst[0] = b + len;
      r.dst[1] = b;
      const double g0 = run<0>(r, stride, len, n), g1 = run<1>(r, stride, len, n);
      const double g2 = run<2>(r, stride, len, n), g4 = run<4>(r, stride, len, n);
      std::printf("{\"round\": %d, \"vect\": %d, \"gbs_direct_nt\": %.1f, \"gbs_direct_t\": %.1f, "
                  "\"gbs_al4_nt\": %.1f, \"gbs_tail_lane\": %.1f}\n", rep, S, g0, g1, g2, g4);
      std::fflush(stdout);
    }
  CK(hipFree(buf));
  return 0;
}
