// dppprobe.hip -- can misaligned rows be read as aligned 16-B loads plus an
// in-register realignment?  A lane loads the 16-B-aligned chunk under its
// bytes, takes the next lane's chunk through DPP wave_shl:1 (lane 63 takes an
// extra one-lane load of the chunk after the wave), and funnels the two with
// v_alignbyte_b32 (a uniform switch on the dword part of the misalignment).
//
// 1. Correctness: realign a buffer at every misalignment 0..15 (+ 16, 34) and
//    compare with the bytes read directly.
// 2. Timing: Encode's mix (12 rows read, 4 written, XOR in place of the GF
//    arithmetic) with every read row misaligned by mr bytes and every written
//    row by mw, read either directly (unaligned dwordx4, what the product
//    kernels do) or through the DPP realignment.
// Not part of the product.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/dppprobe.hip -o tools/dppprobe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

__device__ __forceinline__ u32x4 ld(uint64_t a) {
  return __builtin_nontemporal_load(reinterpret_cast<const gu32x4*>(a));
}
__device__ __forceinline__ void st(u32x4 v, uint64_t a) {
  __builtin_nontemporal_store(v, reinterpret_cast<gu32x4*>(a));
}

// The next lane's dword (lane 63: `old`, the spill-over chunk).
__device__ __forceinline__ uint32_t next_lane(uint32_t old, uint32_t v) {
  return static_cast<uint32_t>(
      __builtin_amdgcn_update_dpp(static_cast<int>(old), static_cast<int>(v), 0x130, 0xf, 0xf, false));
}

// 16 bytes starting `d` (0..15, wave-uniform) bytes into this lane's aligned
// chunk c; nx = the next lane's chunk.
template <int Q>
__device__ __forceinline__ u32x4 funnel_q(const uint32_t (&D)[8], uint32_t r) {
  u32x4 o;
  o.x = __builtin_amdgcn_alignbyte(D[Q + 1], D[Q + 0], r);
  o.y = __builtin_amdgcn_alignbyte(D[Q + 2], D[Q + 1], r);
  o.z = __builtin_amdgcn_alignbyte(D[Q + 3], D[Q + 2], r);
  o.w = __builtin_amdgcn_alignbyte(D[Q + 4], D[Q + 3], r);
  return o;
}

// Load 16 B at byte address `a` (any alignment) as an aligned chunk + realign.
// All lanes of the wave must load consecutive 16-B pieces of one row.
__device__ __forceinline__ u32x4 ld_realign(uint64_t a) {
  const uint32_t d = static_cast<uint32_t>(a) & 15u;  // wave-uniform by contract
  const uint64_t al = a - d;
  const u32x4 c = ld(al);
  if (__builtin_amdgcn_readfirstlane(d) == 0) return c;
  const int lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  u32x4 e = {0, 0, 0, 0};
  if (lane == 63) e = ld(al + 16);
  const uint32_t D[8] = {c.x, c.y, c.z, c.w, next_lane(e.x, c.x), next_lane(e.y, c.y),
                         next_lane(e.z, c.z), next_lane(e.w, c.w)};
  const uint32_t r = d & 3u;
  switch (__builtin_amdgcn_readfirstlane(d >> 2)) {
    case 0: return funnel_q<0>(D, r);
    case 1: return funnel_q<1>(D, r);
    case 2: return funnel_q<2>(D, r);
    default: return funnel_q<3>(D, r);
  }
}

__global__ __launch_bounds__(256) void realign_copy(uint64_t src, uint64_t dst, uint64_t n16,
                                                    uint32_t mis) {
  const uint64_t gid = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (gid >= n16) return;
  st(ld_realign(src + mis + gid * 16), dst + gid * 16);
}

__device__ __forceinline__ int lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

// Realign an aligned chunk c (+ the next lane's chunk, lane 63: e) by d bytes.
__device__ __forceinline__ u32x4 realign(u32x4 c, u32x4 e, uint32_t d) {
  const uint32_t D[8] = {c.x, c.y, c.z, c.w, next_lane(e.x, c.x), next_lane(e.y, c.y),
                         next_lane(e.z, c.z), next_lane(e.w, c.w)};
  const uint32_t r = d & 3u;
  switch (__builtin_amdgcn_readfirstlane(d >> 2)) {
    case 0: return funnel_q<0>(D, r);
    case 1: return funnel_q<1>(D, r);
    case 2: return funnel_q<2>(D, r);
    default: return funnel_q<3>(D, r);
  }
}

// The previous lane's dword (lane 0: `old`).
__device__ __forceinline__ uint32_t prev_lane(uint32_t old, uint32_t v) {
  return static_cast<uint32_t>(
      __builtin_amdgcn_update_dpp(static_cast<int>(old), static_cast<int>(v), 0x138, 0xf, 0xf, false));
}

// Bytes [lo, hi) of the 16-B value v to the aligned chunk at a (narrow stores).
__device__ __forceinline__ void st_bytes(u32x4 v, uint64_t a, uint32_t lo, uint32_t hi) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  for (uint32_t b = lo; b < hi;) {
    const uint32_t sh = 8 * (b & 3);
    if ((b & 3) == 0 && b + 4 <= hi) {
      *reinterpret_cast<__attribute__((address_space(1))) uint32_t*>(a + b) = w[b >> 2];
      b += 4;
    } else if ((b & 1) == 0 && b + 2 <= hi) {
      *reinterpret_cast<__attribute__((address_space(1))) uint16_t*>(a + b) =
          static_cast<uint16_t>(w[b >> 2] >> sh);
      b += 2;
    } else {
      *reinterpret_cast<__attribute__((address_space(1))) uint8_t*>(a + b) =
          static_cast<uint8_t>(w[b >> 2] >> sh);
      b += 1;
    }
  }
}

// Store this lane's 16 output bytes (logically at a, misaligned by d, wave-
// uniform; the wave's lanes cover one contiguous KiB) as aligned chunks: lane
// k writes chunk k = the previous lane's last d bytes + its first 16 - d;
// lane 0 writes only its part of chunk 0, lane 63 also the head of chunk 64.
__device__ __forceinline__ void st_realign(u32x4 o, uint64_t a) {
  const uint32_t d = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a) & 15u);
  if (d == 0) {
    st(o, a);
    return;
  }
  const uint64_t al = a - d;
  const int lane = lane_id();
  // previous lane's output (lane 0: zeros, its chunk is written partially)
  const u32x4 p = {prev_lane(0u, o.x), prev_lane(0u, o.y), prev_lane(0u, o.z), prev_lane(0u, o.w)};
  // chunk = bytes [16 - d, 16) of p followed by bytes [0, 16 - d) of o
  const uint32_t D[8] = {p.x, p.y, p.z, p.w, o.x, o.y, o.z, o.w};
  const uint32_t s = 16 - d, r = s & 3u;
  u32x4 c;
  switch (__builtin_amdgcn_readfirstlane(s >> 2)) {
    case 0: c = funnel_q<0>(D, r); break;
    case 1: c = funnel_q<1>(D, r); break;
    case 2: c = funnel_q<2>(D, r); break;
    default: c = funnel_q<3>(D, r); break;
  }
  if (lane == 0) {
    st_bytes(c, al, d, 16);
  } else {
    st(c, al);
  }
  if (lane == 63) {  // head of chunk 64: bytes [16 - d, 16) of o
    const uint32_t E[8] = {o.x, o.y, o.z, o.w, 0u, 0u, 0u, 0u};
    u32x4 t;
    switch (__builtin_amdgcn_readfirstlane(s >> 2)) {
      case 0: t = funnel_q<0>(E, r); break;
      case 1: t = funnel_q<1>(E, r); break;
      case 2: t = funnel_q<2>(E, r); break;
      default: t = funnel_q<3>(E, r); break;
    }
    st_bytes(t, al + 16, 0, d);
  }
}

__global__ __launch_bounds__(256) void realign_store_copy(uint64_t src, uint64_t dst, uint64_t n16,
                                                          uint32_t mis) {
  const uint64_t gid = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (gid >= n16) return;
  st_realign(ld(src + gid * 16), dst + mis + gid * 16);
}

// Rows: row i of group g at base + (g * 16 + i) * rowlen; lane -> 16 B of the row.
// MODE 2: aligned loads issued together, then realigned; MODE 3: also
// realigned stores.
template <int MODE>
__global__ __launch_bounds__(256) void enc_mix2(uint64_t base, uint64_t rowlen, uint64_t total,
                                               uint32_t mr, uint32_t mw) {
  const uint64_t gid = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (gid >= total) return;
  const uint64_t chunks = (rowlen - 1024) / 16;
  const uint64_t g = gid / chunks, off = (gid - g * chunks) * 16;
  const uint64_t s0 = base + g * 16 * rowlen;
  const uint32_t d = mr & 15u;
  const int lane = lane_id();
  u32x4 c[12], e[12];
#pragma unroll
  for (int k = 0; k < 12; ++k) c[k] = ld(s0 + k * rowlen + off + mr - d);
#pragma unroll
  for (int k = 0; k < 12; ++k) {
    e[k] = u32x4{0, 0, 0, 0};
    if (lane == 63 && d) e[k] = ld(s0 + k * rowlen + off + mr - d + 16);
  }
  u32x4 acc[4] = {};
#pragma unroll
  for (int k = 0; k < 12; ++k) acc[k & 3] ^= d ? realign(c[k], e[k], d) : c[k];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if constexpr (MODE == 3) st_realign(acc[r], s0 + (12 + r) * rowlen + off + mw);
    else st(acc[r], s0 + (12 + r) * rowlen + off + mw);
  }
}

template <int MODE>
double run2(uint8_t* buf, uint64_t rowlen, uint64_t n, uint32_t mr, uint32_t mw) {
  const uint64_t chunks = (rowlen - 1024) / 16, total = chunks * n;
  const uint32_t nblk = static_cast<uint32_t>((total + 255) / 256);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 20; ++i) enc_mix2<MODE><<<nblk, 256>>>((uint64_t)buf, rowlen, total, mr, mw);
  CK(hipEventRecord(e0));
  const int reps = 20;
  for (int i = 0; i < reps; ++i) enc_mix2<MODE><<<nblk, 256>>>((uint64_t)buf, rowlen, total, mr, mw);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return static_cast<double>(total) * 16 * 16 * reps / (ms / 1e3) / 1e9;
}

template <bool DPP>
__global__ __launch_bounds__(256) void enc_mix(uint64_t base, uint64_t rowlen, uint64_t total,
                                              uint32_t mr, uint32_t mw) {
  const uint64_t gid = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (gid >= total) return;
  const uint64_t chunks = (rowlen - 1024) / 16;
  const uint64_t g = gid / chunks, off = (gid - g * chunks) * 16;
  const uint64_t s0 = base + g * 16 * rowlen;
  u32x4 acc[4] = {};
#pragma unroll
  for (int c = 0; c < 12; ++c) {
    const uint64_t a = s0 + c * rowlen + off + mr;
    acc[c & 3] ^= DPP ? ld_realign(a) : ld(a);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) st(acc[r], s0 + (12 + r) * rowlen + off + mw);
}

template <bool DPP>
double run(uint8_t* buf, uint64_t rowlen, uint64_t n, uint32_t mr, uint32_t mw) {
  const uint64_t chunks = (rowlen - 1024) / 16, total = chunks * n;
  const uint32_t nblk = static_cast<uint32_t>((total + 255) / 256);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 20; ++i) enc_mix<DPP><<<nblk, 256>>>((uint64_t)buf, rowlen, total, mr, mw);
  CK(hipEventRecord(e0));
  const int reps = 20;
  for (int i = 0; i < reps; ++i) enc_mix<DPP><<<nblk, 256>>>((uint64_t)buf, rowlen, total, mr, mw);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return static_cast<double>(total) * 16 * 16 * reps / (ms / 1e3) / 1e9;
}

int main() {
  // 1. correctness of the realignment
  {
    const uint64_t n16 = 1 << 16, bytes = n16 * 16 + 64;
    std::vector<uint8_t> h(bytes), g(n16 * 16);
    for (uint64_t i = 0; i < bytes; ++i) h[i] = static_cast<uint8_t>(i * 131 + (i >> 8) * 7 + 1);
    uint8_t *src, *dst;
    CK(hipMalloc(&src, bytes));
    CK(hipMalloc(&dst, n16 * 16));
    CK(hipMemcpy(src, h.data(), bytes, hipMemcpyHostToDevice));
    int bad = 0;
    const uint32_t mis[] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 34};
    for (uint32_t m : mis) {
      realign_copy<<<static_cast<unsigned>(n16 / 256), 256>>>((uint64_t)src, (uint64_t)dst, n16, m);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(g.data(), dst, n16 * 16, hipMemcpyDeviceToHost));
      const bool ok = std::memcmp(g.data(), h.data() + m, n16 * 16) == 0;
      bad += !ok;
      std::printf("{\"check\": \"realign\", \"mis\": %u, \"exact\": %s}\n", m, ok ? "true" : "false");
    }
    // realigned stores: copy an aligned buffer to dst + m; bytes outside untouched
    std::vector<uint8_t> z(bytes + 64, 0xEE), gz(bytes + 64);
    uint8_t* dz;
    CK(hipMalloc(&dz, bytes + 64));
    for (uint32_t m : mis) {
      CK(hipMemcpy(dz, z.data(), bytes + 64, hipMemcpyHostToDevice));
      realign_store_copy<<<static_cast<unsigned>(n16 / 256), 256>>>((uint64_t)src, (uint64_t)dz, n16, m);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(gz.data(), dz, bytes + 64, hipMemcpyDeviceToHost));
      std::vector<uint8_t> want(z);
      std::memcpy(want.data() + m, h.data(), n16 * 16);
      const bool ok = std::memcmp(gz.data(), want.data(), bytes + 64) == 0;
      bad += !ok;
      std::printf("{\"check\": \"realign_store\", \"mis\": %u, \"exact\": %s}\n", m,
                  ok ? "true" : "false");
    }
    CK(hipFree(dz));
    CK(hipFree(src));
    CK(hipFree(dst));
    if (bad) return 1;
  }
  // 2. timing
  const uint64_t rowlen = 64 << 10, n = (4ull << 30) / (16 * rowlen);
  uint8_t* buf;
  CK(hipMalloc(&buf, n * 16 * rowlen + 4096));
  CK(hipMemset(buf, 0x3c, n * 16 * rowlen + 4096));
  const uint32_t mis[][2] = {{0, 0}, {2, 0}, {0, 2}, {2, 2}, {6, 10}, {14, 14}, {18, 18}, {4, 4}};
  for (int rep = 0; rep < 3; ++rep)
    for (const auto& m : mis) {
      const double d = run<false>(buf, rowlen, n, m[0], m[1]);
      const double s = run<true>(buf, rowlen, n, m[0], m[1]);
      const double b = run2<2>(buf, rowlen, n, m[0], m[1]);
      const double w = run2<3>(buf, rowlen, n, m[0], m[1]);
      std::printf("{\"round\": %d, \"mis_read\": %u, \"mis_write\": %u, \"gbs_direct\": %.1f, "
                  "\"gbs_dpp\": %.1f, \"gbs_dpp_batched\": %.1f, \"gbs_dpp_rw\": %.1f}\n", rep, m[0],
                  m[1], d, s, b, w);
      std::fflush(stdout);
    }
  CK(hipFree(buf));
  return 0;
}
