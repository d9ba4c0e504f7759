// alignprobe.hip -- what does a row that is not 128-B aligned cost, and where?
// Streams with Encode's mix (12 rows read, 4 written, 16 B per lane, XOR in
// place of the GF arithmetic) over rows whose base is misaligned by `mr`
// (reads) / `mw` (writes) bytes, in two load shapes:
//   direct: every lane loads its own 16 B at the misaligned address (what the
//           product kernels do today: a wave's 1 KiB touches 9 lines);
//   split : the wave loads the line-aligned 1 KiB that starts at or below its
//           first byte, plus one extra 16-B load on the lanes that cover the
//           spill-over into the next line; cross-lane realignment is modelled
//           by ds_bpermute (4 per 16 B, 8 when mr is not a multiple of 16).
// Timing only (the XOR result is not checked); not part of the product.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/alignprobe.hip -o tools/alignprobe
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

__device__ __forceinline__ u32x4 ld(uint64_t a) {
  return __builtin_nontemporal_load(reinterpret_cast<const gu32x4*>(a));
}
__device__ __forceinline__ void st(u32x4 v, uint64_t a) {
  __builtin_nontemporal_store(v, reinterpret_cast<gu32x4*>(a));
}
__device__ __forceinline__ uint32_t bperm(uint32_t v, int lane) {
  return static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(lane << 2, static_cast<int>(v)));
}
// 16 B of the aligned stream starting `s` chunks after this lane (s wave-uniform):
// this lane's chunk for lanes >= s, the extra chunk of lane t for t < s.
__device__ __forceinline__ u32x4 shift_in(u32x4 c, u32x4 e, int s) {
  const int l = threadIdx.x & 63, t = (l + s) & 63;
  const u32x4 v = l >= s ? c : e;  // what this lane sources (uniform rule)
  u32x4 r;
  r.x = bperm(v.x, t);
  r.y = bperm(v.y, t);
  r.z = bperm(v.z, t);
  r.w = bperm(v.w, t);
  return r;
}

// Rows: row i of "stripe" g at base + (g * 16 + i) * rowlen, rowlen = 64 KiB
// (aligned) -- the misalignment is added per access.  Lane -> 16 B of the
// row; one wave = 1 KiB of one row.
template <bool SPLIT>
__global__ __launch_bounds__(256) void enc_mix(uint64_t base, uint64_t rowlen, uint64_t total,
                                              uint32_t mr, uint32_t mw) {
  const uint64_t gid = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (gid >= total) return;
  const uint64_t chunks = (rowlen - 1024) / 16;  // whole waves; room for the misalignment
  const uint64_t g = gid / chunks, off = (gid - g * chunks) * 16;
  const uint64_t s0 = base + g * 16 * rowlen;
  u32x4 acc[4] = {};
  if constexpr (!SPLIT) {
#pragma unroll
    for (int c = 0; c < 12; ++c) acc[c & 3] ^= ld(s0 + c * rowlen + off + mr);
  } else {
    // wave-aligned: the wave's lanes load [off0 + 16 l) of the aligned stream
    const int s = static_cast<int>(mr >> 4), l = threadIdx.x & 63;
    u32x4 c[12], e[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) {
      c[k] = ld(s0 + k * rowlen + off);
      e[k] = u32x4{0, 0, 0, 0};
      if (l < s) e[k] = ld(s0 + k * rowlen + off + 1024);
    }
#pragma unroll
    for (int k = 0; k < 12; ++k) {
      u32x4 v = shift_in(c[k], e[k], s);
      if (mr & 15) v ^= shift_in(c[k], e[k], s + 1);  // the byte-funnel partner
      acc[k & 3] ^= v;
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) st(acc[r], s0 + (12 + r) * rowlen + off + mw);
}

template <bool SPLIT>
double run(uint8_t* buf, uint64_t rowlen, uint64_t n, uint32_t mr, uint32_t mw) {
  const uint64_t chunks = (rowlen - 1024) / 16, total = chunks * n;
  const uint32_t nblk = static_cast<uint32_t>((total + 255) / 256);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 20; ++i) enc_mix<SPLIT><<<nblk, 256>>>((uint64_t)buf, rowlen, total, mr, mw);
  CK(hipEventRecord(e0));
  const int reps = 20;
  for (int i = 0; i < reps; ++i) enc_mix<SPLIT><<<nblk, 256>>>((uint64_t)buf, rowlen, total, mr, mw);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return static_cast<double>(total) * 16 * 16 * reps / (ms / 1e3) / 1e9;
}

int main() {
  const uint64_t rowlen = 64 << 10, n = (4ull << 30) / (16 * rowlen);
  uint8_t* buf;
  CK(hipMalloc(&buf, n * 16 * rowlen + 4096));
  CK(hipMemset(buf, 0x3c, n * 16 * rowlen + 4096));
  const uint32_t mis[][2] = {{0, 0}, {16, 0}, {0, 16}, {16, 16}, {64, 64}, {2, 2}, {2, 0}, {0, 2}, {34, 34}};
  for (int rep = 0; rep < 2; ++rep)
    for (const auto& m : mis) {
      const double d = run<false>(buf, rowlen, n, m[0], m[1]);
      const double s = run<true>(buf, rowlen, n, m[0], m[1]);
      std::printf("{\"round\": %d, \"mis_read\": %u, \"mis_write\": %u, \"gbs_direct\": %.1f, "
                  "\"gbs_split\": %.1f}\n", rep, m[0], m[1], d, s);
      std::fflush(stdout);
    }
  CK(hipFree(buf));
  return 0;
}
