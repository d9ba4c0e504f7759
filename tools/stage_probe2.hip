// stage_probe2.hip -- the 12+4 two-lost staged Reconst pattern WITH its GF
// arithmetic, in three shapes, to find what holds the product kernel at
// 0.73 of 8 TB/s at 1 MiB vects when the same memory pattern streams at 0.79
// (stage_probe.hip, profiles/r04_stage_probe.log):
//
//   ws<T>    : the product's wave-specialised shape (staged_ws_kernel): a-lanes
//              load the 12 a-rows, rebuild 2 lost a-halves (GF 12 x 2), form 3
//              retrieveRS XOR terms; b-lanes load the 14 b-rows; one LDS
//              hand-off; b-lanes XOR the terms into 3 rows, GF 12 x 2, store.
//              One block per CU at T = 512: nothing overlaps a block's GF work.
//   pipe<I>  : one lane role, I chunks per lane in a loop, phase-pipelined:
//              the b-row loads of chunk j are issued before stage 1 of chunk
//              j runs, the a-row loads of chunk j+1 before stage 3 of chunk j,
//              so each wave's GF work overlaps its own next loads.
//   pipe0<I> : pipe<I> without the GF work (XOR only): its memory ceiling.
//
// Bytes moved per stripe: 26 halves read, 7 written (2 a, 2 b, 3 write-backs).
// GB/s of moved bytes; the XOR/GF results are not checked (timing only; not
// part of the product).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/stage_probe2.hip -o tools/stage_probe2
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>

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

struct GfTab {
  uint32_t lo0, hi0, lo1, hi1, top;
};

__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t gmul(const GfTab& t, uint32_t x) {
  return x3(__builtin_amdgcn_perm(t.hi0, t.lo0, x & 0x07070707u),
            __builtin_amdgcn_perm(t.hi1, t.lo1, (x >> 3) & 0x07070707u),
            __builtin_amdgcn_perm(0u, t.top, (x >> 6) & 0x03030303u));
}
__device__ __forceinline__ void ld4(uint32_t* v, uint64_t a) {
  const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const gu32x4*>(a));
  v[0] = t.x, v[1] = t.y, v[2] = t.z, v[3] = t.w;
}
__device__ __forceinline__ void st4(const uint32_t* v, uint64_t a) {
  u32x4 t;
  t.x = v[0], t.y = v[1], t.z = v[2], t.w = v[3];
  __builtin_nontemporal_store(t, reinterpret_cast<gu32x4*>(a));
}

constexpr int NA = 12, NB = 14, NL = 2, NN = 2, NR = 3;
struct Args {
  GfTab at[NA][NL], bt[NA][NN];
  uint64_t arow[NA], brow[NB], adst[NL], bdst[NN];  // offsets inside a stripe
  uint64_t base, stripe, chunks, total;
  uint32_t k, nblk;
};

__device__ __forceinline__ uint64_t logical_block(uint32_t k, uint32_t nblk) {
  const uint32_t b = blockIdx.x;
  if (k == 0) return b;
  const uint32_t q = b >> 3, g = q / k;
  const uint64_t span = 8ull * k;
  if ((g + 1) * span > nblk) return b;
  return g * span + (b & 7u) * static_cast<uint64_t>(k) + (q - g * k);
}

// stage 1 + the XOR terms: al = at x xa, rx[r] = xa[r] ^ xa[r+3] ^ al[r & 1],
// seed[u] = xa[u + 6] ^ al[u]
template <bool GF>
__device__ __forceinline__ void stage_a(const Args& a, const uint32_t (&xa)[NA][4], uint32_t (&al)[NL][4],
                                        uint32_t (&rx)[NR][4], uint32_t (&seed)[NN][4]) {
#pragma unroll
  for (int w = 0; w < 4; ++w) {
#pragma unroll
    for (int q = 0; q < NL; ++q) {
      uint32_t v = 0;
#pragma unroll
      for (int m = 0; m < NA; ++m) v ^= GF ? gmul(a.at[m][q], xa[m][w]) : xa[m][w];
      al[q][w] = v;
    }
#pragma unroll
    for (int r = 0; r < NR; ++r) rx[r][w] = x3(xa[r][w], xa[r + 3][w], al[r & 1][w]);
#pragma unroll
    for (int u = 0; u < NN; ++u) seed[u][w] = xa[u + 6][w] ^ al[u][w];
  }
}

// retrieveRS on b-rows 11..13, then stage 3: ob = seed ^ bt x xb[0..12)
template <bool GF>
__device__ __forceinline__ void stage_b(const Args& a, uint32_t (&xb)[NB][4], const uint32_t (&rx)[NR][4],
                                        uint32_t (&ob)[NN][4]) {
#pragma unroll
  for (int w = 0; w < 4; ++w) {
#pragma unroll
    for (int r = 0; r < NR; ++r) xb[11 + r][w] ^= rx[r][w];
#pragma unroll
    for (int u = 0; u < NN; ++u) {
      uint32_t v = ob[u][w];
#pragma unroll
      for (int m = 0; m < NA; ++m) v ^= GF ? gmul(a.bt[m][u], xb[m][w]) : xb[m][w];
      ob[u][w] = v;
    }
  }
}

template <int T>
__global__ __launch_bounds__(2 * T) void ws_kernel(const Args a) {
  __shared__ uint4 xfer[NR + NN][T];
  const bool blane = threadIdx.x >= T;
  const uint32_t t = blane ? threadIdx.x - T : threadIdx.x;
  const uint64_t gid = logical_block(a.k, a.nblk) * T + t;
  if (gid >= a.total) return;  // (grids are whole blocks here)
  const uint64_t s = gid / a.chunks, sb = a.base + s * a.stripe + (gid - s * a.chunks) * 16;
  uint32_t xb[NB][4];
  if (!blane) {
    uint32_t xa[NA][4], al[NL][4], rx[NR][4], seed[NN][4];
#pragma unroll
    for (int m = 0; m < NA; ++m) ld4(xa[m], sb + a.arow[m]);
    stage_a<true>(a, xa, al, rx, seed);
#pragma unroll
    for (int r = 0; r < NR; ++r) xfer[r][t] = make_uint4(rx[r][0], rx[r][1], rx[r][2], rx[r][3]);
#pragma unroll
    for (int u = 0; u < NN; ++u) xfer[NR + u][t] = make_uint4(seed[u][0], seed[u][1], seed[u][2], seed[u][3]);
#pragma unroll
    for (int q = 0; q < NL; ++q) st4(al[q], sb + a.adst[q]);
  } else {
#pragma unroll
    for (int m = 0; m < NB; ++m) ld4(xb[m], sb + a.brow[m]);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  if (!blane) return;
  uint32_t rx[NR][4], ob[NN][4];
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const uint4 v = xfer[r][t];
    rx[r][0] = v.x, rx[r][1] = v.y, rx[r][2] = v.z, rx[r][3] = v.w;
  }
#pragma unroll
  for (int u = 0; u < NN; ++u) {
    const uint4 v = xfer[NR + u][t];
    ob[u][0] = v.x, ob[u][1] = v.y, ob[u][2] = v.z, ob[u][3] = v.w;
  }
  stage_b<true>(a, xb, rx, ob);
#pragma unroll
  for (int r = 0; r < NR; ++r) st4(xb[11 + r], sb + a.brow[11 + r]);
#pragma unroll
  for (int u = 0; u < NN; ++u) st4(ob[u], sb + a.bdst[u]);
}

// One lane role, I chunks per lane: wave w of the grid owns chunks
// [w * I * 64, (w + 1) * I * 64), lane l takes chunk base + j * 64 + l.
template <int I, bool GF>
__global__ __launch_bounds__(256) void pipe_kernel(const Args a) {
  const uint64_t wave = logical_block(a.k, a.nblk) * 4 + (threadIdx.x >> 6);
  const uint64_t c0 = wave * I * 64 + (threadIdx.x & 63);
  auto addr = [&](uint64_t c) {
    const uint64_t s = c / a.chunks;
    return a.base + s * a.stripe + (c - s * a.chunks) * 16;
  };
  uint32_t xa[NA][4], xb[NB][4];
  uint64_t sb = addr(c0);
#pragma unroll
  for (int m = 0; m < NA; ++m) ld4(xa[m], sb + a.arow[m]);
#pragma unroll 1
  for (int j = 0; j < I; ++j) {
#pragma unroll
    for (int m = 0; m < NB; ++m) ld4(xb[m], sb + a.brow[m]);
    uint32_t al[NL][4], rx[NR][4], ob[NN][4];
    stage_a<GF>(a, xa, al, rx, ob);
#pragma unroll
    for (int q = 0; q < NL; ++q) st4(al[q], sb + a.adst[q]);
    const uint64_t sn = j + 1 < I ? addr(c0 + (j + 1) * 64) : sb;
    if (j + 1 < I) {
#pragma unroll
      for (int m = 0; m < NA; ++m) ld4(xa[m], sn + a.arow[m]);
    }
    stage_b<GF>(a, xb, rx, ob);
#pragma unroll
    for (int r = 0; r < NR; ++r) st4(xb[11 + r], sb + a.brow[11 + r]);
#pragma unroll
    for (int u = 0; u < NN; ++u) st4(ob[u], sb + a.bdst[u]);
    sb = sn;
  }
}

int main(int argc, char** argv) {
  const uint64_t total_bytes = 4ull << 30;
  const int reps = argc > 1 ? std::atoi(argv[1]) : 20;
  const char* only = argc > 2 ? argv[2] : nullptr;
  uint8_t* buf = nullptr;
  CK(hipMalloc(&buf, total_bytes));
  CK(hipMemset(buf, 1, total_bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (uint64_t S : {uint64_t(4096), uint64_t(1) << 20}) {
    const uint64_t H = S / 2, n = total_bytes / (16 * S);
    Args a;
    std::memset(&a, 0, sizeof a);
    for (int m = 0; m < NA; ++m)
      for (int q = 0; q < 2; ++q) {
        const uint32_t v = 0x9E3779B9u * (m * 2 + q + 1);
        a.at[m][q] = {v, v ^ 0x01020304u, v * 3, v * 5, v & 0x7f7f7f7f};
        a.bt[m][q] = {v * 7, v ^ 0x0a0b0c0du, v * 11, v * 13, v & 0x3f3f3f3f};
      }
    for (int m = 0; m < NA; ++m) a.arow[m] = (2 + m) * S;          // a of shards 2..13
    for (int m = 0; m < NB; ++m) a.brow[m] = (2 + m) * S + H;      // b of shards 2..15
    a.adst[0] = 0, a.adst[1] = S, a.bdst[0] = H, a.bdst[1] = S + H;  // shards 0, 1
    a.base = reinterpret_cast<uint64_t>(buf);
    a.stripe = 16 * S;
    a.chunks = H / 16;
    a.total = a.chunks * n;
    struct Shape {
      const char* name;
      int kind;  // 0 ws, 1 pipe (GF), 2 pipe0 (XOR only)
      int t_or_i;
      uint32_t k;
    } shapes[] = {{"ws512_k128", 0, 512, 128}, {"ws512_k8", 0, 512, 8},    {"ws256_k128", 0, 256, 128},
                  {"ws256_k8", 0, 256, 8},     {"pipe2_k8", 1, 2, 8},      {"pipe4_k8", 1, 4, 8},
                  {"pipe8_k8", 1, 8, 8},       {"pipe4_k32", 1, 4, 32},    {"pipe8_k32", 1, 8, 32},
                  {"pipe16_k8", 1, 16, 8},     {"pipe4_plain", 1, 4, 0},   {"pipe0_4_k8", 2, 4, 8},
                  {"pipe0_8_k8", 2, 8, 8}};
    for (const Shape& sh : shapes) {
      char label[64];
      std::snprintf(label, sizeof label, "%s", sh.name);
      if (only && !std::strstr(label, only)) continue;
      uint64_t blocks;
      if (sh.kind == 0) {
        blocks = a.total / sh.t_or_i;
      } else {
        const uint64_t per_block = 4ull * sh.t_or_i * 64;  // chunks per 256-thread block
        if (a.total % per_block) continue;
        blocks = a.total / per_block;
      }
      a.nblk = static_cast<uint32_t>(blocks);
      a.k = sh.k;
      auto launch = [&] {
        if (sh.kind == 0) {
          if (sh.t_or_i == 512) ws_kernel<512><<<blocks, 1024>>>(a);
          else ws_kernel<256><<<blocks, 512>>>(a);
        } else {
          const bool gf = sh.kind == 1;
          switch (sh.t_or_i) {
            case 2: gf ? pipe_kernel<2, true><<<blocks, 256>>>(a) : pipe_kernel<2, false><<<blocks, 256>>>(a); break;
            case 4: gf ? pipe_kernel<4, true><<<blocks, 256>>>(a) : pipe_kernel<4, false><<<blocks, 256>>>(a); break;
            case 8: gf ? pipe_kernel<8, true><<<blocks, 256>>>(a) : pipe_kernel<8, false><<<blocks, 256>>>(a); break;
            default: gf ? pipe_kernel<16, true><<<blocks, 256>>>(a) : pipe_kernel<16, false><<<blocks, 256>>>(a); break;
          }
        }
      };
      for (int i = 0; i < 3; ++i) launch();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      for (int i = 0; i < reps; ++i) launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipGetLastError());
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double moved = 33.0 * H * n;
      const double gbs = moved / (ms / reps / 1e3) / 1e9;
      std::printf("S=%7llu %-14s %8.1f GB/s  %.3f of 8 TB/s  (%.3f ms)\n", (unsigned long long)S, label,
                  gbs, gbs / 8000.0, ms / reps);
      std::fflush(stdout);
    }
  }
  CK(hipFree(buf));
  return 0;
}
