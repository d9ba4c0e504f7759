// stage_probe.hip -- memory-pattern probe behind the staged Reconst gap
// (VERDICT r3 item 1): why does 2-lost Reconst at 1 MiB vects move bytes at
// 0.72-0.75 of 8 TB/s when the same kernel reaches 0.79 at 4-64 KiB and
// Encode 0.78 at 1 MiB?  Pure streaming with XOR in place of the GF
// arithmetic, over a 12+4 batch (shard stride S, stripe stride 16 S), one
// 16-B chunk of each half-row per lane, every load first:
//
//   encode    : a+b halves of shards 0..11 read, a+b of 12..15 written (32)
//   enc_rmw   : the same reads, the 8 writes go to halves of shards 0..3
//               (written rows were read in the same pass: Update/Replace-like)
//   staged    : 2-lost Reconst at 12+4 (lost 0, 1): a of 2..13 + b of 2..15
//               read (26), a+b of 0, 1 written plus b of 13, 14, 15 written
//               back in place (retrieveRS): 33 halves
//   staged_sc : as staged, the 3 write-backs to a scratch batch instead
//   staged_nowb: as staged without the 3 write-backs (30 halves)
//   read26    : staged's 26 reads only
//
// Each pattern in two block shapes: "one" = one lane role (all loads, XOR,
// stores), "ws" = staged_ws_kernel's split (a-lanes read the a-rows, b-lanes
// the b-rows, one LDS barrier; only for the staged patterns).
// GB/s = halves moved x H / time.  Timing only; not part of the product.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/stage_probe.hip -o tools/stage_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

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

constexpr int kMaxR = 32, kMaxW = 8;
struct Pat {
  uint64_t rd[kMaxR];  // byte offset of the half-row inside a stripe
  uint64_t wr[kMaxW];
  uint32_t wbuf;       // bit w: write w goes to the scratch batch
  int na;              // ws: the first na reads are the a-lanes'
};

struct Args {
  Pat p;
  uint64_t base, scratch, stripe, half, chunks, total;
  uint32_t k;  // XCD block order: logical blocks per XCD per group (0: plain)
  uint32_t nblk;
};

__device__ __forceinline__ uint64_t logical_block(uint32_t k, uint32_t nblk) {
  const uint32_t b = blockIdx.x;
  if (k == 0) return b;
  const uint32_t q = b >> 3, g = q / k;
  const uint64_t span = 8ull * k;
  if ((g + 1) * span > nblk) return b;
  return g * span + (b & 7u) * static_cast<uint64_t>(k) + (q - g * k);
}

template <int NR, int NW, int BS>
__global__ __launch_bounds__(BS) void one_kernel(const Args a) {
  const uint64_t gid = logical_block(a.k, a.nblk) * BS + threadIdx.x;
  if (gid >= a.total) return;
  const uint64_t s = gid / a.chunks, off = (gid - s * a.chunks) * 16;
  const uint64_t sb = a.base + s * a.stripe + off, ss = a.scratch + s * a.stripe + off;
  u32x4 x[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r) x[r] = ld(sb + a.p.rd[r]);
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    u32x4 v = x[w % NR];
#pragma unroll
    for (int r = w + 1; r < NR; r += 3) v ^= x[r];
    st(v, ((a.p.wbuf >> w) & 1u ? ss : sb) + a.p.wr[w]);
  }
  if constexpr (NW == 0) {  // keep the loads alive (never true for the fill pattern)
    u32x4 v = x[0];
#pragma unroll
    for (int r = 1; r < NR; ++r) v ^= x[r];
    if (v.x == 0xdeadbeefu) st(v, ss);
  }
}

// staged_ws_kernel's shape: a-lanes read rd[0, NA) and write wr[0, NWA), the
// b-lanes read rd[NA, NR) and, after one LDS hand-off, write wr[NWA, NW).
template <int NA, int NR, int NWA, int NW, int T>
__global__ __launch_bounds__(2 * T) void ws_kernel(const Args a) {
  __shared__ u32x4 xfer[4][T];
  const bool blane = threadIdx.x >= T;
  const uint32_t t = blane ? threadIdx.x - T : threadIdx.x;
  const uint64_t gid = logical_block(a.k, a.nblk) * T + t;
  const bool valid = gid < a.total;
  const uint64_t s = gid / a.chunks, off = (gid - s * a.chunks) * 16;
  const uint64_t sb = a.base + s * a.stripe + off, ss = a.scratch + s * a.stripe + off;
  u32x4 xb[NR - NA];
  if (!blane) {
    if (valid) {
      u32x4 x[NA];
#pragma unroll
      for (int r = 0; r < NA; ++r) x[r] = ld(sb + a.p.rd[r]);
      u32x4 acc[4] = {};
#pragma unroll
      for (int r = 0; r < NA; ++r) acc[r & 3] ^= x[r];
#pragma unroll
      for (int q = 0; q < 4; ++q) xfer[q][t] = acc[q] ^ x[q];
#pragma unroll
      for (int w = 0; w < NWA; ++w) st(acc[w & 3], ((a.p.wbuf >> w) & 1u ? ss : sb) + a.p.wr[w]);
    }
  } else if (valid) {
#pragma unroll
    for (int r = NA; r < NR; ++r) xb[r - NA] = ld(sb + a.p.rd[r]);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  if (!blane || !valid) return;
  u32x4 acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = xfer[q][t];
#pragma unroll
  for (int r = 0; r < NR - NA; ++r) acc[r & 3] ^= xb[r];
#pragma unroll
  for (int w = NWA; w < NW; ++w) st(acc[w & 3], ((a.p.wbuf >> w) & 1u ? ss : sb) + a.p.wr[w]);
  if constexpr (NW == NWA) {  // keep the loads alive (never true for the fill pattern)
    const u32x4 v = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
    if (v.x == 0xdeadbeefu) st(v, ss);
  }
}

int main(int argc, char** argv) {
  const uint64_t total_bytes = 4ull << 30;
  const int reps = argc > 1 ? std::atoi(argv[1]) : 20;
  const char* only = argc > 2 ? argv[2] : nullptr;
  uint8_t *buf = nullptr, *scr = nullptr;
  CK(hipMalloc(&buf, total_bytes));
  CK(hipMalloc(&scr, total_bytes));
  CK(hipMemset(buf, 1, total_bytes));
  CK(hipMemset(scr, 2, total_bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const bool sweep = argc > 3 && std::strcmp(argv[3], "sweep") == 0;
  if (sweep) {
    // staged pattern only: wave-specialised shape, T = 256 / 512 x block order K
    for (uint64_t S : {uint64_t(1) << 20, uint64_t(256) << 10, uint64_t(4096)}) {
      const uint64_t H = S / 2, stripe = 16 * S, n = total_bytes / stripe;
      Args a;
      std::memset(&a, 0, sizeof a);
      for (int i = 2; i < 14; ++i) a.p.rd[i - 2] = uint64_t(i) * S;
      for (int i = 2; i < 16; ++i) a.p.rd[12 + i - 2] = uint64_t(i) * S + H;
      const uint64_t wr[7] = {0, S, H, S + H, 13 * S + H, 14 * S + H, 15 * S + H};
      for (int w = 0; w < 7; ++w) a.p.wr[w] = wr[w];
      a.base = reinterpret_cast<uint64_t>(buf);
      a.scratch = reinterpret_cast<uint64_t>(scr);
      a.stripe = stripe;
      a.half = H;
      a.chunks = H / 16;
      a.total = a.chunks * n;
      for (int T : {256, 512}) {
        const uint64_t blocks = a.total / T;
        for (uint32_t k : {0u, 1u, 2u, 4u, 8u, 16u, 32u, 64u, 128u, 256u}) {
          a.nblk = static_cast<uint32_t>(blocks);
          a.k = k;
          auto launch = [&] {
            if (T == 256) ws_kernel<12, 26, 2, 7, 256><<<blocks, 512>>>(a);
            else ws_kernel<12, 26, 2, 7, 512><<<blocks, 1024>>>(a);
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
          const double gbs = 33.0 * H * n / (ms / reps / 1e3) / 1e9;
          std::printf("sweep S=%7llu ws%d k=%3u  %8.1f GB/s  %.3f of 8 TB/s\n", (unsigned long long)S, T, k,
                      gbs, gbs / 8000.0);
          std::fflush(stdout);
        }
      }
    }
    return 0;
  }
  for (uint64_t S : {uint64_t(4096), uint64_t(65536), uint64_t(1) << 20}) {
    const uint64_t H = S / 2, stripe = 16 * S, n = total_bytes / stripe;
    auto A = [&](int shard) { return uint64_t(shard) * S; };
    auto B = [&](int shard) { return uint64_t(shard) * S + H; };
    struct Case {
      std::string name;
      std::vector<uint64_t> rd, wr;
      uint32_t wbuf;
      int na, nwa;
    };
    std::vector<Case> cases;
    {
      Case c{"encode", {}, {}, 0, 0, 0};
      for (int i = 0; i < 12; ++i) c.rd.push_back(A(i)), c.rd.push_back(B(i));
      for (int i = 12; i < 16; ++i) c.wr.push_back(A(i)), c.wr.push_back(B(i));
      cases.push_back(c);
      Case r = c;
      r.name = "enc_rmw";
      r.wr.clear();
      for (int i = 0; i < 4; ++i) r.wr.push_back(A(i)), r.wr.push_back(B(i));
      cases.push_back(r);
    }
    {
      Case c{"staged", {}, {}, 0, 12, 2};
      for (int i = 2; i < 14; ++i) c.rd.push_back(A(i));
      for (int i = 2; i < 16; ++i) c.rd.push_back(B(i));
      c.wr = {A(0), A(1), B(0), B(1), B(13), B(14), B(15)};
      cases.push_back(c);
      Case sc = c;
      sc.name = "staged_sc";
      sc.wbuf = (1u << 4) | (1u << 5) | (1u << 6);
      cases.push_back(sc);
      Case nw = c;
      nw.name = "staged_nowb";
      nw.wr = {A(0), A(1), B(0), B(1)};
      cases.push_back(nw);
      Case rd = c;
      rd.name = "read26";
      rd.wr.clear();
      cases.push_back(rd);
    }
    for (const Case& c : cases) {
      for (int shape = 0; shape < 4; ++shape) {
        // 0: one-role 256-thread blocks, XCD order k = 8; 1: same, plain
        // order; 2: ws T = 256; 3: ws T = 512 (staged patterns only)
        const bool ws = shape >= 2;
        if (ws && c.name.rfind("staged", 0) != 0) continue;
        char label[96];
        std::snprintf(label, sizeof label, "%s/%s", c.name.c_str(),
                      shape == 0 ? "one_xcd" : shape == 1 ? "one_plain" : shape == 2 ? "ws256" : "ws512");
        if (only && !std::strstr(label, only)) continue;
        Args a;
        std::memset(&a, 0, sizeof a);
        for (size_t i = 0; i < c.rd.size(); ++i) a.p.rd[i] = c.rd[i];
        for (size_t i = 0; i < c.wr.size(); ++i) a.p.wr[i] = c.wr[i];
        a.p.wbuf = c.wbuf;
        a.p.na = c.na;
        a.base = reinterpret_cast<uint64_t>(buf);
        a.scratch = reinterpret_cast<uint64_t>(scr);
        a.stripe = stripe;
        a.half = H;
        a.chunks = H / 16;
        a.total = a.chunks * n;
        const int T = shape == 3 ? 512 : 256;
        const uint64_t blocks = (a.total + T - 1) / T;
        a.nblk = static_cast<uint32_t>(blocks);
        a.k = shape == 1 ? 0 : 8;
        auto launch = [&] {
          const int nr = static_cast<int>(c.rd.size()), nw = static_cast<int>(c.wr.size());
          if (!ws) {
            if (nr == 24 && nw == 8) one_kernel<24, 8, 256><<<blocks, 256>>>(a);
            else if (nr == 26 && nw == 7) one_kernel<26, 7, 256><<<blocks, 256>>>(a);
            else if (nr == 26 && nw == 4) one_kernel<26, 4, 256><<<blocks, 256>>>(a);
            else if (nr == 26 && nw == 0) one_kernel<26, 0, 256><<<blocks, 256>>>(a);
          } else if (T == 256) {
            if (nw == 7) ws_kernel<12, 26, 2, 7, 256><<<blocks, 512>>>(a);
            else if (nw == 4) ws_kernel<12, 26, 2, 4, 256><<<blocks, 512>>>(a);
            else ws_kernel<12, 26, 0, 0, 256><<<blocks, 512>>>(a);
          } else {
            if (nw == 7) ws_kernel<12, 26, 2, 7, 512><<<blocks, 1024>>>(a);
            else if (nw == 4) ws_kernel<12, 26, 2, 4, 512><<<blocks, 1024>>>(a);
            else ws_kernel<12, 26, 0, 0, 512><<<blocks, 1024>>>(a);
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
        const double moved = double(c.rd.size() + c.wr.size()) * H * n;
        const double gbs = moved / (ms / reps / 1e3) / 1e9;
        std::printf("S=%7llu %-22s halves r%zu w%zu  %8.1f GB/s  %.3f of 8 TB/s  (%.3f ms)\n",
                    (unsigned long long)S, label, c.rd.size(), c.wr.size(), gbs, gbs / 8000.0,
                    ms / reps);
        std::fflush(stdout);
      }
    }
  }
  CK(hipFree(buf));
  CK(hipFree(scr));
  return 0;
}
