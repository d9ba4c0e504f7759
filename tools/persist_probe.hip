// persist_probe.hip -- round trip of a persistent polling kernel against the
// launch-per-batch path, for the batching queue's small zero-copy batches.
//
// A grid of G workgroups stays resident and polls a request counter in
// pinned host memory.  Request s asks for n "stripes": every stripe reads
// 12 x 4 KiB and writes 4 x 4 KiB of pinned host memory (the 12+4 Encode
// traffic, XOR in place of the GF arithmetic); stripe j goes to workgroup
// j mod G.  Each workgroup, after its stripes, releases its stores at system
// scope and counts itself done; the last one writes s to a host word the
// host spins on.  Every wave leaves the loop when the host sets `stop`, or
// after ~2 s without a new request (wall clock), so the grid always drains.
//
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/persist_probe.hip -o tools/persist_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>

struct Ctl {
  uint32_t head;  // host -> device: requests posted
  uint32_t stop;  // host -> device: leave the loop
  uint32_t n;     // stripes of the current request
  uint32_t pad0[13];
  uint32_t done;  // device -> host: last request completed
  uint32_t pad1[15];
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int kBS = 256;
constexpr size_t kS = 4096, kStripe = 16 * kS;

__device__ __forceinline__ uint32_t ld_sys(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(kBS) void persist(Ctl* ctl, uint8_t* base, uint32_t* count,
                                               uint64_t timeout_ticks) {
  __shared__ uint32_t s_head, s_stop, s_n;
  const uint32_t G = gridDim.x;
  uint32_t seen = 0;
  uint64_t t_last = wall_clock64();
  for (;;) {
    if (threadIdx.x == 0) {
      s_head = __hip_atomic_load(&ctl->head, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
      s_stop = ld_sys(&ctl->stop);
      s_n = ld_sys(&ctl->n);
    }
    __syncthreads();
    const uint32_t head = s_head, stop = s_stop, n = s_n;
    __syncthreads();
    if (stop) break;
    if (head == seen) {
      if (wall_clock64() - t_last > timeout_ticks) break;
      __builtin_amdgcn_s_sleep(2);
      continue;
    }
    seen = head;  // (one request at a time in this probe)
    t_last = wall_clock64();
    // stripes j = blockIdx.x, +G, ...: 4 KiB vects, 16 B per lane per half row
    for (uint32_t j = blockIdx.x; j < n; j += G) {
      const uint8_t* st = base + size_t(j) * kStripe;
      for (uint32_t o = threadIdx.x * 16; o < kS; o += kBS * 16) {
        u32x4 acc[4] = {};
        for (int c = 0; c < 12; ++c) {
          const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(st + c * kS + o));
          for (int r = 0; r < 4; ++r) {
            acc[r].x ^= v.x + r;
            acc[r].y ^= v.y;
            acc[r].z ^= v.z;
            acc[r].w ^= v.w;
          }
        }
        for (int r = 0; r < 4; ++r)
          __builtin_nontemporal_store(acc[r], reinterpret_cast<u32x4*>(
                                                  const_cast<uint8_t*>(st) + (12 + r) * kS + o));
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      // this workgroup's stores reach host memory before it counts itself
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      // monotonic: request `head` is complete when the count reaches head * G
      const uint32_t old = __hip_atomic_fetch_add(count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      if (old + 1 == head * G)
        __hip_atomic_store(&ctl->done, head, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// The launch-per-request reference: the same stripes in one grid of n blocks.
__global__ __launch_bounds__(kBS) void once(uint8_t* base, uint32_t n) {
  const uint32_t j = blockIdx.x;
  const uint8_t* st = base + size_t(j) * kStripe;
  for (uint32_t o = threadIdx.x * 16; o < kS; o += kBS * 16) {
    u32x4 acc[4] = {};
    for (int c = 0; c < 12; ++c) {
      const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(st + c * kS + o));
      for (int r = 0; r < 4; ++r) {
        acc[r].x ^= v.x + r;
        acc[r].y ^= v.y;
        acc[r].z ^= v.z;
        acc[r].w ^= v.w;
      }
    }
    for (int r = 0; r < 4; ++r)
      __builtin_nontemporal_store(acc[r], reinterpret_cast<u32x4*>(
                                              const_cast<uint8_t*>(st) + (12 + r) * kS + o));
  }
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

__global__ void tiny_kernel() {}

// Does work on other streams run while the resident kernel sits on stream
// `es`?  (Streams share the process's hardware queues beyond
// GPU_MAX_HW_QUEUES; a kernel queued behind a resident one on the same
// hardware queue waits for it to leave.)
static void blocking_check(const char* name, hipStream_t es, Ctl* ctl, Ctl* ctl_d, uint8_t* host_d,
                           uint32_t* count, hipStream_t* others, int n_others) {
  volatile Ctl* vc = ctl;
  vc->stop = 0;
  vc->head = 0;
  vc->done = 0;
  (void)hipMemset(count, 0, 4);
  (void)hipDeviceSynchronize();
  hipLaunchKernelGGL(persist, dim3(8), dim3(kBS), 0, es, ctl_d, host_d, count, uint64_t(200000000));
  // the resident kernel answers a request: it is running
  __atomic_store_n(&ctl->head, 1u, __ATOMIC_RELEASE);
  vc->n = 1;
  const double t0 = now_us();
  while (vc->done != 1 && now_us() - t0 < 1e6) {
  }
  int blocked = 0;
  for (int i = 0; i < n_others; ++i) hipLaunchKernelGGL(tiny_kernel, dim3(1), dim3(64), 0, others[i]);
  const double t1 = now_us();
  for (int i = 0; i < n_others; ++i) {
    while (hipStreamQuery(others[i]) == hipErrorNotReady && now_us() - t1 < 200000) {
    }
    if (hipStreamQuery(others[i]) == hipErrorNotReady) ++blocked;
  }
  vc->stop = 1;
  (void)hipStreamSynchronize(es);
  for (int i = 0; i < n_others; ++i) (void)hipStreamSynchronize(others[i]);
  std::printf("%-44s resident answered: %s; %d of %d other streams blocked for 200 ms\n", name,
              vc->done == 1 ? "yes" : "NO", blocked, n_others);
  std::fflush(stdout);
}

int main(int argc, char** argv) {
  Ctl* ctl = nullptr;
  uint8_t* host = nullptr;
  uint32_t* count = nullptr;
  const uint32_t maxn = 64;
  if (hipHostMalloc(&ctl, sizeof(Ctl), hipHostMallocMapped) != hipSuccess) return 1;
  if (hipHostMalloc(&host, maxn * kStripe, hipHostMallocMapped) != hipSuccess) return 1;
  if (hipMalloc(&count, 4) != hipSuccess || hipMemset(count, 0, 4) != hipSuccess) return 1;
  std::memset(ctl, 0, sizeof(Ctl));
  std::memset(host, 3, maxn * kStripe);
  Ctl* ctl_d;
  uint8_t* host_d;
  (void)hipHostGetDevicePointer(reinterpret_cast<void**>(&ctl_d), ctl, 0);
  (void)hipHostGetDevicePointer(reinterpret_cast<void**>(&host_d), host, 0);
  hipStream_t s, s2;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  volatile Ctl* vc = ctl;

  if (argc > 1 && std::strcmp(argv[1], "block") == 0) {
    hipStream_t others[8];
    for (auto& o : others) (void)hipStreamCreateWithFlags(&o, hipStreamNonBlocking);
    hipStream_t e1, e2, e3, e4;
    (void)hipStreamCreateWithFlags(&e1, hipStreamNonBlocking);
    blocking_check("ordinary stream (created after 8 others)", e1, ctl, ctl_d, host_d, count, others, 8);
    int lo = 0, hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
    (void)hipStreamCreateWithPriority(&e2, hipStreamNonBlocking, hi);
    blocking_check("greatest-priority stream", e2, ctl, ctl_d, host_d, count, others, 8);
    uint32_t all[8] = {~0u, ~0u, ~0u, ~0u, ~0u, ~0u, ~0u, ~0u};
    (void)hipExtStreamCreateWithCUMask(&e3, 8, all);
    blocking_check("CU-mask stream (all CUs)", e3, ctl, ctl_d, host_d, count, others, 8);
    uint32_t some[8] = {0x01010101u, 0x01010101u, 0, 0, 0, 0, 0, 0};
    (void)hipExtStreamCreateWithCUMask(&e4, 8, some);
    blocking_check("CU-mask stream (8 CUs)", e4, ctl, ctl_d, host_d, count, others, 8);
    return 0;
  }

  for (uint32_t G : {8u, 32u, 64u}) {
    vc->stop = 0;
    vc->head = 0;
    vc->done = 0;
    (void)hipMemset(count, 0, 4);
    (void)hipDeviceSynchronize();
    hipLaunchKernelGGL(persist, dim3(G), dim3(kBS), 0, s, ctl_d, host_d, count,
                       uint64_t(200000000));  // 2 s at 100 MHz
    uint32_t seq = 0;
    for (uint32_t n : {1u, 8u, 16u, 32u, 64u}) {
      vc->n = n;
      const int reps = 3000;
      double tot = 0;
      for (int i = 0; i < reps + 100; ++i) {
        const double t0 = now_us();
        __atomic_store_n(&ctl->head, ++seq, __ATOMIC_RELEASE);
        while (vc->done != seq) {
          if (now_us() - t0 > 1e6) {
            std::printf("persistent G=%u n=%u: request %u not done after 1 s\n", G, n, seq);
            vc->stop = 1;
            (void)hipStreamSynchronize(s);
            return 3;
          }
        }
        if (i >= 100) tot += now_us() - t0;
      }
      std::printf("persistent G=%2u  n=%2u stripes: post->done %6.2f us\n", G, n, tot / reps);
      std::fflush(stdout);
    }
    vc->stop = 1;
    if (hipStreamSynchronize(s) != hipSuccess) return 2;
  }
  for (uint32_t n : {1u, 8u, 16u, 32u, 64u}) {
    const int reps = 3000;
    double tot = 0;
    for (int i = 0; i < reps + 100; ++i) {
      const double t0 = now_us();
      hipLaunchKernelGGL(once, dim3(n), dim3(kBS), 0, s2, host_d, n);
      while (hipStreamQuery(s2) == hipErrorNotReady) {
      }
      if (i >= 100) tot += now_us() - t0;
    }
    std::printf("launch per request   n=%2u stripes: launch->done %6.2f us\n", n, tot / reps);
    std::fflush(stdout);
  }
  (void)hipHostFree(host);
  (void)hipHostFree(ctl);
  (void)hipFree(count);
  return 0;
}
