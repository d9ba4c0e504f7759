// qlat_probe.hip -- where a small batching-queue batch spends its time: the
// launch call on the CPU, and launch to completion seen by a spinning
// hipStreamQuery, for an empty kernel and for xrs_encode_batched /
// xrs_reconst_one_batched on 12+4 4 KiB stripes in device memory and in
// pinned, device-mapped host memory (the queue's zero-copy staging).
//
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 -Iinclude tools/qlat_probe.hip \
//       -Lxrs_amd -lxrs_hip -Wl,-rpath,'$ORIGIN/../xrs_amd' -o tools/qlat_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#include "xrs_hip.h"

__global__ void empty_kernel() {}

// One lane writes `v` to a host-mapped word (system scope, vector store).
__global__ void flag_kernel(uint32_t* flag, uint32_t v) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// launch(v) enqueues work that ends by writing v to *flag; spin on the flag.
template <class F>
static void measure_flag(const char* name, volatile uint32_t* flag, F launch) {
  uint32_t v = *flag;
  for (int i = 0; i < 200; ++i) {
    if (int e = launch(++v)) {
      std::printf("%s: launch failed (%d)\n", name, e);
      std::fflush(stdout);
      return;
    }
    const double t0 = now_us();
    while (*flag != v) {
      if (now_us() - t0 > 1e6) {
        std::printf("%s: no completion after 1 s\n", name);
        std::fflush(stdout);
        std::_Exit(9);
      }
    }
  }
  const int reps = 3000;
  double api = 0, tot = 0;
  for (int i = 0; i < reps; ++i) {
    const double t0 = now_us();
    if (launch(++v)) std::abort();
    const double t1 = now_us();
    while (*flag != v) {
    }
    const double t2 = now_us();
    api += t1 - t0;
    tot += t2 - t0;
  }
  std::printf("%-44s launch call %6.2f us   launch->flag %6.2f us\n", name, api / reps, tot / reps);
  std::fflush(stdout);
}

template <class F>
static void measure(const char* name, hipStream_t s, F launch) {
  for (int i = 0; i < 200; ++i) {
    if (launch()) std::abort();
    while (hipStreamQuery(s) == hipErrorNotReady) {
    }
  }
  const int reps = 3000;
  double api = 0, tot = 0;
  for (int i = 0; i < reps; ++i) {
    const double t0 = now_us();
    if (launch()) std::abort();
    const double t1 = now_us();
    while (hipStreamQuery(s) == hipErrorNotReady) {
    }
    const double t2 = now_us();
    api += t1 - t0;
    tot += t2 - t0;
  }
  std::printf("%-44s launch call %6.2f us   launch->done %6.2f us\n", name, api / reps, tot / reps);
  std::fflush(stdout);
}

int main() {
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
  xrs_codec* c = nullptr;
  if (xrs_new(12, 4, &c)) return 2;
  const size_t size = 4096, stripe = 16 * size, maxn = 64;
  uint8_t* dev = nullptr;
  if (hipMalloc(&dev, maxn * stripe) != hipSuccess) return 3;
  uint8_t* host = static_cast<uint8_t*>(xrs_host_alloc(maxn * stripe));
  if (!host) return 4;
  std::memset(host, 7, maxn * stripe);
  (void)hipMemset(dev, 7, maxn * stripe);
  uint8_t* hdev = static_cast<uint8_t*>(xrs_host_device_pointer(host));
  (void)hipDeviceSynchronize();

  measure("empty kernel", s, [&] {
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
    return 0;
  });
  for (size_t n : {size_t(1), size_t(8), size_t(16), size_t(32), size_t(64)}) {
    char nm[96];
    std::snprintf(nm, sizeof nm, "encode %zu x 4 KiB, device memory", n);
    measure(nm, s, [&] { return xrs_encode_batched(c, dev, size, size, stripe, n, s); });
    std::snprintf(nm, sizeof nm, "encode %zu x 4 KiB, mapped host memory", n);
    measure(nm, s, [&] { return xrs_encode_batched(c, hdev, size, size, stripe, n, s); });
  }
  uint32_t* flag_h = static_cast<uint32_t*>(xrs_host_alloc(4096));
  *flag_h = 0;
  uint32_t* flag_d = static_cast<uint32_t*>(xrs_host_device_pointer(flag_h));
  hipEvent_t ev;
  (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  measure("empty kernel, hipEventQuery spin", s, [&] {
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
    return static_cast<int>(hipEventRecord(ev, s));
  });
  measure_flag("flag kernel alone", flag_h, [&](uint32_t v) {
    hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, s, flag_d, v);
    return 0;
  });
  measure_flag("hipStreamWriteValue32 alone", flag_h, [&](uint32_t v) {
    return static_cast<int>(hipStreamWriteValue32(s, flag_d, v, 0));
  });
  for (size_t n : {size_t(1), size_t(8), size_t(32)}) {
    char nm[96];
    std::snprintf(nm, sizeof nm, "encode %zu mapped + flag kernel", n);
    measure_flag(nm, flag_h, [&](uint32_t v) {
      if (int e = xrs_encode_batched(c, hdev, size, size, stripe, n, s)) return e;
      hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, s, flag_d, v);
      return 0;
    });
    std::snprintf(nm, sizeof nm, "encode %zu mapped + hipStreamWriteValue32", n);
    measure_flag(nm, flag_h, [&](uint32_t v) {
      if (int e = xrs_encode_batched(c, hdev, size, size, stripe, n, s)) return e;
      return static_cast<int>(hipStreamWriteValue32(s, flag_d, v, 0));
    });
  }
  // A sync call's shape: gather 48 KiB of inputs (CPU memcpy into the mapped
  // staging), launch, completion word.  "launch first": the kernel is
  // enqueued behind hipStreamWaitValue32 on a signal word before the gather,
  // and the host releases it after the copy, so launch and copy overlap.
  {
    std::vector<uint8_t> src(12 * size, 9);
    uint32_t* sig = nullptr;
    const bool have_sig = hipExtMallocWithFlags(reinterpret_cast<void**>(&sig), 64, hipMallocSignalMemory) == hipSuccess;
    measure_flag("copy 48 KiB, then encode 1 + flag", flag_h, [&](uint32_t v) {
      std::memcpy(host, src.data(), src.size());
      if (int e = xrs_encode_batched(c, hdev, size, size, stripe, 1, s)) return e;
      return static_cast<int>(hipStreamWriteValue32(s, flag_d, v, 0));
    });
    if (have_sig) {
      volatile uint32_t* vs = sig;
      *vs = 0;
      uint32_t gate = 0;
      measure_flag("wait-value, encode 1 + flag, then copy", flag_h, [&](uint32_t v) {
        ++gate;
        if (hipStreamWaitValue32(s, sig, gate, hipStreamWaitValueGte, 0xffffffffu) != hipSuccess) return 7;
        if (int e = xrs_encode_batched(c, hdev, size, size, stripe, 1, s)) return e;
        if (hipStreamWriteValue32(s, flag_d, v, 0) != hipSuccess) return 8;
        std::memcpy(host, src.data(), src.size());
        __atomic_store_n(const_cast<uint32_t*>(vs), gate, __ATOMIC_RELEASE);
        return 0;
      });
    } else {
      std::printf("hipMallocSignalMemory unavailable; trying a pinned host word\n");
      std::fflush(stdout);
      volatile uint32_t* vs = flag_h + 16;  // same pinned page, another line
      *vs = 0;
      uint32_t gate = 0;
      measure_flag("wait-value (pinned word), encode 1 + flag, then copy", flag_h, [&](uint32_t v) {
        ++gate;
        if (hipStreamWaitValue32(s, flag_d + 16, gate, hipStreamWaitValueGte, 0xffffffffu) != hipSuccess)
          return 7;
        if (int e = xrs_encode_batched(c, hdev, size, size, stripe, 1, s)) return e;
        if (hipStreamWriteValue32(s, flag_d, v, 0) != hipSuccess) return 8;
        std::memcpy(host, src.data(), src.size());
        __atomic_store_n(const_cast<uint32_t*>(vs), gate, __ATOMIC_RELEASE);
        return 0;
      });
    }
  }
  for (size_t n : {size_t(1), size_t(16)}) {
    char nm[96];
    std::snprintf(nm, sizeof nm, "reconst_one %zu x 4 KiB, mapped host memory", n);
    measure(nm, s, [&] { return xrs_reconst_one_batched(c, hdev, size, size, stripe, n, 3, s); });
  }
  xrs_host_free(host);
  (void)hipFree(dev);
  xrs_free(c);
  return 0;
}
