// unaligned_probe.hip -- are byte-misaligned global_load/store_dwordx4 exact
// on MI355X (the runtime's unaligned access mode), and what do they cost?
// Copies n bytes src+so -> dst+do with 16 B per lane (nontemporal, like the
// product kernels), checks the bytes on the host, and times 1 GiB copies at
// several (so, do).  Every index is bounded by n; buffers carry 64 B slack.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 gu32x4;

__global__ __launch_bounds__(256) void copy16(const uint8_t* src, uint8_t* dst, uint64_t n16) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n16) return;
  const u32x4 v = __builtin_nontemporal_load(
      reinterpret_cast<const gu32x4*>(reinterpret_cast<uint64_t>(src) + i * 16));
  __builtin_nontemporal_store(v, reinterpret_cast<gu32x4*>(reinterpret_cast<uint64_t>(dst) + i * 16));
}

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      std::exit(1);                                                         \
    }                                                                       \
  } while (0)

int main() {
  const uint64_t small = 1 << 20, big = 1ull << 30;
  uint8_t *src, *dst;
  CK(hipMalloc(&src, big + 64));
  CK(hipMalloc(&dst, big + 64));
  std::vector<uint8_t> h(small + 64), g(small + 64);
  for (size_t i = 0; i < h.size(); ++i) h[i] = static_cast<uint8_t>(i * 131 + 7);
  CK(hipMemcpy(src, h.data(), h.size(), hipMemcpyHostToDevice));
  const int offs[][2] = {{0, 0}, {1, 0}, {0, 1}, {3, 5}, {4, 8}, {8, 4}, {15, 1}};
  for (auto& o : offs) {
    CK(hipMemset(dst, 0, small + 64));
    const uint64_t n16 = small / 16;
    copy16<<<(n16 + 255) / 256, 256>>>(src + o[0], dst + o[1], n16);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(g.data(), dst, g.size(), hipMemcpyDeviceToHost));
    const bool ok = std::memcmp(g.data() + o[1], h.data() + o[0], small) == 0;
    std::printf("{\"check\": \"src+%d -> dst+%d\", \"exact\": %s}\n", o[0], o[1], ok ? "true" : "false");
  }
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (auto& o : offs) {
    const uint64_t n16 = big / 16;
    for (int w = 0; w < 20; ++w) copy16<<<(n16 + 255) / 256, 256>>>(src + o[0], dst + o[1], n16);
    CK(hipEventRecord(a));
    for (int r = 0; r < 10; ++r) copy16<<<(n16 + 255) / 256, 256>>>(src + o[0], dst + o[1], n16);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    std::printf("{\"copy\": \"src+%d -> dst+%d\", \"gbs\": %.1f}\n", o[0], o[1],
                2.0 * big * 10 / (ms / 1e3) / 1e9);
  }
  CK(hipFree(src));
  CK(hipFree(dst));
  return 0;
}
