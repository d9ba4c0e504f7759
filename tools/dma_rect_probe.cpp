// dma_rect_probe.cpp -- which hipMemcpy2DAsync / hipMemcpyAsync shapes the
// runtime's DMA engine path refuses ("DMA buffer failed
// with code 4097" on odd-size host-pipeline copies).  For each case it prints
// a marker line on stderr, so that AMD_LOG_LEVEL=1's runtime lines that follow
// belong to it, then times the copy and checks its bytes.
//
//   g++ -O2 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include tools/dma_rect_probe.cpp \
//       -L/opt/rocm/lib -lamdhip64 -o tools/dma_rect_probe
//   AMD_LOG_LEVEL=1 tools/dma_rect_probe 2>&1 | tee gpurun_out/dma_rect_probe.log
#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

int main() {
  const size_t rows = 1024, cap = rows * 8192 + 64;
  uint8_t *pinned = nullptr, *dev = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void**>(&pinned), cap, hipHostMallocDefault));
  CK(hipMalloc(reinterpret_cast<void**>(&dev), cap));
  std::vector<uint8_t> pageable(cap), check(cap);
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  struct Case {
    size_t hoff, hpitch, width, doff, dpitch;
  };
  std::vector<Case> cases;
  // host offset, host pitch, width, device offset, device pitch
  for (size_t hoff : {0, 1, 2})
    for (size_t hpitch : {8192, 8194})
      for (size_t width : {4096, 4098, 4097})
        for (size_t doff : {0, 2}) cases.push_back({hoff, hpitch, width, doff, 8192});
  cases.push_back({0, 8192, 4096, 0, 8196});
  cases.push_back({0, 8192, 4096, 0, 8194});
  for (int kind = 0; kind < 2; ++kind) {
    uint8_t* host = kind ? pageable.data() : pinned;
    for (const Case& c : cases) {
      for (int dir = 0; dir < 2; ++dir) {
        for (size_t i = 0; i < cap; ++i) host[i] = static_cast<uint8_t>(i * 131 + 7 + dir);
        CK(hipMemsetAsync(dev, 0, cap, s));
        CK(hipStreamSynchronize(s));
        std::fprintf(stderr, "CASE %s %s hoff=%zu hpitch=%zu width=%zu doff=%zu dpitch=%zu\n",
                     kind ? "pageable" : "pinned", dir ? "D2H" : "H2D", c.hoff, c.hpitch, c.width,
                     c.doff, c.dpitch);
        std::fflush(stderr);
        double us = 0;
        if (dir == 0) {
          auto t0 = std::chrono::steady_clock::now();
          CK(hipMemcpy2DAsync(dev + c.doff, c.dpitch, host + c.hoff, c.hpitch, c.width, rows,
                              hipMemcpyHostToDevice, s));
          CK(hipStreamSynchronize(s));
          us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
          CK(hipMemcpy(check.data(), dev, cap, hipMemcpyDeviceToHost));
          bool ok = true;
          for (size_t r = 0; r < rows && ok; ++r)
            ok = !std::memcmp(check.data() + c.doff + r * c.dpitch, host + c.hoff + r * c.hpitch, c.width);
          std::printf("%s H2D hoff=%zu hpitch=%zu width=%zu doff=%zu dpitch=%zu: %s %.1f us %.2f GB/s\n",
                      kind ? "pageable" : "pinned", c.hoff, c.hpitch, c.width, c.doff, c.dpitch,
                      ok ? "exact" : "WRONG", us, rows * c.width / us / 1e3);
        } else {
          // device holds a pattern; copy its rows out into a zeroed host area
          for (size_t i = 0; i < cap; ++i) check[i] = static_cast<uint8_t>(i * 17 + 3);
          CK(hipMemcpy(dev, check.data(), cap, hipMemcpyHostToDevice));
          std::memset(host, 0, cap);
          auto t0 = std::chrono::steady_clock::now();
          CK(hipMemcpy2DAsync(host + c.hoff, c.hpitch, dev + c.doff, c.dpitch, c.width, rows,
                              hipMemcpyDeviceToHost, s));
          CK(hipStreamSynchronize(s));
          us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
          bool ok = true;
          for (size_t r = 0; r < rows && ok; ++r) {
            ok = !std::memcmp(host + c.hoff + r * c.hpitch, check.data() + c.doff + r * c.dpitch, c.width);
            // nothing outside the rows written
            const size_t end = c.hoff + r * c.hpitch + c.width;
            if (ok && r + 1 < rows)
              for (size_t i = end; i < c.hoff + (r + 1) * c.hpitch; ++i) ok = ok && host[i] == 0;
          }
          std::printf("%s D2H hoff=%zu hpitch=%zu width=%zu doff=%zu dpitch=%zu: %s %.1f us %.2f GB/s\n",
                      kind ? "pageable" : "pinned", c.hoff, c.hpitch, c.width, c.doff, c.dpitch,
                      ok ? "exact" : "WRONG", us, rows * c.width / us / 1e3);
        }
        std::fflush(stdout);
      }
    }
  }
  // 1-D copies at odd offsets and sizes
  for (int kind = 0; kind < 2; ++kind) {
    uint8_t* host = kind ? pageable.data() : pinned;
    for (size_t off : {0, 1, 2})
      for (size_t n : {size_t(4098), size_t(4097), size_t(1) << 20, (size_t(1) << 20) + 2}) {
        std::fprintf(stderr, "CASE1D %s off=%zu n=%zu\n", kind ? "pageable" : "pinned", off, n);
        std::fflush(stderr);
        for (size_t i = 0; i < n; ++i) host[off + i] = static_cast<uint8_t>(i * 29 + off);
        CK(hipMemcpyAsync(dev + off, host + off, n, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));  // (pinned: the DMA reads host memory later)
        std::memset(host, 0, n + 8);
        CK(hipMemcpyAsync(host + off, dev + off, n, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        bool ok = true;
        for (size_t i = 0; i < n && ok; ++i) ok = host[off + i] == static_cast<uint8_t>(i * 29 + off);
        std::printf("%s 1D off=%zu n=%zu: %s\n", kind ? "pageable" : "pinned", off, n, ok ? "exact" : "WRONG");
        std::fflush(stdout);
      }
  }
  CK(hipHostFree(pinned));
  CK(hipFree(dev));
  std::printf("done\n");
  return 0;
}
