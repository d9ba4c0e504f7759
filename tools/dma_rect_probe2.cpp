// dma_rect_probe2.cpp -- large rectangles: which (width, pitch, rows) the
// runtime's hipMemcpy2DAsync accepts and copies exactly with 4-byte aligned
// bases, pinned + mapped host memory (as the queue's staging) and pageable.
// Prints the HIP status of each copy (no exit on error).
//   g++ -O2 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include tools/dma_rect_probe2.cpp \
//       -L/opt/rocm/lib -lamdhip64 -o tools/dma_rect_probe2
#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

int main() {
  const size_t cap = size_t(80) << 20;
  uint8_t *pinned = nullptr, *dev = nullptr;
  if (hipHostMalloc(reinterpret_cast<void**>(&pinned), cap, hipHostMallocMapped) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&dev), cap) != hipSuccess) {
    std::printf("alloc failed\n");
    return 1;
  }
  std::vector<uint8_t> pageable(cap), back(cap);
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  struct C { size_t width, pitch, rows, off; };
  std::vector<C> cases;
  for (size_t pitch : {size_t(16777248), size_t(16777216), size_t(1) << 22, size_t(1) << 20,
                       size_t(65536 + 32), size_t(1) << 18, (size_t(1) << 18) + 4})
    for (size_t width : {size_t(12582939), size_t(12582936), size_t(3145731), size_t(1048578),
                         size_t(1048581), size_t(262147), size_t(65539), size_t(16387), size_t(4099)})
      for (size_t rows : {size_t(1), size_t(3)})
        if (width <= pitch && (rows - 1) * pitch + width + 16 <= cap) cases.push_back({width, pitch, rows, 12});
  for (int kind = 0; kind < 2; ++kind) {
    uint8_t* host = kind ? pageable.data() : pinned;
    for (const C& c : cases)
      for (int dir = 0; dir < 2; ++dir) {
        const size_t span = (c.rows - 1) * c.pitch + c.width + c.off;
        for (size_t i = 0; i < span; i += 4093) host[i] = static_cast<uint8_t>(i * 7 + dir);
        hipError_t e;
        auto t0 = std::chrono::steady_clock::now();
        if (dir == 0) {
          e = hipMemcpy2DAsync(dev + c.off, c.pitch, host + c.off, c.pitch, c.width, c.rows,
                               hipMemcpyHostToDevice, s);
        } else {
          (void)hipMemcpy(dev, host, span, hipMemcpyHostToDevice);
          e = hipMemcpy2DAsync(back.data() + c.off, c.pitch, dev + c.off, c.pitch, c.width, c.rows,
                               hipMemcpyDeviceToHost, s);
        }
        const hipError_t e2 = hipStreamSynchronize(s);
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        bool ok = e == hipSuccess && e2 == hipSuccess;
        if (ok && dir == 0) {
          (void)hipMemcpy(back.data(), dev, span, hipMemcpyDeviceToHost);
        }
        if (ok)
          for (size_t r = 0; r < c.rows && ok; ++r)
            ok = !std::memcmp(back.data() + c.off + r * c.pitch, host + c.off + r * c.pitch, c.width);
        std::printf("%s %s width=%zu pitch=%zu rows=%zu: copy=%d sync=%d %s %.0f us\n",
                    kind ? "pageable" : "pinned-mapped", dir ? "D2H" : "H2D", c.width, c.pitch, c.rows,
                    static_cast<int>(e), static_cast<int>(e2), ok ? "exact" : "FAIL", us);
        std::fflush(stdout);
        (void)hipGetLastError();
      }
  }
  std::printf("done\n");
  return 0;
}
