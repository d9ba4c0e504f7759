// hostreg_test.cpp -- CPU test of the registered-range table
// (xrs_amd/csrc/hostreg.cpp, compiled alone: no HIP): lookups at range edges,
// replacement, and readers racing a writer that registers and unregisters,
// with every replaced table freed by the writer once no reader can hold it (a
// two-generation grace period; a writer waits for a view held across it).  Built twice, under
// ThreadSanitizer and under AddressSanitizer (tests/test_cpp.py).
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "hostreg.h"

using xrs_detail::HostRangesView;

#define CHECK(c)                                                  \
  do {                                                            \
    if (!(c)) {                                                   \
      std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);   \
      std::exit(1);                                               \
    }                                                             \
  } while (0)

static uint64_t dev_of(const void* p, size_t n) {
  const HostRangesView v;
  return v.device(p, n);
}

int main(int argc, char** argv) {
  const int replacements = argc > 1 ? std::atoi(argv[1]) : 20000;
  static char a[4096], b[4096];
  CHECK(dev_of(a, 1) == 0);
  xrs_detail::host_ranges_add(a, sizeof a, reinterpret_cast<void*>(0x100000));
  xrs_detail::host_ranges_add(b, 1024, reinterpret_cast<void*>(0x900000));
  CHECK(dev_of(a, 4096) == 0x100000);
  CHECK(dev_of(a + 100, 10) == 0x100000 + 100);
  CHECK(dev_of(a + 4090, 7) == 0);  // runs past the end
  CHECK(dev_of(a - 1, 1) == 0);  // below a (b's registered part is < 4 KiB long)
  CHECK(dev_of(b + 1000, 24) == 0x900000 + 1000);
  CHECK(dev_of(b + 1000, 25) == 0);
  xrs_detail::host_ranges_add(b, 2048, reinterpret_cast<void*>(0xA00000));  // re-register: replaced
  CHECK(dev_of(b + 2000, 48) == 0xA00000 + 2000);
  xrs_detail::host_ranges_remove(a);
  CHECK(dev_of(a, 1) == 0);
  CHECK(dev_of(b, 1) == 0xA00000);
  xrs_detail::host_ranges_remove(a);  // absent: no-op
  CHECK(xrs_detail::host_ranges_retired() == 0);  // no reader: freed at once

  // a view held across a replacement: the writer waits for it, and the view's
  // table stays readable until it is dropped (ASan: no use after free)
  {
    std::atomic<bool> wrote{false};
    std::thread w;
    {
      const HostRangesView held;
      w = std::thread([&] {
        xrs_detail::host_ranges_add(a, 8, reinterpret_cast<void*>(0x300000));
        wrote = true;
      });
      std::this_thread::sleep_for(std::chrono::milliseconds(50));
      CHECK(!wrote.load());                      // blocked on the held view
      CHECK(held.device(b + 4, 4) == 0xA00000 + 4);  // the old table, intact
      CHECK(held.device(a, 1) == 0);             // a was removed in that table
    }
    w.join();
    CHECK(wrote.load() && dev_of(a, 8) == 0x300000);
    xrs_detail::host_ranges_remove(a);
  }

  // readers race a writer flipping 64 ranges; a reader must always see either
  // nothing or the right address for a flipping range, and b throughout
  static char pool[64][256];
  std::atomic<bool> stop{false};
  std::atomic<long> lookups{0};
  std::vector<std::thread> th;
  for (int t = 0; t < 8; ++t)
    th.emplace_back([&, t] {
      unsigned r = 12345u * (t + 1);
      while (!stop.load(std::memory_order_relaxed)) {
        const HostRangesView v;
        for (int k = 0; k < 16; ++k) {
          r = r * 1664525u + 1013904223u;
          const int i = (r >> 8) % 64;
          const uint64_t d = v.device(pool[i] + 8, 16);
          CHECK(d == 0 || d == 0x10000000ull * (i + 1) + 8);
          CHECK(v.device(b + 8, 8) == 0xA00000 + 8);
        }
        lookups.fetch_add(16, std::memory_order_relaxed);
      }
    });
  for (int round = 0; round < replacements; ++round) {
    const int i = round % 64;
    if ((round / 64) % 2 == 0)
      xrs_detail::host_ranges_add(pool[i], sizeof pool[i], reinterpret_cast<void*>(0x10000000ull * (i + 1)));
    else
      xrs_detail::host_ranges_remove(pool[i]);
    CHECK(xrs_detail::host_ranges_retired() == 0);  // freed by the writer, under load
  }
  stop = true;
  for (auto& x : th) x.join();
  xrs_detail::host_ranges_add(a, 16, reinterpret_cast<void*>(0x100000));
  CHECK(xrs_detail::host_ranges_retired() == 0);
  std::printf("PASS hostreg: %ld lookups against %d replacements\n", lookups.load(), replacements);
  return 0;
}
