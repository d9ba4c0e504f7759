// sync_bench.cpp -- per-stripe drop-in call cost (xrs_encode / xrs_reconst_one
// on host vects, like Go's x.Encode(vects)) and the batching queue
// (xrs_queue_*) with T concurrent caller threads.
//
//   g++ -O2 -std=c++17 -Iinclude tools/sync_bench.cpp -Lxrs_amd -lxrs_hip \
//       -Wl,-rpath,$PWD/xrs_amd -lpthread -o tools/sync_bench
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <thread>
#include <vector>

#include "xrs_hip.h"

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// CPU seconds used by the whole process (every caller thread plus the
// library's launcher and completion threads).
static double cpu_now() {
  timespec ts;
  clock_gettime(CLOCK_PROCESS_CPUTIME_ID, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

// A caller's vects: n buffers of `size` bytes, from ordinary (pageable)
// memory, or -- g_reg, the "...reg" modes -- from one xrs_host_alloc
// allocation the library knows as pinned and mapped, so the per-stripe calls
// skip the CPU copies through staging (the cgo shim's pinned buffer pool).
static bool g_reg = false;
static bool g_mixed = false;  // "queuemixed": odd caller threads registered, even ones plain
struct Bufs {
  std::vector<std::vector<uint8_t>> own;
  void* pinned = nullptr;
  std::vector<uint8_t*> p;
  Bufs(int n, size_t size, uint8_t fill, bool reg = g_reg) {
    const size_t stride = (size + 63) / 64 * 64;
    if (reg) {
      pinned = xrs_host_alloc(stride * n);
      if (!pinned) {
        std::printf("xrs_host_alloc failed\n");
        std::fflush(stdout);
        std::_Exit(4);
      }
      for (int i = 0; i < n; ++i) {
        p.push_back(static_cast<uint8_t*>(pinned) + i * stride);
        std::memset(p.back(), fill, size);
      }
    } else {
      own.assign(n, std::vector<uint8_t>(size, fill));
      for (auto& x : own) p.push_back(x.data());
    }
  }
  ~Bufs() {
    if (pinned) xrs_host_free(pinned);
  }
};

// `sync_bench ref`: every sub-benchmark of the reference's xrs_test.go
// (:471-680) as a per-stripe synchronous call on host vects, one thread, the
// way `go test -bench` runs it (one stripe, b.N calls), with its SetBytes.
static int ref_mode(xrs_codec* c) {
  constexpr int d = 12, p = 4;
  auto run = [](const char* name, size_t size, double bytes, auto&& call) {
    if (call()) std::exit(3);
    long n = 0;
    const double t0 = now();
    while (now() - t0 < 1.0) {
      if (call()) std::exit(3);
      ++n;
    }
    const double dt = (now() - t0) / n;
    std::printf("{\"bench\": \"%s\", \"vect_bytes\": %zu, \"ns_per_op\": %.0f, \"MB_s\": %.1f}\n",
                name, size, dt * 1e9, bytes / dt / 1e6);
    std::fflush(stdout);
  };
  auto vects = [](size_t size) {
    std::vector<std::vector<uint8_t>> v(d + p, std::vector<uint8_t>(size));
    uint32_t s = 0x5EED;
    for (int j = 0; j < d; ++j)
      for (auto& b : v[j]) b = static_cast<uint8_t>((s = s * 1664525u + 1013904223u) >> 24);
    return v;
  };
  char name[128];
  for (size_t size : {size_t(4) << 10, size_t(1) << 20, size_t(8) << 20}) {
    auto v = vects(size);
    std::vector<uint8_t*> ptr;
    for (auto& x : v) ptr.push_back(x.data());
    std::snprintf(name, sizeof name, "BenchmarkXRS_Encode/(12+4)-%s",
                  size < (1u << 20) ? "4KB" : size == (1u << 20) ? "1MB" : "8MB");
    run(name, size, double(d + p) * size, [&] { return xrs_encode(c, ptr.data(), d + p, size); });
  }
  const size_t size = 4096;
  auto v = vects(size);
  std::vector<uint8_t*> ptr;
  for (auto& x : v) ptr.push_back(x.data());
  if (xrs_encode(c, ptr.data(), d + p, size)) return 3;
  for (int i = 1; i <= p; ++i) {
    std::vector<int> lost, has;
    for (int j = 0; j < d + p; ++j) (j < i ? lost : has).push_back(j);
    const double bytes = i == 1 ? (d - 1 + 2 + 3) * size / 2.0 + size : double(d + i) * size;
    std::snprintf(name, sizeof name, "BenchmarkXRS_Reconst/(12+4)-4KB-reconst_%d_data_vects", i);
    run(name, size, bytes, [&] {
      return xrs_reconst(c, ptr.data(), d + p, size, has.data(), static_cast<int>(has.size()),
                         lost.data(), i);
    });
  }
  std::vector<uint8_t> nd(size, 0x5a);
  run("BenchmarkXRS_Update/(12+4)-4KB", size, double(2 * p + 2) * size,
      [&] { return xrs_update(c, ptr[5], nd.data(), size, 5, ptr.data() + d, p); });
  for (int n = 1; n <= d - p; ++n) {
    std::vector<int> rows;
    for (int j = 0; j < n; ++j) rows.push_back(j);
    std::snprintf(name, sizeof name, "BenchmarkXRS_Replace/(12+4)-4KB-replace_%d_data_vects", n);
    run(name, size, double(n + 2 * p) * size,
        [&] { return xrs_replace(c, ptr.data(), rows.data(), n, size, ptr.data() + d, p); });
  }
  return 0;
}

int main(int argc, char** argv) {
  const int seconds = 2;
  xrs_codec* c = nullptr;
  if (xrs_new(12, 4, &c)) return 2;
  if (argc > 1 && std::strcmp(argv[1], "ref") == 0) {
    const int rc = ref_mode(c);
    xrs_free(c);
    std::fflush(stdout);
    std::_Exit(rc);
  }
  // `sync_bench stress SECONDS THREADS`: liveness soak of the queue and the
  // shared codec.  Every thread loops over random ops for SECONDS: explicit
  // queue calls (Encode, ReconstOne, Update, Reconst of one loss pattern,
  // Replace of one rows set) on queues of two vect sizes, and the plain API
  // on the shared codec (auto queue) at three sizes; queues are created and
  // freed under load every second.  Even threads' vects are registered
  // (xrs_host_alloc: in-place sync calls, table-mode queue batches); thread 1
  // unregisters and re-registers its own buffer every 64 calls, so the
  // registry changes under the other callers' lookups.  Results are not
  // checked here (the GPU tests do that); any error or a call stuck 20 s is a
  // failure (exit 5 / 6, with the queue dump).
  if (argc > 1 && std::strcmp(argv[1], "stress") == 0) {
    const int secs = argc > 2 ? std::atoi(argv[2]) : 60;
    const int threads = argc > 3 ? std::atoi(argv[3]) : 32;
    const size_t sizes[3] = {4096, 1030, 65536};
    // explicit queues, replaced every second; a caller holds its slot's
    // shared lock for the call, so a queue is freed only once idle (the
    // Python tests cover xrs_queue_free with callers inside)
    std::atomic<xrs_queue*> qs[2];
    std::shared_mutex qmu[2];
    for (int i = 0; i < 2; ++i) {
      xrs_queue* q = nullptr;
      if (xrs_queue_new(c, sizes[i], 64, 50, &q)) return 4;
      qs[i] = q;
    }
    std::atomic<bool> stop{false};
    std::atomic<long> calls{0};
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t)
      th.emplace_back([&, t] {
        uint64_t r = 0x9E3779B97F4A7C15ull * (t + 1);
        auto rnd = [&] { r ^= r << 13; r ^= r >> 7; r ^= r << 17; return r; };
        constexpr size_t kVect = 65536;
        std::vector<std::vector<uint8_t>> v;
        std::vector<uint8_t> churn;
        uint8_t* reg = nullptr;
        std::vector<uint8_t*> p;
        if (t % 2 == 0 && (reg = static_cast<uint8_t*>(xrs_host_alloc(16 * kVect)))) {
          for (int j = 0; j < 16; ++j) p.push_back(reg + j * kVect);
        } else if (t == 1) {
          churn.assign(16 * kVect, static_cast<uint8_t>(t));
          for (int j = 0; j < 16; ++j) p.push_back(churn.data() + j * kVect);
        } else {
          v.assign(16, std::vector<uint8_t>(kVect, static_cast<uint8_t>(t)));
          for (auto& x : v) p.push_back(x.data());
        }
        bool churn_reg = false;
        long mine = 0;
        const int has[] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 14, 15}, need[] = {0, 13};
        const int rows[] = {3, 7};
        while (!stop.load(std::memory_order_relaxed)) {
          if (t == 1 && mine++ % 64 == 0) {  // flip the registration (no call in flight)
            const int e = churn_reg ? xrs_host_unregister(churn.data())
                                    : xrs_host_register(churn.data(), churn.size());
            if (e) {
              std::printf("STRESS FAIL: host (un)register rc %d\n", e);
              std::fflush(stdout);
              std::_Exit(5);
            }
            churn_reg = !churn_reg;
          }
          const int op = static_cast<int>(rnd() % 12);
          int rc = 0;
          if (op >= 10) {  // asynchronous: submit, poll, wait (the shared lock spans the ticket)
            const int qi = static_cast<int>(rnd() % 2);
            std::shared_lock<std::shared_mutex> g(qmu[qi]);
            xrs_queue* q = qs[qi].load();
            xrs_queue_ticket* tk = nullptr;
            rc = op == 10 ? xrs_queue_submit_encode(q, p.data(), 16, &tk)
                          : xrs_queue_submit_reconst_one(q, p.data(), 16, static_cast<int>(rnd() % 12), &tk);
            if (rc == XRS_ERR_BUSY) {
              rc = xrs_queue_encode(q, p.data(), 16);
            } else if (rc == 0) {
              for (int i = 0; i < 8 && xrs_queue_poll(tk) == 0; ++i) std::this_thread::yield();
              rc = xrs_queue_wait(tk);
            }
          } else if (op < 5) {  // explicit queue
            const int qi = static_cast<int>(rnd() % 2);
            std::shared_lock<std::shared_mutex> g(qmu[qi]);
            xrs_queue* q = qs[qi].load();
            switch (op) {
              case 0: rc = xrs_queue_encode(q, p.data(), 16); break;
              case 1: rc = xrs_queue_reconst_one(q, p.data(), 16, static_cast<int>(rnd() % 12)); break;
              case 2: rc = xrs_queue_update(q, p[1], p[2], static_cast<int>(rnd() % 12), p.data() + 12, 4); break;
              case 3: rc = xrs_queue_reconst(q, p.data(), 16, has, 14, need, 2); break;
              default: rc = xrs_queue_replace(q, p.data(), rows, 2, p.data() + 12, 4); break;
            }
          } else {  // the plain API on the shared codec
            const size_t sz = sizes[rnd() % 3];
            switch (op) {
              case 5: rc = xrs_encode(c, p.data(), 16, sz); break;
              case 6: rc = xrs_reconst_one(c, p.data(), 16, sz, static_cast<int>(rnd() % 12)); break;
              case 7: rc = xrs_update(c, p[1], p[2], sz, static_cast<int>(rnd() % 12), p.data() + 12, 4); break;
              case 8: rc = xrs_reconst(c, p.data(), 16, sz, has, 14, need, 2); break;
              default: rc = xrs_replace(c, p.data(), rows, 2, sz, p.data() + 12, 4); break;
            }
          }
          if (rc) {
            std::printf("STRESS FAIL: op %d rc %d\n", op, rc);
            std::fflush(stdout);
            std::_Exit(5);
          }
          ++calls;
        }
        if (churn_reg) (void)xrs_host_unregister(churn.data());
        if (reg) xrs_host_free(reg);
      });
    // every second: replace one explicit queue (xrs_queue_free under load),
    // and watch for progress
    const double t0 = now();
    long seen = 0;
    double t_seen = now();
    int gen = 0;
    while (now() - t0 < secs) {
      std::this_thread::sleep_for(std::chrono::milliseconds(250));
      const long n = calls.load();
      if (n != seen) {
        seen = n;
        t_seen = now();
      } else if (now() - t_seen > 20) {
        static char dump[8192];
        for (int i = 0; i < 2; ++i) {
          xrs_queue_dump(qs[i].load(), dump, sizeof dump);
          std::printf("HANG: no call finished for 20 s; queue %d:\n%s", i, dump);
        }
        std::fflush(stdout);
        std::_Exit(6);
      }
      if (gen % 40 == 39) {  // a progress line every 10 s
        std::printf("stress: %.0f s, %ld calls\n", now() - t0, calls.load());
        std::fflush(stdout);
      }
      if (++gen % 4 == 0) {
        const int i = (gen / 4) % 2;
        xrs_queue* fresh = nullptr;
        if (xrs_queue_new(c, sizes[i], 64, 50, &fresh)) return 4;
        xrs_queue* old;
        {
          std::unique_lock<std::shared_mutex> g(qmu[i]);
          old = qs[i].exchange(fresh);
        }
        xrs_queue_free(old);
      }
    }
    stop = true;
    for (auto& x : th) x.join();
    for (int i = 0; i < 2; ++i) xrs_queue_free(qs[i].load());
    xrs_free(c);
    std::printf("{\"stress_seconds\": %d, \"threads\": %d, \"calls\": %ld, \"queues_replaced\": %d}\n",
                secs, threads, calls.load(), gen / 4);
    std::fflush(stdout);
    std::_Exit(0);
  }
  const size_t size = argc > 1 ? std::strtoull(argv[1], nullptr, 0) : 4096;
  // `sync_bench SIZE syncmt [THREADS...]`: T threads calling the plain
  // per-stripe xrs_encode / xrs_update on ONE codec (the drop-in call
  // pattern; contended calls go through the codec's auto queue)
  // "...reg": the same on registered (xrs_host_alloc) vects
  if (argc > 2 && (std::strcmp(argv[2], "syncmtreg") == 0 || std::strcmp(argv[2], "queuereg") == 0 ||
                   std::strcmp(argv[2], "queueasyncreg") == 0)) {
    g_reg = true;
    argv[2][std::strlen(argv[2]) - 3] = 0;
  }
  if (argc > 2 && std::strcmp(argv[2], "syncmt") == 0) {
    std::vector<int> tl = {1, 8, 32};
    if (argc > 3) {
      tl.clear();
      for (int i = 3; i < argc; ++i) tl.push_back(std::atoi(argv[i]));
    }
    for (int upd = 0; upd < 2; ++upd)
      for (int threads : tl) {
        std::atomic<long> total{0};
        std::atomic<bool> stop{false};
        std::vector<std::thread> th;
        for (int t = 0; t < threads; ++t)
          th.emplace_back([&, t] {
            Bufs b(16, size, static_cast<uint8_t>(t));
            std::vector<uint8_t*>& p = b.p;
            long n = 0;
            while (!stop.load(std::memory_order_relaxed)) {
              const int rc = upd ? xrs_update(c, p[t % 12], p[(t + 1) % 12], size, t % 12, p.data() + 12, 4)
                                 : xrs_encode(c, p.data(), 16, size);
              if (rc) {
                std::printf("call failed: %d\n", rc);
                std::fflush(stdout);
                std::_Exit(5);
              }
              ++n;
            }
            total += n;
          });
        const double t0 = now(), c0 = cpu_now();
        std::this_thread::sleep_for(std::chrono::seconds(seconds));
        stop = true;
        for (auto& x : th) x.join();
        const double dt = now() - t0, cpu = cpu_now() - c0;
        const double gib = total * (upd ? 10.0 : 16.0) * size / (1 << 30);
        std::printf("{\"api\": \"%s (per-stripe, shared codec)\", \"vect_bytes\": %zu, \"threads\": %d, "
                    "\"registered\": %s, \"calls_per_s\": %.0f, \"gibps\": %.3f, \"cpu_cores\": %.2f, "
                    "\"cpu_seconds_per_gib\": %.3f}\n", upd ? "xrs_update" : "xrs_encode", size,
                    threads, g_reg ? "true" : "false", total / dt, gib / dt, cpu / dt,
                    gib > 0 ? cpu / gib : 0.0);
        std::fflush(stdout);
      }
    xrs_free(c);
    std::fflush(stdout);
    std::_Exit(0);
  }
  // `sync_bench SIZE queueasync WAIT_US WINDOW [THREADS...]`: T threads, each
  // keeping WINDOW Encode stripes in flight through xrs_queue_submit_encode /
  // xrs_queue_wait (one cgo call site with k stripes outstanding); a BUSY
  // submit waits on the thread's oldest ticket first.  "...reg": registered
  // vects.
  if (argc > 2 && std::strcmp(argv[2], "queuemixed") == 0) {  // then as "queue"
    g_mixed = true;
    argv[2][5] = 0;
  }
  if (argc > 2 && std::strcmp(argv[2], "queueasync") == 0) {
    const int wait_us = argc > 3 ? std::atoi(argv[3]) : 50;
    const int window = argc > 4 ? std::max(1, std::atoi(argv[4])) : 8;
    std::vector<int> tlist = {1, 8, 32};
    if (argc > 5) {
      tlist.clear();
      for (int i = 5; i < argc; ++i) tlist.push_back(std::atoi(argv[i]));
    }
    const char* mb = std::getenv("XRS_BENCH_MAX_BATCH");
    const size_t max_batch = mb && *mb ? std::strtoull(mb, nullptr, 0) : 1024;
    for (int threads : tlist) {
      xrs_queue* q = nullptr;
      if (int e = xrs_queue_new(c, size, max_batch, wait_us, &q)) {
        std::printf("xrs_queue_new failed: %d\n", e);
        std::fflush(stdout);
        return 4;
      }
      std::atomic<long> total{0}, busy{0};
      std::atomic<bool> stop{false};
      std::vector<std::thread> th;
      for (int t = 0; t < threads; ++t)
        th.emplace_back([&, t] {
          std::vector<std::unique_ptr<Bufs>> bufs;
          for (int w = 0; w < window; ++w) bufs.emplace_back(new Bufs(16, size, static_cast<uint8_t>(t + w)));
          std::vector<xrs_queue_ticket*> live(window, nullptr);  // ring, oldest at head
          int head = 0, n_live = 0;
          long n = 0, nb = 0;
          auto wait_oldest = [&] {
            if (int rc = xrs_queue_wait(live[head])) {
              std::printf("xrs_queue_wait failed: %d\n", rc);
              std::fflush(stdout);
              std::_Exit(5);
            }
            live[head] = nullptr;
            head = (head + 1) % window;
            --n_live;
            ++n;
          };
          while (!stop.load(std::memory_order_relaxed)) {
            if (n_live == window) wait_oldest();
            const int slot = (head + n_live) % window;
            xrs_queue_ticket* tk = nullptr;
            const int rc = xrs_queue_submit_encode(q, bufs[slot]->p.data(), 16, &tk);
            if (rc == XRS_ERR_BUSY) {  // wait on our oldest; with none, the blocking call
              ++nb;
              if (n_live) {
                wait_oldest();
              } else if (int rs = xrs_queue_encode(q, bufs[slot]->p.data(), 16)) {
                std::printf("xrs_queue_encode failed: %d\n", rs);
                std::fflush(stdout);
                std::_Exit(5);
              } else {
                ++n;
              }
              continue;
            }
            if (rc) {
              std::printf("xrs_queue_submit_encode failed: %d\n", rc);
              std::fflush(stdout);
              std::_Exit(5);
            }
            live[slot] = tk;
            ++n_live;
          }
          while (n_live) wait_oldest();
          total += n;
          busy += nb;
        });
      const double t0 = now(), c0 = cpu_now();
      std::this_thread::sleep_for(std::chrono::seconds(seconds));
      stop = true;
      for (auto& x : th) x.join();
      const double dt = now() - t0, cpu = cpu_now() - c0;
      const double gib = total * 16.0 * size / (1 << 30);
      uint64_t st[4] = {0, 0, 0, 0};
      xrs_queue_stats(q, st);
      const double nbt = st[0] ? static_cast<double>(st[0]) : 1.0;
      std::printf("{\"api\": \"xrs_queue_submit_encode + xrs_queue_wait\", \"vect_bytes\": %zu, "
                  "\"threads\": %d, \"window\": %d, \"registered\": %s, \"stripes_per_s\": %.0f, "
                  "\"gibps\": %.3f, \"batches\": %llu, \"stripes_per_batch\": %.1f, "
                  "\"run_us_per_batch\": %.1f, \"wait_us_per_batch\": %.1f, \"busy_returns\": %ld, "
                  "\"cpu_cores\": %.2f, \"cpu_seconds_per_gib\": %.3f}\n",
                  size, threads, window, g_reg ? "true" : "false", total / dt, gib / dt,
                  (unsigned long long)st[0], st[1] / nbt, st[2] / nbt / 1e3, st[3] / nbt / 1e3,
                  busy.load(), cpu / dt, gib > 0 ? cpu / gib : 0.0);
      std::fflush(stdout);
      xrs_queue_free(q);
    }
    xrs_free(c);
    std::fflush(stdout);
    std::_Exit(0);
  }
  // --- plain sync calls, one thread
  if (!(argc > 2 && std::strcmp(argv[2], "queue") == 0)) {
    std::vector<std::vector<uint8_t>> v(16, std::vector<uint8_t>(size, 1));
    std::vector<uint8_t*> p;
    for (auto& x : v) p.push_back(x.data());
    auto timeit = [&](const char* api, double bytes, auto&& call) {
      if (call()) std::exit(3);
      long n = 0;
      const double t0 = now();
      while (now() - t0 < seconds) {
        if (call()) std::exit(3);
        ++n;
      }
      const double dt = (now() - t0) / n;
      std::printf("{\"api\": \"%s\", \"vect_bytes\": %zu, \"threads\": 1, \"us_per_call\": %.1f, "
                  "\"gibps\": %.3f}\n", api, size, dt * 1e6, bytes / dt / (1 << 30));
      std::fflush(stdout);
    };
    timeit("xrs_encode", 16.0 * size, [&] { return xrs_encode(c, p.data(), 16, size); });
    timeit("xrs_reconst_one", 9.0 * size, [&] { return xrs_reconst_one(c, p.data(), 16, size, 0); });
    const int has[] = {2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, need[] = {0, 1};
    timeit("xrs_reconst_2", 14.0 * size,
           [&] { return xrs_reconst(c, p.data(), 16, size, has, 14, need, 2); });
    timeit("xrs_update", 10.0 * size,
           [&] { return xrs_update(c, p[0], p[1], size, 0, p.data() + 12, 4); });
  }
  if (argc > 2 && std::strcmp(argv[2], "sync") == 0) {
    xrs_free(c);
    std::fflush(stdout);
    std::_Exit(0);
  }
  // --- batching queue, T threads
  // `sync_bench SIZE queue [WAIT_US] [THREADS...]`: the queue only
  const bool qonly = argc > 2 && std::strcmp(argv[2], "queue") == 0;
  const int wait_us = qonly && argc > 3 ? std::atoi(argv[3]) : 50;
  std::vector<int> tlist = {1, 8, 32, 128};
  if (qonly && argc > 4) {
    tlist.clear();
    for (int i = 4; i < argc; ++i) tlist.push_back(std::atoi(argv[i]));
  }
  for (int upd = 0; upd < (qonly ? 1 : 2); ++upd)
  for (int threads : tlist) {
    xrs_queue* q = nullptr;
    if (int e = xrs_queue_new(c, size, 1024, wait_us, &q)) {
      std::printf("xrs_queue_new failed: %d\n", e);
      std::fflush(stdout);
      return 4;
    }
    std::atomic<long> total{0};
    std::atomic<bool> stop{false};
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t)
      th.emplace_back([&, t] {
        Bufs b(16, size, static_cast<uint8_t>(t), g_mixed ? (t % 2 == 1) : g_reg);
        std::vector<uint8_t*>& p = b.p;
        long n = 0;
        while (!stop.load(std::memory_order_relaxed)) {
          const int rc = upd ? xrs_queue_update(q, p[t % 12], p[(t + 1) % 12], t % 12, p.data() + 12, 4)
                             : xrs_queue_encode(q, p.data(), 16);
          if (rc) {
            std::printf("queue call failed: %d\n", rc);
            std::fflush(stdout);
            std::_Exit(5);
          }
          ++n;
        }
        total += n;
      });
    const double t0 = now(), c0 = cpu_now();
    std::this_thread::sleep_for(std::chrono::seconds(seconds));
    stop = true;
    // watchdog: callers that do not all return within 10 s are stuck
    std::atomic<bool> joined{false};
    std::thread wd([&] {
      for (int i = 0; i < 1000 && !joined.load(); ++i)
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
      if (joined.load()) return;
      uint64_t st[4] = {0, 0, 0, 0};
      xrs_queue_stats(q, st);
      std::printf("HANG: callers or xrs_queue_free stuck 10 s after stop (batches %llu, stripes %llu)\n",
                  (unsigned long long)st[0], (unsigned long long)st[1]);
      static char dump[8192];
      xrs_queue_dump(q, dump, sizeof dump);
      std::printf("%s", dump);
      std::fflush(stdout);
      std::_Exit(6);
    });
    for (auto& x : th) x.join();
    const double dt = now() - t0, cpu = cpu_now() - c0;
    const double gib = total * (upd ? 10.0 : 16.0) * size / (1 << 30);
    uint64_t st[4] = {0, 0, 0, 0};
    xrs_queue_stats(q, st);
    const double nb = st[0] ? static_cast<double>(st[0]) : 1.0;
    std::printf("{\"api\": \"%s\", \"vect_bytes\": %zu, \"threads\": %d, \"registered\": %s, "
                "\"stripes_per_s\": %.0f, \"gibps\": %.3f, \"batches\": %llu, "
                "\"stripes_per_batch\": %.1f, \"run_us_per_batch\": %.1f, "
                "\"wait_us_per_batch\": %.1f, \"cpu_cores\": %.2f, \"cpu_seconds_per_gib\": %.3f}\n",
                upd ? "xrs_queue_update" : "xrs_queue_encode",
                size, threads, g_mixed ? "\"half\"" : g_reg ? "true" : "false", total / dt, gib / dt, (unsigned long long)st[0], st[1] / nb,
                st[2] / nb / 1e3, st[3] / nb / 1e3, cpu / dt, gib > 0 ? cpu / gib : 0.0);
    std::fflush(stdout);
    if (std::getenv("XRS_QUEUE_DUMP")) {
      static char dump[8192];
      xrs_queue_dump(q, dump, sizeof dump);
      std::printf("%s", dump);
      std::fflush(stdout);
    }
    xrs_queue_free(q);
    joined = true;
    wd.join();
  }
  xrs_free(c);
  std::fflush(stdout);
  std::_Exit(0);
}
