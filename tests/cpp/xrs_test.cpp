// xrs_test.cpp -- the reference's test file (/root/reference/xrs_test.go)
// ported to C++ over include/xrs.hpp (the C++ mirror of the Go method set).
// Fixed seeds instead of the reference's clock seeds (xrs_test.go:26-31).
//
//   xrs_test --cpu   host-logic tests only (no GPU needed)
//   xrs_test         all tests (needs the MI355X)
//   xrs_test NAME..  only the named tests
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <random>
#include <string>
#include <thread>

#include <hip/hip_runtime_api.h>

#include "xrs.hpp"

using xrs::Error;
using xrs::Vect;
using xrs::Vects;
using xrs::XRS;

static int g_fail = 0;
#if defined(__has_feature)
#if __has_feature(address_sanitizer)
#define XRS_TEST_ASAN 1
#endif
#endif
#if defined(__SANITIZE_ADDRESS__) || defined(XRS_TEST_ASAN)
static constexpr bool kAsanBuild = true;
#else
static constexpr bool kAsanBuild = false;
#endif
#define FATAL(...)                          \
  do {                                      \
    std::printf("FAIL %s: ", __func__);     \
    std::printf(__VA_ARGS__);               \
    std::printf("\n");                      \
    ++g_fail;                               \
    return;                                 \
  } while (0)

static const int kData = 12, kParity = 4, kShard = 1024;  // xrs_test.go:21-23

static Vects new_shard_matrix(int shards, int size) { return Vects(shards, Vect(size, 0)); }
static void fill_random(std::mt19937_64& r, Vect& v) {
  for (auto& b : v) b = static_cast<uint8_t>(r());
}
static bool is_in(int e, const std::vector<int>& s) {
  return std::find(s.begin(), s.end(), e) != s.end();
}
static std::unique_ptr<XRS> must_new(int d, int p) {
  std::unique_ptr<XRS> x;
  if (Error e = XRS::New(d, p, &x)) {
    std::printf("New(%d,%d): %s\n", d, p, e.msg.c_str());
    std::exit(2);
  }
  return x;
}

// xrs_test.go:83-99 makeXORSetOld
static std::map<int, std::vector<int>> make_xorset_old(int d, int p) {
  std::map<int, std::vector<int>> m;
  int a = 0;
  for (;;) {
    if (a == d) break;
    for (int i = d + 1; i < d + p; ++i) {
      if (a == d) break;
      m[i].push_back(a);
      ++a;
    }
  }
  return m;
}

// xrs_test.go:51-80
static void TestMakeXORSet() {
  for (int d = 1; d <= 255; ++d)
    for (int p = 2; p <= 255; ++p) {
      if (d + p > 256) continue;
      auto x = must_new(d, p);
      if (x->XORSet() != make_xorset_old(d, p)) FATAL("mismatch %d+%d", d, p);
    }
}

// xrs_test.go:124-156
static void TestXRS_GetNeedVects() {
  for (int d = 1; d <= 255; ++d)
    for (int p = 2; p <= 255; ++p) {
      if (d + p > 256) continue;
      auto x = must_new(d, p);
      for (int i = 0; i < d; ++i) {
        std::vector<int> a, b;
        if (Error e = x->GetNeedVects(i, &a, &b)) FATAL("%s", e.msg.c_str());
        a.push_back(i);
        std::sort(a.begin(), a.end());
        if (a != x->XORSet().at(b[1])) FATAL("element mismatch %d+%d i=%d", d, p, i);
      }
    }
}

static void TestErrors() {
  std::unique_ptr<XRS> x;
  Error e = XRS::New(10, 1, &x);
  if (e.msg != "illegal parity") FATAL("got '%s'", e.msg.c_str());
  x = must_new(kData, kParity);
  std::vector<int> a, b;
  e = x->GetNeedVects(12, &a, &b);
  if (e.msg != "illegal data index: 12") FATAL("got '%s'", e.msg.c_str());
  Vects odd = new_shard_matrix(kData + kParity, 3);
  e = x->Encode(odd);
  if (e.msg != "vect size not even: 3") FATAL("got '%s'", e.msg.c_str());
}

// xrs_test.go:101-122 ("Powered by MATLAB")
static void TestXRS_Encode() {
  auto x = must_new(5, 5);
  Vects vects = {{0, 0}, {4, 7}, {2, 4}, {6, 9}, {8, 11}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}};
  if (Error e = x->Encode(vects)) FATAL("%s", e.msg.c_str());
  Vects exp = {{0, 0}, {4, 7}, {2, 4}, {6, 9}, {8, 11}, {97, 156}, {173, 117}, {218, 110},
               {107, 59}, {110, 153}};
  for (size_t i = 0; i < exp.size(); ++i)
    if (vects[i] != exp[i]) FATAL("encode failed: vect %zu mismatch", i);
}

// xrs_test.go:162-227 testReconstOne
static void testReconstOne(int data, int parity, int size) {
  std::mt19937_64 r(1);
  for (int lost = 0; lost < data; ++lost) {
    Vects expect = new_shard_matrix(data + parity, size);
    for (int j = 0; j < data; ++j) fill_random(r, expect[j]);
    auto x = must_new(data, parity);
    if (Error e = x->Encode(expect)) FATAL("%s", e.msg.c_str());
    Vects result = expect;
    result[lost].assign(size, 0);
    std::vector<int> a_need, b_need;
    if (Error e = x->GetNeedVects(lost, &a_need, &b_need)) FATAL("%s", e.msg.c_str());
    const int half = size / 2;
    for (int j = 0; j < data + parity; ++j) {
      if (!is_in(j, a_need)) std::fill(result[j].begin(), result[j].begin() + half, 0);
      if (j >= data && !is_in(j, b_need)) std::fill(result[j].begin() + half, result[j].end(), 0);
    }
    std::fill(result[lost].begin() + half, result[lost].end(), 0);
    if (Error e = x->ReconstOne(result, lost)) FATAL("%s", e.msg.c_str());
    if (result[lost] != expect[lost]) FATAL("mismatch reconstOne; vect: %d; size: %d", lost, size);
  }
}
static void TestXRS_ReconstOne() {
  testReconstOne(kData, kParity, 2);  // xrs_test.go:159
  testReconstOne(kData, kParity, 4096);
}

static std::vector<int> make_lost_random(std::mt19937_64& r, int n, int lost_n) {
  std::vector<int> l;
  while (static_cast<int>(l.size()) < lost_n) {
    int v = static_cast<int>(r() % n);
    if (!is_in(v, l)) l.push_back(v);
  }
  return l;
}
static std::vector<int> make_has_from_lost(int n, const std::vector<int>& lost) {
  std::vector<int> s;
  for (int i = 0; i < n; ++i)
    if (!is_in(i, lost)) s.push_back(i);
  return s;
}

// xrs_test.go:265-314 testReconst
static void testReconst(int data, int parity, int size, int loop) {
  std::mt19937_64 r(2);
  auto x = must_new(data, parity);
  for (int i = 0; i < loop; ++i) {
    Vects exp = new_shard_matrix(data + parity, size), act = new_shard_matrix(data + parity, size);
    for (int j = 0; j < data; ++j) fill_random(r, exp[j]);
    if (Error e = x->Encode(exp)) FATAL("%s", e.msg.c_str());
    std::vector<int> lost = make_lost_random(r, data + parity, static_cast<int>(r() % (parity + 1)));
    std::vector<int> need(lost.begin(), lost.begin() + r() % (lost.size() + 1));
    if (need.size() == 1) lost = need;
    std::vector<int> has = make_has_from_lost(data + parity, lost);
    for (int h : has) act[h] = exp[h];
    for (int nr : need)
      if (r() % 4 == 0) act[nr] = exp[nr];
    if (Error e = x->Reconst(act, has, need)) FATAL("%s", e.msg.c_str());
    for (int n : need)
      if (exp[n] != act[n]) FATAL("reconst failed: vect: %d, size: %d", n, size);
  }
}
static void TestXRS_Reconst() { testReconst(kData, kParity, kShard, 128); }

// xrs_test.go:320-359 testUpdate
static void testUpdate(int data, int parity, int size) {
  std::mt19937_64 r(3);
  auto x = must_new(data, parity);
  for (int i = 0; i < data; ++i) {
    Vects act = new_shard_matrix(data + parity, size), exp = new_shard_matrix(data + parity, size);
    for (int j = 0; j < data; ++j) {
      fill_random(r, exp[j]);
      act[j] = exp[j];
    }
    if (Error e = x->Encode(act)) FATAL("%s", e.msg.c_str());
    Vect nd(size);
    fill_random(r, nd);
    if (Error e = x->Update(act[i], nd, i, xrs::slices(act, data))) FATAL("%s", e.msg.c_str());
    exp[i] = nd;
    if (Error e = x->Encode(exp)) FATAL("%s", e.msg.c_str());
    for (int j = data; j < data + parity; ++j)
      if (act[j] != exp[j]) FATAL("update failed: vect: %d, size: %d", j, size);
  }
}
static void TestXRS_Update() { testUpdate(kData, kParity, kShard); }

// xrs_test.go:423-441
static std::vector<int> make_replace_rows_random(std::mt19937_64& r, int data) {
  const int n = static_cast<int>(r() % (data + 1));
  std::vector<int> s;
  for (int i = 0; i < 64 && static_cast<int>(s.size()) < n; ++i) {
    int v = static_cast<int>(r() % data);
    if (!is_in(v, s)) s.push_back(v);
  }
  if (s.empty()) s.push_back(0);
  return s;
}

// xrs_test.go:366-421 testReplace
static void testReplace(int data, int parity, int size, int loop, bool to_zero) {
  std::mt19937_64 r(to_zero ? 4 : 5);
  auto x = must_new(data, parity);
  for (int i = 0; i < loop; ++i) {
    std::vector<int> rows = make_replace_rows_random(r, data);
    Vects act = new_shard_matrix(data + parity, size), exp = new_shard_matrix(data + parity, size);
    for (int j = 0; j < data; ++j) {
      fill_random(r, exp[j]);
      act[j] = exp[j];
    }
    Vects dv;
    for (int rr : rows) dv.push_back(exp[rr]);
    if (to_zero)
      for (int rr : rows) exp[rr].assign(size, 0);
    if (Error e = x->Encode(exp)) FATAL("%s", e.msg.c_str());
    if (!to_zero)
      for (int rr : rows) act[rr].assign(size, 0);
    if (Error e = x->Encode(act)) FATAL("%s", e.msg.c_str());
    if (Error e = x->Replace(xrs::slices(dv), rows, xrs::slices(act, data)))
      FATAL("%s", e.msg.c_str());
    for (int j = data; j < data + parity; ++j)
      if (act[j] != exp[j]) FATAL("replace failed: vect: %d, size: %d", j, size);
  }
}
static void TestXRS_Replace() {
  testReplace(kData, kParity, kShard, 1024, true);
  testReplace(kData, kParity, kShard, 1024, false);
}

// Not in the reference: the batching queue from 16 threads, each checking its
// own stripes against the synchronous calls (Encode, Update of random rows,
// ReconstOne, two-loss Reconst), then the queue destroyed while nothing is in
// flight.
static void TestQueue_Concurrent() {
  auto x = must_new(kData, kParity);
  std::unique_ptr<xrs::Queue> q;
  if (Error e = xrs::Queue::New(*x, kShard, &q, 64, 100)) FATAL("Queue::New: %s", e.msg.c_str());
  std::atomic<int> bad{0};
  std::vector<std::thread> th;
  for (int t = 0; t < 16; ++t)
    th.emplace_back([&, t] {
      std::mt19937_64 r(100 + t);
      Vects v = new_shard_matrix(kData + kParity, kShard);
      for (int j = 0; j < kData; ++j) fill_random(r, v[j]);
      Vects ref = v;
      if (q->Encode(v) || x->Encode(ref) || v != ref) ++bad;
      for (int i = 0; i < 20; ++i) {
        const int row = static_cast<int>(r() % kData);
        Vect nd(kShard);
        fill_random(r, nd);
        auto pv = xrs::slices(v, kData), pr = xrs::slices(ref, kData);
        if (q->Update(v[row], nd, row, pv) || x->Update(ref[row], nd, row, pr)) ++bad;
        v[row] = nd;
        ref[row] = nd;
        if (v != ref) ++bad;
        const int k = static_cast<int>(r() % kData);
        Vects w = v;
        std::fill(w[k].begin(), w[k].end(), 0);
        if (q->ReconstOne(w, k) || w[k] != v[k]) ++bad;
        // two lost (one data, one parity), both needed: queue vs sync call
        const std::vector<int> lost = {k, kData + 1 + (i % (kParity - 1))};
        std::vector<int> has;
        for (int j = 0; j < kData + kParity; ++j)
          if (!is_in(j, lost)) has.push_back(j);
        Vects g1 = v, g2 = v;
        for (int j : lost) {
          std::fill(g1[j].begin(), g1[j].end(), 0x5a);
          std::fill(g2[j].begin(), g2[j].end(), 0x5a);
        }
        if (q->Reconst(g1, has, lost) || x->Reconst(g2, has, lost) || g1 != g2) ++bad;
        // Replace of two rows with fresh data: queue vs sync call
        const std::vector<int> rr = {row, (row + 5) % kData};
        Vects nd2 = new_shard_matrix(2, kShard);
        for (auto& z : nd2) fill_random(r, z);
        Vects pq(v.begin() + kData, v.end()), ps = pq;
        if (q->Replace(xrs::slices(nd2), rr, xrs::slices(pq)) ||
            x->Replace(xrs::slices(nd2), rr, xrs::slices(ps)) || pq != ps)
          ++bad;
      }
    });
  for (auto& t : th) t.join();
  if (bad) FATAL("%d mismatches or errors", bad.load());
  Vects par = new_shard_matrix(kParity, kShard);
  if (Error e = q->Update(Vect(kShard), Vect(kShard), kData, xrs::slices(par));
      !e || e.msg != "illegal data index: 12")
    FATAL("Update(row=d): got \"%s\"", e.msg.c_str());
}

// Not in the reference: the asynchronous queue calls.  8 threads, each keeping
// a window of 6 stripes in flight (xrs::Queue::SubmitEncode /
// SubmitReconstOne, then Ticket::Wait oldest first; a "queue busy" submit
// waits on the oldest ticket and retries), every stripe equal to a second
// codec's synchronous call.  One cgo call site with k stripes outstanding
// (the reference's call, xrs_test.go:498-521, is one x.Encode per stripe).
static void TestQueue_Async() {
  constexpr int kThreads = 8, kWin = 6, kStripes = 48, kSize = 4096;
  auto x = must_new(kData, kParity), y = must_new(kData, kParity);
  std::unique_ptr<xrs::Queue> q;
  if (Error e = xrs::Queue::New(*x, kSize, &q, 8, 50)) FATAL("Queue::New: %s", e.msg.c_str());
  std::atomic<int> bad{0}, busy{0};
  std::vector<std::thread> th;
  for (int t = 0; t < kThreads; ++t)
    th.emplace_back([&, t] {
      std::mt19937_64 r(900 + t);
      std::vector<Vects> v(kStripes, new_shard_matrix(kData + kParity, kSize));
      std::vector<Vects> ref(kStripes);
      for (int s = 0; s < kStripes; ++s) {
        for (int j = 0; j < kData; ++j) fill_random(r, v[s][j]);
        ref[s] = v[s];
        if (y->Encode(ref[s])) ++bad;
      }
      std::vector<int> ks(kStripes);
      for (int& k : ks) k = static_cast<int>(r() % kData);
      for (int pass = 0; pass < 2; ++pass) {
        std::vector<xrs::Queue::Ticket> tk(kStripes);
        int oldest = 0;
        for (int s = 0; s < kStripes; ++s) {
          if (s - oldest >= kWin && tk[oldest++].Wait()) ++bad;
          for (;;) {
            Error e = pass == 0 ? q->SubmitEncode(xrs::slices(v[s]), &tk[s])
                                : q->SubmitReconstOne(xrs::slices(v[s]), ks[s], &tk[s]);
            if (!e) break;
            if (e.msg != "queue busy") {
              ++bad;
              break;
            }
            ++busy;
            if (oldest < s) {
              if (tk[oldest++].Wait()) ++bad;
            } else {
              std::this_thread::yield();
            }
          }
        }
        for (; oldest < kStripes; ++oldest)
          if (tk[oldest].Wait()) ++bad;
        for (int s = 0; s < kStripes; ++s)
          if (v[s] != ref[s]) ++bad;
        if (pass == 0)
          for (int s = 0; s < kStripes; ++s) std::fill(v[s][ks[s]].begin(), v[s][ks[s]].end(), 0);
      }
    });
  for (auto& t : th) t.join();
  std::printf("  async: %d busy returns\n", busy.load());
  if (bad) FATAL("%d mismatches or errors", bad.load());
}

// Not in the reference: 32 threads released together (a spin barrier) make
// one per-stripe Encode and one ReconstOne per round on ONE queue, as many
// goroutines calling x.Encode per stripe would (xrs_test.go:498-521): the
// queue must coalesce them (fewer batches than calls, several of 4 stripes or
// more; measured 512 calls in 263 batches, 17 of >= 4 stripes), and every
// result equals a second codec's sync call.
static void TestQueue_Coalesces() {
  constexpr int kThreads = 32, kRounds = 8, kSize = 4096;
  auto x = must_new(kData, kParity), y = must_new(kData, kParity);
  std::unique_ptr<xrs::Queue> q;
  if (Error e = xrs::Queue::New(*x, kSize, &q, 1024, 50)) FATAL("Queue::New: %s", e.msg.c_str());
  std::vector<Vects> v(kThreads), ref(kThreads);
  std::mt19937_64 r(4242);
  for (int t = 0; t < kThreads; ++t) {
    v[t] = new_shard_matrix(kData + kParity, kSize);
    for (int j = 0; j < kData; ++j) fill_random(r, v[t][j]);
    ref[t] = v[t];
    if (y->Encode(ref[t])) FATAL("reference encode");
  }
  std::atomic<int> arrived{0}, bad{0};
  auto barrier = [&](int phase) {  // phase p: every thread waits for (p+1) * kThreads arrivals
    arrived.fetch_add(1);
    while (arrived.load() < (phase + 1) * kThreads) std::this_thread::yield();
  };
  std::vector<std::thread> th;
  for (int t = 0; t < kThreads; ++t)
    th.emplace_back([&, t] {
      for (int i = 0; i < kRounds; ++i) {
        barrier(2 * i);
        for (int j = kData; j < kData + kParity; ++j) std::fill(v[t][j].begin(), v[t][j].end(), 0);
        if (q->Encode(v[t]) || v[t] != ref[t]) ++bad;
        const int k = (t + i) % kData;
        std::fill(v[t][k].begin(), v[t][k].end(), 0x3c);
        barrier(2 * i + 1);
        if (q->ReconstOne(v[t], k) || v[t] != ref[t]) ++bad;
      }
    });
  for (auto& t : th) t.join();
  if (bad) FATAL("%d mismatches or errors", bad.load());
  const std::vector<uint64_t> sizes = q->BatchSizes();
  uint64_t batches = 0, stripes = 0, big = 0;
  for (size_t n = 0; n < sizes.size(); ++n) {
    batches += sizes[n];
    stripes += n * sizes[n];
    if (n >= 4) big += sizes[n];
  }
  std::printf("  queue: %d calls in %llu batches (%llu of >= 4 stripes)\n", 2 * kThreads * kRounds,
              static_cast<unsigned long long>(batches), static_cast<unsigned long long>(big));
  if (stripes != 2u * kThreads * kRounds) FATAL("stripes run %llu", static_cast<unsigned long long>(stripes));
  if (batches >= static_cast<uint64_t>(2 * kThreads * kRounds) || big < 3)
    FATAL("no coalescing: %llu batches for %d calls, %llu of >= 4 stripes",
          static_cast<unsigned long long>(batches), 2 * kThreads * kRounds,
          static_cast<unsigned long long>(big));
}

// Not in the reference: the plain per-stripe calls from 16 threads on ONE
// codec (a Go server's goroutines sharing an *XRS).  Contended calls batch
// through the codec's own queue (codec.cpp auto_queue); every result must
// equal a second codec's, driven from one thread at a time.
static void TestXRS_SharedCodecConcurrent() {
  auto x = must_new(kData, kParity), y = must_new(kData, kParity);
  std::mutex ymu;
  std::atomic<int> bad{0};
  std::vector<std::thread> th;
  for (int t = 0; t < 16; ++t)
    th.emplace_back([&, t] {
      std::mt19937_64 r(500 + t);
      for (int i = 0; i < 30; ++i) {
        Vects v = new_shard_matrix(kData + kParity, kShard);
        for (int j = 0; j < kData; ++j) fill_random(r, v[j]);
        Vects ref = v;
        {
          std::lock_guard<std::mutex> g(ymu);
          if (y->Encode(ref)) ++bad;
        }
        if (x->Encode(v) || v != ref) ++bad;
        const int row = static_cast<int>(r() % kData);
        Vect nd(kShard);
        fill_random(r, nd);
        auto pv = xrs::slices(v, kData), pr = xrs::slices(ref, kData);
        {
          std::lock_guard<std::mutex> g(ymu);
          if (y->Update(ref[row], nd, row, pr)) ++bad;
        }
        if (x->Update(v[row], nd, row, pv)) ++bad;
        v[row] = nd;
        ref[row] = nd;
        if (v != ref) ++bad;
        const int k = static_cast<int>(r() % kData);
        Vects w = v;
        std::fill(w[k].begin(), w[k].end(), 0);
        if (x->ReconstOne(w, k) || w[k] != v[k]) ++bad;
        // two lost (one data, one parity), both needed
        const std::vector<int> lost = {k, kData + 1 + (i % (kParity - 1))};
        std::vector<int> has;
        for (int j = 0; j < kData + kParity; ++j)
          if (!is_in(j, lost)) has.push_back(j);
        Vects g1 = v, g2 = v;
        for (int j : lost) {
          std::fill(g1[j].begin(), g1[j].end(), 0x5a);
          std::fill(g2[j].begin(), g2[j].end(), 0x5a);
        }
        {
          std::lock_guard<std::mutex> g(ymu);
          if (y->Reconst(g2, has, lost)) ++bad;
        }
        if (x->Reconst(g1, has, lost) || g1 != g2) ++bad;
        // Replace of two rows with fresh data
        const std::vector<int> rr = {row, (row + 5) % kData};
        Vects nd2 = new_shard_matrix(2, kShard);
        for (auto& z : nd2) fill_random(r, z);
        Vects pq(v.begin() + kData, v.end()), ps = pq;
        {
          std::lock_guard<std::mutex> g(ymu);
          if (y->Replace(xrs::slices(nd2), rr, xrs::slices(ps))) ++bad;
        }
        if (x->Replace(xrs::slices(nd2), rr, xrs::slices(pq)) || pq != ps) ++bad;
      }
    });
  for (auto& t : th) t.join();
  if (bad) FATAL("%d mismatches or errors", bad.load());
}

// Not in the reference: slot recycling under oversubscription.
// Two staging batches of two stripes, one in flight, 32 callers: a batch is
// freed and reopened while other callers of its previous use still copy out,
// so a caller that read the batch's slot count after its own release could
// free a batch that is running.  Every Encode is checked against a serial
// codec.
static void TestQueue_Oversubscribed() {
  setenv("XRS_QUEUE_BATCHES", "2", 1);
  setenv("XRS_QUEUE_INFLIGHT", "1", 1);
  auto x = must_new(kData, kParity), y = must_new(kData, kParity);
  std::unique_ptr<xrs::Queue> q;
  Error e = xrs::Queue::New(*x, kShard, &q, 2, 0);
  unsetenv("XRS_QUEUE_BATCHES");
  unsetenv("XRS_QUEUE_INFLIGHT");
  if (e) FATAL("Queue::New: %s", e.msg.c_str());
  std::mutex ymu;
  std::atomic<int> bad{0};
  std::vector<std::thread> th;
  for (int t = 0; t < 32; ++t)
    th.emplace_back([&, t] {
      std::mt19937_64 r(900 + t);
      for (int i = 0; i < 150; ++i) {
        Vects v = new_shard_matrix(kData + kParity, kShard);
        for (int j = 0; j < kData; ++j) fill_random(r, v[j]);
        Vects ref = v;
        {
          std::lock_guard<std::mutex> g(ymu);
          if (y->Encode(ref)) ++bad;
        }
        if (q->Encode(v) || v != ref) ++bad;
      }
    });
  for (auto& t : th) t.join();
  if (bad) FATAL("%d mismatches or errors", bad.load());
}

// Not in the reference: the persistent staged kernel forced for every
// 2-lost launch (XRS_WSP=512; by default it runs only for large batches), on
// an 8-block grid so each block takes many tiles from its launch's counter,
// from 8 threads on one codec: counters come from the library's
// stream-ordered pool while other launches hold theirs.  Host-resident
// batches of 4 stripes of 1 MiB vects in pinned, mapped memory (the kernels
// run in place over PCIe).  The rebuilt data vects must equal the encoded
// ones (the surviving parity's b-halves come back in RS form, the
// reference's retrieveRS side effect, so parity is not compared).
static void TestXRS_ReconstPersistent() {
  setenv("XRS_WSP", "512", 1);
  setenv("XRS_WSP_GRID", "8", 1);
  auto x = must_new(kData, kParity);
  xrs_trace_kernels(1);
  std::atomic<int> bad{0};
  std::vector<std::thread> th;
  constexpr size_t S = 1 << 20, n = 4, stripe = (kData + kParity) * S;
  for (int t = 0; t < 8; ++t)
    th.emplace_back([&, t] {
      std::mt19937_64 r(700 + t);
      uint8_t* h = static_cast<uint8_t*>(xrs_host_alloc(n * stripe));
      if (!h) {
        ++bad;
        return;
      }
      for (int i = 0; i < 3; ++i) {
        for (size_t st = 0; st < n; ++st)
          for (size_t b = 0; b < kData * S; b += 8) {
            const uint64_t v = r();
            std::memcpy(h + st * stripe + b, &v, 8);
          }
        if (xrs_encode_host(x->codec(), h, S, S, stripe, n)) ++bad;
        std::vector<uint8_t> orig(h, h + n * stripe);
        const int a = static_cast<int>(r() % kData), b = (a + 1 + static_cast<int>(r() % (kData - 1))) % kData;
        const int lost[2] = {a, b};
        std::vector<int> has;
        for (int j = 0; j < kData + kParity; ++j)
          if (j != a && j != b) has.push_back(j);
        for (size_t st = 0; st < n; ++st)
          for (int j : lost) std::memset(h + st * stripe + j * S, 0x5a, S);
        if (xrs_reconst_host(x->codec(), h, S, S, stripe, n, has.data(), static_cast<int>(has.size()), lost, 2))
          ++bad;
        for (size_t st = 0; st < n; ++st)
          if (std::memcmp(h + st * stripe, orig.data() + st * stripe, kData * S) != 0) ++bad;
      }
      xrs_host_free(h);
    });
  for (auto& t : th) t.join();
  xrs_trace_kernels(0);
  std::string names(xrs_traced_kernels(nullptr, 0) + 1, '\0');
  xrs_traced_kernels(&names[0], names.size());
  unsetenv("XRS_WSP");
  unsetenv("XRS_WSP_GRID");
  if (bad) FATAL("%d mismatches or errors", bad.load());
  if (names.find("staged_wsp_kernel<12, ") == std::string::npos)
    FATAL("the persistent kernel did not run: %s", names.c_str());
}

// A vect shorter or longer than vects[0] is rejected before the C ABI call
// (which reads and writes `size` bytes of every vect): ADVICE r1.
// Not in the reference: per-stripe calls on registered host memory
// (xrs_host_alloc, and xrs_host_register on one thread's buffer).  8 threads
// on ONE codec and ONE queue: lone sync calls run in place, contended ones go
// through the codec's auto-queue, queue calls batch in table mode (one
// indirect-row launch over the callers' bytes).  Every result equals the same
// call on plain copies.  Vects start 2 bytes past a 16-byte boundary.
static void TestRegistered_SyncAndQueue() {
  constexpr size_t S = 4096, kStride = S + 64;
  constexpr int kRows = kData + kParity + 4;  // + new data, two Replace rows, spare
  auto x = must_new(kData, kParity);
  xrs_queue* q = nullptr;
  if (xrs_queue_new(x->codec(), S, 64, 50, &q)) FATAL("xrs_queue_new");
  std::atomic<int> bad{0};
  std::vector<std::thread> th;
  for (int t = 0; t < 8; ++t)
    th.emplace_back([&, t] {
      const size_t bytes = (kRows * kStride + 65535) / 65536 * 65536;
      uint8_t* base = nullptr;
      std::vector<uint8_t> own;
      if (t == 3) {  // caller memory pinned with xrs_host_register
        own.resize(bytes + 65536);
        base = own.data() + (65536 - reinterpret_cast<uintptr_t>(own.data()) % 65536) % 65536;
        if (xrs_host_register(base, bytes)) {
          ++bad;
          return;
        }
      } else if (!(base = static_cast<uint8_t*>(xrs_host_alloc(bytes)))) {
        ++bad;
        return;
      }
      std::vector<uint8_t*> v(kRows);
      for (int j = 0; j < kRows; ++j) v[j] = base + j * kStride + 2;
      std::mt19937_64 r(700 + t);
      auto fill = [&](uint8_t* p) { for (size_t i = 0; i < S; ++i) p[i] = static_cast<uint8_t>(r()); };
      auto copy = [&](int from, int to) {
        Vects c = new_shard_matrix(to - from, S);
        for (int j = from; j < to; ++j) std::memcpy(c[j - from].data(), v[j], S);
        return c;
      };
      auto same = [&](const Vects& c, int from) {
        for (size_t j = 0; j < c.size(); ++j)
          if (std::memcmp(c[j].data(), v[from + j], S)) return false;
        return true;
      };
      const int n = kData + kParity;
      for (int it = 0; it < 24; ++it) {
        const bool viaq = (it + t) % 2 == 0;
        for (int j = 0; j < kData; ++j) fill(v[j]);
        Vects ref = copy(0, n);
        int rc = viaq ? xrs_queue_encode(q, v.data(), n) : xrs_encode(x->codec(), v.data(), n, S);
        if (rc || x->Encode(ref) || !same(ref, 0)) ++bad;
        const int k = static_cast<int>(r() % kData);
        std::memset(v[k], 0, S);
        rc = viaq ? xrs_queue_reconst_one(q, v.data(), n, k) : xrs_reconst_one(x->codec(), v.data(), n, S, k);
        if (rc || !same(ref, 0)) ++bad;
        // Update of row k with fresh bytes (v[n] holds them)
        fill(v[n]);
        Vects newd = copy(n, n + 1);
        rc = viaq ? xrs_queue_update(q, v[k], v[n], k, v.data() + kData, kParity)
                  : xrs_update(x->codec(), v[k], v[n], S, k, v.data() + kData, kParity);
        auto pr = xrs::slices(ref, kData);
        if (rc || x->Update(ref[k], newd[0], k, pr)) ++bad;
        std::memcpy(v[k], v[n], S);
        ref[k] = newd[0];
        if (!same(ref, 0)) ++bad;
        // Replace of two rows (v[n+1], v[n+2] hold their data)
        const std::vector<int> rows = {k, (k + 7) % kData};
        fill(v[n + 1]);
        fill(v[n + 2]);
        Vects rd = copy(n + 1, n + 3);
        rc = viaq ? xrs_queue_replace(q, v.data() + n + 1, rows.data(), 2, v.data() + kData, kParity)
                  : xrs_replace(x->codec(), v.data() + n + 1, rows.data(), 2, S, v.data() + kData, kParity);
        if (rc || x->Replace(xrs::slices(rd), rows, xrs::slices(ref, kData)) || !same(ref, 0)) ++bad;
        // Reconst of one data and one parity vect, both needed
        const std::vector<int> lost = {k, kData + 1 + it % (kParity - 1)};
        std::vector<int> has;
        for (int j = 0; j < n; ++j)
          if (!is_in(j, lost)) has.push_back(j);
        for (int j : lost) {
          std::memset(v[j], 0x5a, S);
          std::fill(ref[j].begin(), ref[j].end(), 0x5a);
        }
        rc = viaq ? xrs_queue_reconst(q, v.data(), n, has.data(), 14, lost.data(), 2)
                  : xrs_reconst(x->codec(), v.data(), n, S, has.data(), 14, lost.data(), 2);
        if (rc || x->Reconst(ref, has, lost) || !same(ref, 0)) ++bad;
      }
      if (t == 3) {
        if (xrs_host_unregister(base)) ++bad;
      } else {
        xrs_host_free(base);
      }
    });
  for (auto& t : th) t.join();
  xrs_queue_free(q);
  if (bad) FATAL("%d mismatches or errors", bad.load());
}

// Registered pages handed back and reused.  A buffer is
// pinned with xrs_host_register, an in-place Encode runs on it (xrs.go:103-128,
// the call whose buffers a cgo BufPool pools), then it is unregistered and
// freed, and the allocator hands the same pages out again -- what a Go
// BufPool.Close() followed by GC and new allocations does.
// On the reused pages: the runtime's pageable copies (hipMemcpy H2D from
// them and D2H into them) and a pageable host-resident Encode
// (xrs_encode_host, hipMemcpy2DAsync chunks) must be exact and leave no
// error.  64 KiB buffers come from the heap, 2 MiB ones first from mmap.
static void TestRegistered_UnregisterFreeReuse() {
  constexpr size_t S = 4096, kStripe = (kData + kParity) * S;  // 64 KiB
  auto x = must_new(kData, kParity);
  std::mt19937_64 r(4242);
  int reused = 0, rounds = 0;
  uint8_t* dev = nullptr;
  if (hipMalloc(reinterpret_cast<void**>(&dev), size_t(2) << 20) != hipSuccess) FATAL("hipMalloc");
  auto overlaps = [](const uint8_t* a, const uint8_t* b, size_t n) { return b < a + n && a < b + n; };
  auto encoded_copy = [&](const uint8_t* base, size_t n_stripes) {
    Vects all;
    for (size_t s = 0; s < n_stripes; ++s) {
      Vects v = new_shard_matrix(kData + kParity, S);
      for (int j = 0; j < kData + kParity; ++j) std::memcpy(v[j].data(), base + s * kStripe + j * S, S);
      if (x->Encode(v)) return Vects();
      for (auto& e : v) all.push_back(std::move(e));
    }
    return all;
  };
  auto same = [&](const Vects& want, const uint8_t* base) {
    if (want.empty()) return false;
    for (size_t i = 0; i < want.size(); ++i)
      if (std::memcmp(want[i].data(), base + i * S, S)) return false;
    return true;
  };
  for (size_t bytes : {kStripe, size_t(2) << 20}) {
    const size_t n_stripes = bytes / kStripe;
    for (int round = 0; round < 8; ++round, ++rounds) {
      // 1. register a page-aligned malloc buffer; Encode in place on it
      uint8_t* a = static_cast<uint8_t*>(std::aligned_alloc(4096, bytes));
      for (size_t i = 0; i < bytes; ++i) a[i] = static_cast<uint8_t>(r());
      const Vects want_a = encoded_copy(a, 1);
      if (xrs_host_register(a, bytes)) FATAL("xrs_host_register");
      std::vector<uint8_t*> v(kData + kParity);
      for (int j = 0; j < kData + kParity; ++j) v[j] = a + j * S;
      if (xrs_encode(x->codec(), v.data(), kData + kParity, S) || !same(want_a, a))
        FATAL("in-place Encode on registered memory, round %d", round);
      // 2. unregister, free
      if (xrs_host_unregister(a)) FATAL("xrs_host_unregister");
      std::free(a);
      // 3. allocate until the allocator hands back a page of the old buffer
      uint8_t* b = nullptr;
      std::vector<uint8_t*> held;
      for (int t = 0; t < 32 && !b; ++t) {
        uint8_t* c = static_cast<uint8_t*>(std::aligned_alloc(4096, bytes));
        if (overlaps(a, c, bytes)) b = c;
        else held.push_back(c);
      }
      if (b) ++reused;
      else {
        b = held.back();
        held.pop_back();
      }
      for (uint8_t* h : held) std::free(h);
      // 4. the runtime's pageable copies to and from the reused pages
      for (size_t i = 0; i < bytes; ++i) b[i] = static_cast<uint8_t>(r());
      std::vector<uint8_t> back(bytes), keep(b, b + bytes);
      if (hipMemcpy(dev, b, bytes, hipMemcpyHostToDevice) != hipSuccess ||
          hipMemcpy(back.data(), dev, bytes, hipMemcpyDeviceToHost) != hipSuccess ||
          std::memcmp(back.data(), b, bytes))
        FATAL("pageable H2D from reused pages, %zu B, round %d", bytes, round);
      std::memset(b, 0, bytes);
      if (hipMemcpy(b, dev, bytes, hipMemcpyDeviceToHost) != hipSuccess ||
          std::memcmp(keep.data(), b, bytes))
        FATAL("pageable D2H into reused pages, %zu B, round %d", bytes, round);
      // 5. a pageable host-resident Encode over them
      const Vects want_b = encoded_copy(b, n_stripes);
      if (xrs_encode_host(x->codec(), b, S, S, kStripe, n_stripes) || !same(want_b, b))
        FATAL("xrs_encode_host on reused pages, %zu B, round %d", bytes, round);
      if (hipDeviceSynchronize() != hipSuccess || hipGetLastError() != hipSuccess)
        FATAL("HIP error after round %d", round);
      std::free(b);
    }
  }
  (void)hipFree(dev);
  std::printf("  unregister -> free -> reuse: a freed page came back in %d of %d rounds\n", reused,
              rounds);
  // (ASan's allocator quarantines freed memory, so its build never sees reuse:
  // there the test checks only the copies and the Encodes)
  if (reused == 0 && !kAsanBuild)
    FATAL("the allocator never reused a freed registered page: the test tested nothing");
}

static void TestMismatchedVects() {
  std::unique_ptr<XRS> x;
  if (Error e = XRS::New(kData, kParity, &x)) FATAL("New: %s", e.msg.c_str());
  Vects v = new_shard_matrix(kData + kParity, 64);
  v[14].resize(32);
  if (Error e = x->Encode(v); !e || e.msg != "illegal vects") FATAL("Encode: \"%s\"", e.msg.c_str());
  if (Error e = x->ReconstOne(v, 0); !e || e.msg != "illegal vects")
    FATAL("ReconstOne: \"%s\"", e.msg.c_str());
  if (Error e = x->Reconst(v, {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11}, {12, 13}); !e || e.msg != "illegal vects")
    FATAL("Reconst: \"%s\"", e.msg.c_str());
  Vects par = new_shard_matrix(kParity, 64);
  if (Error e = x->Update(Vect(64), Vect(63 + 1 - 2), 0, xrs::slices(par)); !e || e.msg != "illegal vects")
    FATAL("Update: \"%s\"", e.msg.c_str());
  Vects data = new_shard_matrix(2, 64);
  data[1].resize(128);
  if (Error e = x->Replace(xrs::slices(data), {0, 1}, xrs::slices(par)); !e || e.msg != "illegal vects")
    FATAL("Replace: \"%s\"", e.msg.c_str());
  // the even-size rule comes first (xrs.go:105)
  Vects odd = new_shard_matrix(kData + kParity, 63);
  odd[3].resize(10);
  if (Error e = x->Encode(odd); !e || e.msg != "vect size not even: 63")
    FATAL("Encode odd: \"%s\"", e.msg.c_str());
}

int main(int argc, char** argv) {
  // xrs_test [--cpu] [name ...]: host-logic tests only, and/or only the named tests
  bool cpu_only = false;
  std::vector<std::string> only;
  for (int i = 1; i < argc; ++i) {
    if (std::strcmp(argv[i], "--cpu") == 0) cpu_only = true;
    else only.push_back(argv[i]);
  }
  struct T {
    const char* name;
    void (*fn)();
    bool gpu;
  } tests[] = {
      {"TestMakeXORSet", TestMakeXORSet, false},
      {"TestXRS_GetNeedVects", TestXRS_GetNeedVects, false},
      {"TestErrors", TestErrors, false},
      {"TestMismatchedVects", TestMismatchedVects, false},
      {"TestXRS_Encode", TestXRS_Encode, true},
      {"TestXRS_ReconstOne", TestXRS_ReconstOne, true},
      {"TestXRS_Reconst", TestXRS_Reconst, true},
      {"TestXRS_Update", TestXRS_Update, true},
      {"TestXRS_Replace", TestXRS_Replace, true},
      {"TestQueue_Concurrent", TestQueue_Concurrent, true},
      {"TestQueue_Oversubscribed", TestQueue_Oversubscribed, true},
      {"TestQueue_Coalesces", TestQueue_Coalesces, true},
      {"TestQueue_Async", TestQueue_Async, true},
      {"TestXRS_SharedCodecConcurrent", TestXRS_SharedCodecConcurrent, true},
      {"TestXRS_ReconstPersistent", TestXRS_ReconstPersistent, true},
      {"TestRegistered_SyncAndQueue", TestRegistered_SyncAndQueue, true},
      {"TestRegistered_UnregisterFreeReuse", TestRegistered_UnregisterFreeReuse, true},
  };
  for (const T& t : tests) {
    if (cpu_only && t.gpu) continue;
    if (!only.empty() && std::find(only.begin(), only.end(), t.name) == only.end()) continue;
    const int before = g_fail;
    t.fn();
    std::printf("%s %s\n", g_fail == before ? "ok  " : "FAIL", t.name);
  }
  std::printf("%s\n", g_fail ? "FAIL" : "PASS");
  std::fflush(stdout);
  // Skip static teardown: under a host-ASan build the HSA runtime's own
  // finalizer trips the sanitizer allocator (not this program's memory).
  std::_Exit(g_fail ? 1 : 0);
}
