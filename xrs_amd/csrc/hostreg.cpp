// hostreg.cpp -- the registered host ranges (hostreg.h).
#include "hostreg.h"

#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <thread>
#include <vector>

namespace xrs_detail {
namespace {

struct Range {
  uintptr_t lo, hi;  // [lo, hi)
  uintptr_t dev;     // device address of lo
};
using Table = std::vector<Range>;

// Reader counts, striped over cache lines so concurrent callers do not share
// one, in two generations.  A reader increments its lane's count of the
// current generation, then loads the table pointer, and holds both for one
// call's lookups (microseconds).  A writer swaps the pointer, then makes two
// grace periods: flip the generation and wait until the old generation's
// counts are all zero, twice.  A reader that loaded the replaced table had
// incremented a count (of either generation) before the swap, and each
// generation is waited for after the swap, so the replaced table is freed at
// once, with no reader on it; readers arriving meanwhile count in the other
// generation, so under steady traffic each wait ends (the round-5
// table waited for all 16 lanes to read zero at once, which steady traffic
// may never give, and retired tables could pile up).  Every operation is
// seq_cst.
constexpr unsigned kLanes = 16;
struct alignas(64) Lane {
  std::atomic<uint32_t> n[2] = {{0}, {0}};
};
Lane g_lanes[kLanes];
std::atomic<unsigned> g_next_lane{0};
std::atomic<unsigned> g_gen{0};

std::atomic<const Table*> g_table{nullptr};
std::mutex g_mu;

unsigned my_lane() {
  thread_local const unsigned lane = g_next_lane.fetch_add(1, std::memory_order_relaxed) % kLanes;
  return lane;
}

void drain(unsigned gen) {  // (a view lasts microseconds: spin first)
  for (const Lane& l : g_lanes)
    for (unsigned i = 0; l.n[gen].load(); ++i) {
      if (i < 4096) _mm_pause();
      else std::this_thread::yield();
    }
}

void publish(Table* t) {  // (g_mu held)
  std::sort(t->begin(), t->end(), [](const Range& a, const Range& b) { return a.lo < b.lo; });
  const Table* old = g_table.exchange(t);
  if (!old) return;
  for (int phase = 0; phase < 2; ++phase) {
    const unsigned g = g_gen.load();
    g_gen.store(g ^ 1u);
    drain(g);
  }
  delete old;
}

}  // namespace

void host_ranges_add(const void* p, size_t bytes, const void* dev) {
  if (!p || !bytes || !dev) return;
  std::lock_guard<std::mutex> g(g_mu);
  const Table* cur = g_table.load();
  auto* t = new Table();
  const uintptr_t lo = reinterpret_cast<uintptr_t>(p);
  if (cur)
    for (const Range& r : *cur)
      if (r.lo != lo) t->push_back(r);
  t->push_back({lo, lo + bytes, reinterpret_cast<uintptr_t>(dev)});
  publish(t);
}

void host_ranges_remove(const void* p) {
  std::lock_guard<std::mutex> g(g_mu);
  const Table* cur = g_table.load();
  const uintptr_t lo = reinterpret_cast<uintptr_t>(p);
  if (!cur || std::none_of(cur->begin(), cur->end(), [lo](const Range& r) { return r.lo == lo; }))
    return;
  auto* t = new Table();
  for (const Range& r : *cur)
    if (r.lo != lo) t->push_back(r);
  publish(t);
}

HostRangesView::HostRangesView() : lane_(my_lane()) {
  gen_ = g_gen.load();
  g_lanes[lane_].n[gen_].fetch_add(1);
  table_ = g_table.load();
}

HostRangesView::~HostRangesView() { g_lanes[lane_].n[gen_].fetch_sub(1); }

uint64_t HostRangesView::device(const void* p, size_t bytes) const {
  const Table* t = static_cast<const Table*>(table_);
  if (!t || t->empty() || !p) return 0;
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  // the last range starting at or below a
  auto it = std::upper_bound(t->begin(), t->end(), a, [](uintptr_t v, const Range& r) { return v < r.lo; });
  if (it == t->begin()) return 0;
  --it;
  if (a + bytes > it->hi || a + bytes < a) return 0;
  return it->dev + (a - it->lo);
}

size_t host_ranges_retired() { return 0; }  // (replaced tables are freed in publish)

}  // namespace xrs_detail
