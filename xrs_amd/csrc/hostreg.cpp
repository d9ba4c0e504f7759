// hostreg.cpp -- the registered host ranges (hostreg.h).
#include "hostreg.h"

#include <algorithm>
#include <atomic>
#include <mutex>
#include <vector>

namespace xrs_detail {
namespace {

struct Range {
  uintptr_t lo, hi;  // [lo, hi)
  uintptr_t dev;     // device address of lo
};
using Table = std::vector<Range>;

// Reader counts, striped over cache lines so concurrent callers do not share
// one.  Every operation is seq_cst: a reader increments its lane before it
// loads the table pointer, and a writer swaps the pointer before it reads the
// lanes, so a reader the writer sees at zero loads the new table.
constexpr unsigned kLanes = 16;
struct alignas(64) Lane {
  std::atomic<uint32_t> n{0};
};
Lane g_lanes[kLanes];
std::atomic<unsigned> g_next_lane{0};

std::atomic<const Table*> g_table{nullptr};
std::mutex g_mu;
std::vector<const Table*> g_retired;  // (g_mu) replaced, maybe still read

unsigned my_lane() {
  thread_local const unsigned lane = g_next_lane.fetch_add(1, std::memory_order_relaxed) % kLanes;
  return lane;
}

bool quiescent() {
  for (const Lane& l : g_lanes)
    if (l.n.load()) return false;
  return true;
}

void publish(Table* t) {  // (g_mu held)
  std::sort(t->begin(), t->end(), [](const Range& a, const Range& b) { return a.lo < b.lo; });
  const Table* old = g_table.exchange(t);
  if (old) g_retired.push_back(old);
  // a reader still holding a retired table keeps its lane above zero; any
  // reader arriving later loads t
  if (quiescent()) {
    for (const Table* r : g_retired) delete r;
    g_retired.clear();
  }
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
  g_lanes[lane_].n.fetch_add(1);
  table_ = g_table.load();
}

HostRangesView::~HostRangesView() { g_lanes[lane_].n.fetch_sub(1); }

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

size_t host_ranges_retired() {
  std::lock_guard<std::mutex> g(g_mu);
  return g_retired.size();
}

}  // namespace xrs_detail
