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

// Readers load the current table without a lock.  A table is never freed once
// published (a reader may still hold it); register / unregister are rare, so
// the retired tables stay small.
std::atomic<const std::vector<Range>*> g_table{nullptr};
std::mutex g_mu;
std::vector<const std::vector<Range>*> g_retired;

void publish(std::vector<Range>* t) {  // (g_mu held)
  std::sort(t->begin(), t->end(), [](const Range& a, const Range& b) { return a.lo < b.lo; });
  const std::vector<Range>* old = g_table.exchange(t, std::memory_order_acq_rel);
  if (old) g_retired.push_back(old);
}

}  // namespace

void host_ranges_add(const void* p, size_t bytes, const void* dev) {
  if (!p || !bytes || !dev) return;
  std::lock_guard<std::mutex> g(g_mu);
  const std::vector<Range>* cur = g_table.load(std::memory_order_acquire);
  auto* t = new std::vector<Range>();
  const uintptr_t lo = reinterpret_cast<uintptr_t>(p);
  if (cur)
    for (const Range& r : *cur)
      if (r.lo != lo) t->push_back(r);
  t->push_back({lo, lo + bytes, reinterpret_cast<uintptr_t>(dev)});
  publish(t);
}

void host_ranges_remove(const void* p) {
  std::lock_guard<std::mutex> g(g_mu);
  const std::vector<Range>* cur = g_table.load(std::memory_order_acquire);
  const uintptr_t lo = reinterpret_cast<uintptr_t>(p);
  if (!cur || std::none_of(cur->begin(), cur->end(), [lo](const Range& r) { return r.lo == lo; }))
    return;
  auto* t = new std::vector<Range>();
  for (const Range& r : *cur)
    if (r.lo != lo) t->push_back(r);
  publish(t);
}

uint64_t host_ranges_device(const void* p, size_t bytes) {
  const std::vector<Range>* t = g_table.load(std::memory_order_acquire);
  if (!t || t->empty() || !p) return 0;
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  // the last range starting at or below a
  auto it = std::upper_bound(t->begin(), t->end(), a,
                             [](uintptr_t v, const Range& r) { return v < r.lo; });
  if (it == t->begin()) return 0;
  --it;
  if (a + bytes > it->hi || a + bytes < a) return 0;
  return it->dev + (a - it->lo);
}

}  // namespace xrs_detail
