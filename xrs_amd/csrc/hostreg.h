// hostreg.h -- process-wide table of the host ranges the library has pinned
// and mapped (xrs_host_alloc / xrs_host_register).  Internal.
//
// A per-stripe call whose vects all lie in such ranges runs without the CPU
// gather / scatter through pinned staging: the kernels read and write the
// caller's buffers in place over PCIe (a lone call through Layout::table, a
// queue batch through its row table), addressed by the device pointer
// recorded here.  A lookup takes no lock and makes no HIP call: an immutable
// sorted table behind an atomic pointer, which register / unregister replace.
// A replaced table is freed by the register / unregister that replaced it,
// after a grace period: HostRangesView keeps a reader count (one of a few
// cache lines, two generations) for the few microseconds of one call's
// lookups, and the writer waits for the counts that may cover the old table.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace xrs_detail {

// Record [p, p + bytes) as pinned and mapped, with device address dev of p.
void host_ranges_add(const void* p, size_t bytes, const void* dev);
// Forget the range starting at p (no-op if there is none).
void host_ranges_remove(const void* p);

// The current table, held for the view's lifetime: one view per call, then
// any number of lookups.
class HostRangesView {
 public:
  HostRangesView();
  ~HostRangesView();
  HostRangesView(const HostRangesView&) = delete;
  HostRangesView& operator=(const HostRangesView&) = delete;
  // Device address of p if [p, p + bytes) lies inside one recorded range, else 0.
  uint64_t device(const void* p, size_t bytes) const;

 private:
  const void* table_;
  unsigned lane_, gen_;
};

// Replaced tables not yet freed (tests; always 0 since round 6).
size_t host_ranges_retired();

}  // namespace xrs_detail
