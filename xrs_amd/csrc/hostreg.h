// hostreg.h -- process-wide table of the host ranges the library has pinned
// and mapped (xrs_host_alloc / xrs_host_register).  Internal.
//
// A per-stripe call whose vects all lie in such ranges runs without the CPU
// gather / scatter through pinned staging: the kernels read and write the
// caller's buffers in place over PCIe (a lone call through Layout::table, a
// queue batch through its row table), addressed by the device pointer
// recorded here.  A lookup takes no lock and makes no HIP call: an immutable
// sorted table behind an atomic pointer, which register / unregister replace.
// A replaced table is freed once no lookup can still hold it (HostRangesView
// keeps a reader count on one of a few cache lines).
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
  unsigned lane_;
};

// Retired tables not yet freed (tests).
size_t host_ranges_retired();

}  // namespace xrs_detail
