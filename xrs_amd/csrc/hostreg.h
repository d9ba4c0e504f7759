// hostreg.h -- process-wide table of the host ranges the library has pinned
// and mapped (xrs_host_alloc / xrs_host_register).  Internal.
//
// A per-stripe call whose vects all lie in such ranges runs without the CPU
// gather / scatter through pinned staging: the kernels (or the queue's
// gather / scatter kernels) read and write the caller's buffers in place over
// PCIe, addressed by the device pointer recorded here.  A lookup takes no
// lock and makes no HIP call (an immutable sorted table behind an atomic
// pointer; the rare register / unregister builds a new one).
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace xrs_detail {

// Record [p, p + bytes) as pinned and mapped, with device address dev of p.
void host_ranges_add(const void* p, size_t bytes, const void* dev);
// Forget the range starting at p (no-op if there is none).
void host_ranges_remove(const void* p);
// Device address of p if [p, p + bytes) lies inside one recorded range, else 0.
uint64_t host_ranges_device(const void* p, size_t bytes);

}  // namespace xrs_detail
