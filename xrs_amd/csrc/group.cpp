// group.cpp -- one process driving several GPUs: one codec
// per device, built by xrs_new with that device current, and one host thread
// per device per call.
//
// Stripes are independent (xrs.go has no cross-stripe state), so a batch is
// split into contiguous stripe ranges, one per member, with no exchange
// between GPUs.  For host-resident batches every GPU moves its share over its
// own PCIe link, so the PCIe-bound host rate adds up across
// the group.
#include <hip/hip_runtime.h>

#include <thread>
#include <vector>

#include "xrs_hip.h"

struct xrs_group {
  std::vector<int> devices;
  std::vector<xrs_codec*> codecs;
};

namespace {

// Contiguous balanced split (xrs_amd/dist.py stripe_range): member i owns
// stripes [start, start + count).
void stripe_range(size_t n, int i, int members, size_t* start, size_t* count) {
  const size_t base = n / members, extra = n % members;
  const size_t ui = static_cast<size_t>(i);
  *start = ui * base + (ui < extra ? ui : extra);
  *count = base + (ui < extra ? 1 : 0);
}

// Run fn(member, first stripe, stripe count) for every member with work, one
// thread per member (the caller's thread runs the last), each with its
// member's device current.  Returns the first member's error in member order.
template <class F>
int for_members(xrs_group* g, size_t n_stripes, F fn) {
  const int m = static_cast<int>(g->codecs.size());
  std::vector<int> err(m, XRS_OK);
  auto job = [&](int i) {
    size_t start, count;
    stripe_range(n_stripes, i, m, &start, &count);
    if (count == 0) return;
    int prev = -1;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(g->devices[i]);
    err[i] = fn(i, start, count);
    if (prev >= 0) (void)hipSetDevice(prev);
  };
  std::vector<std::thread> th;
  for (int i = 0; i + 1 < m; ++i) th.emplace_back(job, i);
  job(m - 1);
  for (auto& t : th) t.join();
  for (int e : err)
    if (e) return e;
  return XRS_OK;
}

}  // namespace

extern "C" {

int xrs_group_new(int data_num, int parity_num, const int* devices, int n_devices,
                  xrs_group** out) {
  if (!out) return XRS_ERR_INVALID_ARG;
  *out = nullptr;
  if (!devices || n_devices < 1) return XRS_ERR_INVALID_ARG;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
    (void)hipGetLastError();
    return XRS_ERR_NO_DEVICE;
  }
  for (int i = 0; i < n_devices; ++i)
    if (devices[i] < 0 || devices[i] >= count) return XRS_ERR_INVALID_ARG;
  auto* g = new xrs_group();
  int prev = -1;
  (void)hipGetDevice(&prev);
  int e = XRS_OK;
  for (int i = 0; i < n_devices && !e; ++i) {
    if (hipSetDevice(devices[i]) != hipSuccess) {
      e = XRS_ERR_HIP;
      break;
    }
    xrs_codec* c = nullptr;
    e = xrs_new(data_num, parity_num, &c);  // binds c to devices[i]
    if (!e) {
      g->devices.push_back(devices[i]);
      g->codecs.push_back(c);
    }
  }
  if (prev >= 0) (void)hipSetDevice(prev);
  if (e) {
    xrs_group_free(g);
    return e;
  }
  *out = g;
  return XRS_OK;
}

void xrs_group_free(xrs_group* g) {
  if (!g) return;
  for (xrs_codec* c : g->codecs) xrs_free(c);
  delete g;
}

int xrs_group_size(const xrs_group* g) { return g ? static_cast<int>(g->codecs.size()) : 0; }

const xrs_codec* xrs_group_codec(const xrs_group* g, int i) {
  if (!g || i < 0 || i >= static_cast<int>(g->codecs.size())) return nullptr;
  return g->codecs[i];
}

// xrs.go:103 Encode over a host-resident batch, split across the group.
int xrs_group_encode_host(xrs_group* g, uint8_t* host_base, size_t size, size_t shard_stride,
                          size_t stripe_stride, size_t n_stripes) {
  if (!g) return XRS_ERR_INVALID_ARG;
  if (size & 1) return XRS_ERR_SIZE_NOT_EVEN;
  if (n_stripes == 0 || size == 0) return XRS_OK;
  if (!host_base) return XRS_ERR_INVALID_ARG;
  return for_members(g, n_stripes, [&](int i, size_t start, size_t count) {
    return xrs_encode_host(g->codecs[i], host_base + start * stripe_stride, size, shard_stride,
                           stripe_stride, count);
  });
}

// xrs.go:175 ReconstOne(k) over a host-resident batch, split across the group.
int xrs_group_reconst_one_host(xrs_group* g, uint8_t* host_base, size_t size, size_t shard_stride,
                               size_t stripe_stride, size_t n_stripes, int k) {
  if (!g) return XRS_ERR_INVALID_ARG;
  if (size & 1) return XRS_ERR_SIZE_NOT_EVEN;
  int an[256], alen = 0, bn[2];
  const int e = xrs_get_need_vects(g->codecs[0], k, an, &alen, bn);  // validates k
  if (e) return e;
  if (n_stripes == 0 || size == 0) return XRS_OK;
  if (!host_base) return XRS_ERR_INVALID_ARG;
  return for_members(g, n_stripes, [&](int i, size_t start, size_t count) {
    return xrs_reconst_one_host(g->codecs[i], host_base + start * stripe_stride, size,
                                shard_stride, stripe_stride, count, k);
  });
}

// xrs.go:236 Reconst(dpHas, need) over a host-resident batch, split across
// the group (validation and side effects: xrs_reconst_host).
int xrs_group_reconst_host(xrs_group* g, uint8_t* host_base, size_t size, size_t shard_stride,
                           size_t stripe_stride, size_t n_stripes, const int* dp_has, int n_has,
                           const int* need, int n_need) {
  if (!g || n_has < 0 || n_need < 0 || (n_has && !dp_has) || (n_need && !need))
    return XRS_ERR_INVALID_ARG;
  if (n_need == 1 && need[0] < xrs_data_num(g->codecs[0]))  // xrs.go:238-240
    return xrs_group_reconst_one_host(g, host_base, size, shard_stride, stripe_stride, n_stripes,
                                      need[0]);
  if (size & 1) return XRS_ERR_SIZE_NOT_EVEN;
  if (n_stripes == 0 || size == 0) return XRS_OK;
  if (!host_base) return XRS_ERR_INVALID_ARG;
  return for_members(g, n_stripes, [&](int i, size_t start, size_t count) {
    return xrs_reconst_host(g->codecs[i], host_base + start * stripe_stride, size, shard_stride,
                            stripe_stride, count, dp_has, n_has, need, n_need);
  });
}

// xrs.go:324 Update over host-resident rows, split across the group.
int xrs_group_update_host(xrs_group* g, const uint8_t* old_base, size_t old_stripe_stride,
                          const uint8_t* new_base, size_t new_stripe_stride, size_t size, int row,
                          uint8_t* parity_base, size_t parity_shard_stride,
                          size_t parity_stripe_stride, size_t n_stripes) {
  if (!g) return XRS_ERR_INVALID_ARG;
  if (size & 1) return XRS_ERR_SIZE_NOT_EVEN;
  if (row < 0 || row >= xrs_data_num(g->codecs[0])) return XRS_ERR_ILLEGAL_DATA_INDEX;
  if (n_stripes == 0 || size == 0) return XRS_OK;
  if (!old_base || !new_base || !parity_base) return XRS_ERR_INVALID_ARG;
  return for_members(g, n_stripes, [&](int i, size_t start, size_t count) {
    return xrs_update_host(g->codecs[i], old_base + start * old_stripe_stride, old_stripe_stride,
                           new_base + start * new_stripe_stride, new_stripe_stride, size, row,
                           parity_base + start * parity_stripe_stride, parity_shard_stride,
                           parity_stripe_stride, count);
  });
}

// xrs.go:363 Replace over host-resident rows, split across the group.
int xrs_group_replace_host(xrs_group* g, const uint8_t* data_base, size_t data_shard_stride,
                           size_t data_stripe_stride, const int* rows, int n, size_t size,
                           uint8_t* parity_base, size_t parity_shard_stride,
                           size_t parity_stripe_stride, size_t n_stripes) {
  if (!g) return XRS_ERR_INVALID_ARG;
  // same order as the single codec's check_replace (codec.cpp) and the oracle
  if (n < 1) return XRS_ERR_ILLEGAL_VECTS;
  if (size & 1) return XRS_ERR_SIZE_NOT_EVEN;
  if (n > xrs_data_num(g->codecs[0])) return XRS_ERR_ILLEGAL_VECTS;
  if (!rows) return XRS_ERR_INVALID_ARG;
  for (int i = 0; i < n; ++i)
    if (rows[i] < 0 || rows[i] >= xrs_data_num(g->codecs[0])) return XRS_ERR_ILLEGAL_DATA_INDEX;
  if (n_stripes == 0 || size == 0) return XRS_OK;
  if (!data_base || !parity_base) return XRS_ERR_INVALID_ARG;
  return for_members(g, n_stripes, [&](int i, size_t start, size_t count) {
    return xrs_replace_host(g->codecs[i], data_base + start * data_stripe_stride,
                            data_shard_stride, data_stripe_stride, rows, n, size,
                            parity_base + start * parity_stripe_stride, parity_shard_stride,
                            parity_stripe_stride, count);
  });
}

}  // extern "C"
