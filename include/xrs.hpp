// xrs.hpp -- C++ mirror of the Go method set of *xrs.XRS over the C ABI in
// xrs_hip.h (header-only).  Same names, argument meaning and error behaviour
// as /root/reference/xrs.go: every method returns an Error that is "nil"
// (false) on success and carries the Go message text otherwise.
//
//   std::unique_ptr<xrs::XRS> x;
//   if (auto err = xrs::XRS::New(12, 4, &x)) { ... err.msg ... }   // xrs.go:55
//   xrs::Vects vects(16, std::vector<uint8_t>(4096));
//   x->Encode(vects);                                             // xrs.go:103
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "xrs_hip.h"

namespace xrs {

// Go `error`: code 0 / empty message is nil.
struct Error {
  int code = 0;
  std::string msg;
  explicit operator bool() const { return code != 0; }
};

inline Error make_error(int rc, long long arg = 0) {
  Error e;
  e.code = rc;
  if (rc) {
    char buf[128];
    xrs_format_error(rc, arg, buf, sizeof buf);
    e.msg = buf;
  }
  return e;
}

using Vect = std::vector<uint8_t>;  // Go []byte
using Vects = std::vector<Vect>;    // Go [][]byte

// A non-owning []byte (Go slices such as vects[d:] alias the caller's data).
struct Slice {
  uint8_t* p;
  size_t n;
};

inline std::vector<uint8_t*> ptrs(std::vector<Slice>& v) {
  std::vector<uint8_t*> out;
  for (auto& s : v) out.push_back(s.p);
  return out;
}
inline std::vector<Slice> slices(Vects& v, size_t from = 0, size_t to = SIZE_MAX) {
  std::vector<Slice> out;
  for (size_t i = from; i < v.size() && i < to; ++i) out.push_back({v[i].data(), v[i].size()});
  return out;
}

// Every non-null slice of `v` is `n` bytes long.  The C ABI reads and writes
// `size` bytes of every vect, so a shorter one must be rejected here, before
// the call (the Go dependency rejects mismatched vects too: ILLEGAL_VECTS).
inline bool same_len(const std::vector<Slice>& v, size_t n) {
  for (const Slice& s : v)
    if (s.p && s.n != n) return false;
  return true;
}
// Size check first (xrs.go:105 checkSize runs before the dependency's checks).
inline bool lens_bad(const std::vector<Slice>& v, size_t n) { return !(n & 1) && !same_len(v, n); }

class XRS {
 public:
  // xrs.go:55 New(dataNum, parityNum)
  static Error New(int data_num, int parity_num, std::unique_ptr<XRS>* out) {
    xrs_codec* c = nullptr;
    const int rc = xrs_new(data_num, parity_num, &c);
    if (rc) return make_error(rc);
    out->reset(new XRS(c));
    return {};
  }
  ~XRS() { xrs_free(c_); }
  XRS(const XRS&) = delete;
  XRS& operator=(const XRS&) = delete;

  int DataNum() const { return xrs_data_num(c_); }      // x.RS.DataNum
  int ParityNum() const { return xrs_parity_num(c_); }  // x.RS.ParityNum
  const std::map<int, std::vector<int>>& XORSet() const { return xorset_; }  // xrs.go:49
  xrs_codec* codec() const { return c_; }

  // xrs.go:103
  Error Encode(std::vector<Slice> vects) {
    auto p = ptrs(vects);
    const size_t size = vects.empty() ? 0 : vects[0].n;
    if (lens_bad(vects, size)) return make_error(XRS_ERR_ILLEGAL_VECTS);
    return make_error(xrs_encode(c_, p.data(), static_cast<int>(p.size()), size),
                      static_cast<long long>(size));
  }
  Error Encode(Vects& vects) { return Encode(slices(vects)); }

  // xrs.go:146
  Error GetNeedVects(int k, std::vector<int>* a_need, std::vector<int>* b_need) const {
    std::vector<int> a(DataNum() > 0 ? DataNum() : 1);
    int n = 0, b[2] = {0, 0};
    const int rc = xrs_get_need_vects(c_, k, a.data(), &n, b);
    if (rc) return make_error(rc, k);
    a_need->assign(a.begin(), a.begin() + n);
    b_need->assign({b[0], b[1]});
    return {};
  }

  // xrs.go:175
  Error ReconstOne(std::vector<Slice> vects, int k) {
    auto p = ptrs(vects);
    const size_t size = vects.empty() ? 0 : vects[0].n;
    if (lens_bad(vects, size)) return make_error(XRS_ERR_ILLEGAL_VECTS);
    const int rc = xrs_reconst_one(c_, p.data(), static_cast<int>(p.size()), size, k);
    return make_error(rc, rc == XRS_ERR_SIZE_NOT_EVEN ? static_cast<long long>(size) : k);
  }
  Error ReconstOne(Vects& vects, int k) { return ReconstOne(slices(vects), k); }

  // xrs.go:236
  Error Reconst(std::vector<Slice> vects, const std::vector<int>& dp_has,
                const std::vector<int>& need) {
    auto p = ptrs(vects);
    const size_t size = vects.empty() ? 0 : vects[0].n;
    if (lens_bad(vects, size)) return make_error(XRS_ERR_ILLEGAL_VECTS);
    const int rc = xrs_reconst(c_, p.data(), static_cast<int>(p.size()), size, dp_has.data(),
                               static_cast<int>(dp_has.size()), need.data(),
                               static_cast<int>(need.size()));
    return make_error(rc, rc == XRS_ERR_SIZE_NOT_EVEN ? static_cast<long long>(size)
                                                      : (need.empty() ? 0 : need[0]));
  }
  Error Reconst(Vects& vects, const std::vector<int>& dp_has, const std::vector<int>& need) {
    return Reconst(slices(vects), dp_has, need);
  }

  // xrs.go:324
  Error Update(const Vect& old_data, const Vect& new_data, int row, std::vector<Slice> parity) {
    auto p = ptrs(parity);
    if (!(old_data.size() & 1) &&
        (new_data.size() != old_data.size() || !same_len(parity, old_data.size())))
      return make_error(XRS_ERR_ILLEGAL_VECTS);
    const int rc = xrs_update(c_, old_data.data(), new_data.data(), old_data.size(), row, p.data(),
                              static_cast<int>(p.size()));
    return make_error(rc, rc == XRS_ERR_SIZE_NOT_EVEN ? static_cast<long long>(old_data.size())
                                                      : row);
  }

  // xrs.go:363
  Error Replace(std::vector<Slice> data, const std::vector<int>& rows, std::vector<Slice> parity) {
    auto d = ptrs(data);
    auto p = ptrs(parity);
    const size_t size = data.empty() ? 0 : data[0].n;
    if (lens_bad(data, size) || lens_bad(parity, size)) return make_error(XRS_ERR_ILLEGAL_VECTS);
    const int rc = xrs_replace(c_, d.data(), rows.data(), static_cast<int>(rows.size()), size,
                               p.data(), static_cast<int>(p.size()));
    long long arg = 0;
    for (int r : rows)
      if (r < 0 || r >= DataNum()) {
        arg = r;
        break;
      }
    return make_error(rc, rc == XRS_ERR_SIZE_NOT_EVEN ? static_cast<long long>(size) : arg);
  }

 private:
  explicit XRS(xrs_codec* c) : c_(c) {
    const int d = DataNum(), p = ParityNum();
    std::vector<int> idx(d > 0 ? d : 1);
    for (int h = d + 1; h < d + p; ++h) {
      int n = 0;
      if (xrs_xorset(c_, h, idx.data(), d, &n) == 0 && n > 0)
        xorset_[h] = std::vector<int>(idx.begin(), idx.begin() + n);
    }
  }
  xrs_codec* c_;
  std::map<int, std::vector<int>> xorset_;
};

// Batching queue over a codec (xrs_queue_*): the same Encode / ReconstOne /
// Reconst / Update / Replace methods, callable from many threads at once; concurrent calls are
// coalesced into device batches (one per vect size `size`).
class Queue {
 public:
  static Error New(const XRS& x, size_t size, std::unique_ptr<Queue>* out,
                   size_t max_batch_stripes = 1024, int max_wait_us = 50) {
    xrs_queue* q = nullptr;
    const int rc = xrs_queue_new(x.codec(), size, max_batch_stripes, max_wait_us, &q);
    if (rc) return make_error(rc, static_cast<long long>(size));
    out->reset(new Queue(q, size, x.DataNum()));
    return {};
  }
  ~Queue() { xrs_queue_free(q_); }  // calls still in flight complete first
  Queue(const Queue&) = delete;
  Queue& operator=(const Queue&) = delete;

  // xrs.go:103
  Error Encode(std::vector<Slice> vects) {
    auto p = ptrs(vects);
    if (!same_len(vects, size_)) return make_error(XRS_ERR_ILLEGAL_VECTS);
    return make_error(xrs_queue_encode(q_, p.data(), static_cast<int>(p.size())),
                      static_cast<long long>(size_));
  }
  Error Encode(Vects& vects) { return Encode(slices(vects)); }
  // xrs.go:175
  Error ReconstOne(std::vector<Slice> vects, int k) {
    auto p = ptrs(vects);
    if (!same_len(vects, size_)) return make_error(XRS_ERR_ILLEGAL_VECTS);
    return make_error(xrs_queue_reconst_one(q_, p.data(), static_cast<int>(p.size()), k), k);
  }
  Error ReconstOne(Vects& vects, int k) { return ReconstOne(slices(vects), k); }
  // xrs.go:236 (batches keyed by the (dpHas, need) pattern)
  Error Reconst(std::vector<Slice> vects, const std::vector<int>& dp_has,
                const std::vector<int>& need) {
    auto p = ptrs(vects);
    if (!same_len(vects, size_)) return make_error(XRS_ERR_ILLEGAL_VECTS);
    const int rc = xrs_queue_reconst(q_, p.data(), static_cast<int>(p.size()), dp_has.data(),
                                     static_cast<int>(dp_has.size()), need.data(),
                                     static_cast<int>(need.size()));
    return make_error(rc, rc == XRS_ERR_SIZE_NOT_EVEN ? static_cast<long long>(size_)
                                                      : (need.empty() ? 0 : need[0]));
  }
  Error Reconst(Vects& vects, const std::vector<int>& dp_has, const std::vector<int>& need) {
    return Reconst(slices(vects), dp_has, need);
  }
  // xrs.go:363 (batches keyed by the rows set)
  Error Replace(std::vector<Slice> data, const std::vector<int>& rows, std::vector<Slice> parity) {
    auto d = ptrs(data);
    auto p = ptrs(parity);
    if (!same_len(data, size_) || !same_len(parity, size_)) return make_error(XRS_ERR_ILLEGAL_VECTS);
    const int rc = xrs_queue_replace(q_, d.data(), rows.data(), static_cast<int>(rows.size()),
                                     p.data(), static_cast<int>(p.size()));
    long long arg = 0;
    for (int r : rows)
      if (r < 0 || r >= codec_d_) {
        arg = r;
        break;
      }
    return make_error(rc, arg);
  }
  // xrs.go:324
  Error Update(const Vect& old_data, const Vect& new_data, int row, std::vector<Slice> parity) {
    auto p = ptrs(parity);
    if (old_data.size() != size_ || new_data.size() != size_ || !same_len(parity, size_))
      return make_error(XRS_ERR_ILLEGAL_VECTS);
    return make_error(xrs_queue_update(q_, old_data.data(), new_data.data(), row, p.data(),
                                       static_cast<int>(p.size())),
                      row);
  }
  // Asynchronous Encode / ReconstOne (xrs_queue_submit_*): the stripe is
  // staged now and *t set; t->Wait() blocks until it is done and returns the
  // call's error.  The vects must not be touched until then.  A submit that
  // finds every staging batch held by unwaited tickets returns the "queue
  // busy" error with nothing staged: Wait on an earlier ticket and resubmit.
  class Ticket {
   public:
    Ticket() = default;
    Ticket(const Ticket&) = delete;
    Ticket& operator=(const Ticket&) = delete;
    ~Ticket() { (void)Wait(); }
    bool Done() const { return !t_ || xrs_queue_poll(t_) == 1; }
    Error Wait() {
      if (!t_) return {};
      const int rc = xrs_queue_wait(t_);
      t_ = nullptr;
      return make_error(rc, arg_);
    }

   private:
    friend class Queue;
    xrs_queue_ticket* t_ = nullptr;
    long long arg_ = 0;
  };
  Error SubmitEncode(std::vector<Slice> vects, Ticket* t) {
    (void)t->Wait();
    auto p = ptrs(vects);
    if (!same_len(vects, size_)) return make_error(XRS_ERR_ILLEGAL_VECTS);
    t->arg_ = static_cast<long long>(size_);
    return make_error(xrs_queue_submit_encode(q_, p.data(), static_cast<int>(p.size()), &t->t_),
                      t->arg_);
  }
  Error SubmitReconstOne(std::vector<Slice> vects, int k, Ticket* t) {
    (void)t->Wait();
    auto p = ptrs(vects);
    if (!same_len(vects, size_)) return make_error(XRS_ERR_ILLEGAL_VECTS);
    t->arg_ = k;
    return make_error(xrs_queue_submit_reconst_one(q_, p.data(), static_cast<int>(p.size()), k, &t->t_),
                      k);
  }
  // Batches run so far by stripe count (xrs_queue_batch_sizes): element n =
  // batches of n stripes, the last element = batches of 64 or more.
  std::vector<uint64_t> BatchSizes() const {
    std::vector<uint64_t> c(65, 0);
    if (xrs_queue_batch_sizes(q_, c.data(), static_cast<int>(c.size())) != XRS_OK) c.clear();
    return c;
  }

 private:
  Queue(xrs_queue* q, size_t size, int d) : q_(q), size_(size), codec_d_(d) {}
  xrs_queue* q_;
  size_t size_;
  int codec_d_;
};

}  // namespace xrs
