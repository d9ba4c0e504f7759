// queue.cpp -- batching queue behind the per-stripe drop-in calls.
//
// A Go storage server calls x.Encode(vects) / x.ReconstOne(vects, k) per
// stripe from many goroutines.  One GPU launch per 4 KiB
// stripe is latency bound, so the queue coalesces concurrent per-stripe calls
// into device batches:
//
//   caller thread: reserve a slot in the open batch (under the queue mutex,
//     a few hundred ns) -> copy its vects into the batch's pinned staging
//     (callers copy in parallel) -> sleep on the batch's completion word (a
//     futex) -> copy its outputs back -> release the slot.
//   launcher threads (XRS_QUEUE_WORKERS, default 1): take a batch, wait for
//     its slots to be staged, enqueue it on the batch's own stream followed by
//     a write of the batch's sequence number to a pinned host word, and move
//     on: a launcher never waits for the GPU.
//     Batches of up to XRS_QUEUE_ZC_MAX bytes (default 4 MiB) skip both
//     copies: the kernel reads and writes the pinned, device-mapped staging
//     over PCIe (measured faster than DMA at these sizes);
//     larger ones get one H2D of the whole batch, one kernel and one D2H.
//   completion thread: spins on the in-flight batches' host words (no HIP
//     call on the fast path; hipStreamQuery now and then catches a failed
//     stream), and for each finished batch bumps its futex word: one wake
//     releases every caller of the batch at once.
//
// When a launcher closes the open batch (XRS_QUEUE_POLICY):
//   "free" (default): as soon as fewer than XRS_QUEUE_INFLIGHT (default 4)
//     batches are in flight, so each batch holds the calls that arrived
//     while the previous ones ran (sizes follow the load);
//   "timer": when it is full, when nothing is in flight (a lone caller does
//     not wait for company), or after max_wait_us.
// Completion latency, not bandwidth, bounds per-stripe calls at 4 KiB (a
// 28-stripe batch is 1.8 MB of PCIe traffic, ~35 us at 55 GB/s).  Measured on
// MI355X (tools/qlat_probe.hip, profiles/r03_queue_latency_probe.log): a
// spinning hipStreamQuery sees an empty kernel done 12-16 us after the launch
// call, a host word written by the stream 7.4 us after; the round-2 queue also
// woke a batch's callers through one condition variable and mutex (a chain of
// hand-offs, one context switch per caller).
//
// Every stripe's arithmetic is the batched device path (encode_dev /
// reconst_one_dev); results are bit-identical to the per-stripe calls.
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <linux/futex.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "hostreg.h"
#include "xrs_hip.h"

namespace xrs_detail {
int encode_dev(const xrs_codec* x, uint8_t* base, size_t size, size_t shard_stride,
               size_t stripe_stride, size_t n_stripes, void* stream);
int reconst_one_dev(const xrs_codec* x, uint8_t* base, size_t size, size_t shard_stride,
                    size_t stripe_stride, size_t n_stripes, int k, void* stream);
int need_set(const xrs_codec* x, int k, std::vector<int>* a_need, int* bi);
// table mode: the callers' rows through per-stripe row tables (codec.cpp)
int encode_table(const xrs_codec* x, const uint64_t* tab, size_t tab_stride, size_t size,
                 size_t n, void* stream);
int reconst_one_table(const xrs_codec* x, const uint64_t* tab, size_t tab_stride, size_t size,
                      size_t n, int k, void* stream);
int reconst_table(const xrs_codec* x, const uint64_t* tab, size_t tab_stride, size_t size, size_t n,
                  const int* dp_has, int n_has, const int* need, int n_need, void* stream);
int update_rows_table(const xrs_codec* x, const uint64_t* tab, size_t tab_stride, size_t size,
                      const int32_t* rows, size_t n, void* stream);
int replace_table(const xrs_codec* x, const uint64_t* tab, size_t tab_stride, const int* rows,
                  int n_rows, size_t size, size_t n, void* stream);
int copy_rows_mirror(bool to_device, uint8_t* dev, uint8_t* host, size_t pitch, size_t len,
                     size_t rows, void* stream);
int codec_device(const xrs_codec* x);
int codec_d(const xrs_codec* x);
int codec_p(const xrs_codec* x);
// xrs_reconst without the hand-over to a busy codec's auto queue
int reconst_direct(const xrs_codec* x, uint8_t* const* vects, int n, size_t size,
                   const int* dp_has, int n_has, const int* need, int n_need);
}  // namespace xrs_detail

using Clock = std::chrono::steady_clock;

namespace {

constexpr int kMaxWorkers = 8;   // launcher threads: XRS_QUEUE_WORKERS, default 1
constexpr int kBatches = 16;     // staging buffers: XRS_QUEUE_BATCHES, default in-flight + 2
constexpr int kFlagStride = 16;  // uint32 words between batches' host words (64 B)
constexpr size_t kMaxBatchBytes = 64u << 20;
constexpr uint64_t kStuckNs = 20000000;  // in flight this long: ask the stream for errors

// A 32-bit futex word: waiters sleep in the kernel until it changes, and one
// wake releases all of them together.
static_assert(sizeof(std::atomic<uint32_t>) == sizeof(uint32_t), "futex word");
void futex_wait(std::atomic<uint32_t>* w, uint32_t v) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAIT_PRIVATE, v, nullptr, nullptr, 0);
}
void futex_wake_all(std::atomic<uint32_t>* w) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAKE_PRIVATE, INT_MAX, nullptr, nullptr,
          0);
}

uint64_t ns_since(Clock::time_point t0) {
  return static_cast<uint64_t>(
      std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - t0).count());
}

// Spin (pause) for about `spin_ns`, then yield, until pred() holds.
template <class F>
void spin_until(F pred, uint64_t spin_ns) {
  const auto t0 = Clock::now();
  for (int i = 0; !pred(); ++i) {
    if ((i & 63) == 63 && ns_since(t0) > spin_ns)
      std::this_thread::yield();
    else
      _mm_pause();
  }
}

enum State { FREE, OPEN, CLOSED, LAUNCHING, INFLIGHT, DONE };

struct Batch {
  uint8_t* host = nullptr;      // pinned staging, compact [stripe][shard][size]
  uint8_t* host_dev = nullptr;  // its device address (zero-copy batches)
  uint8_t* dev = nullptr;
  int32_t* rows = nullptr;      // pinned, mapped: Update's data row per slot
  int32_t* rows_dev = nullptr;  // its device address (read by the kernel)
  // Row tables (pinned, mapped; per slot, two entries per staged row: the
  // device addresses of its a-half and b-half) -- the caller's own vect when
  // it lies in registered memory (hostreg.h), else the slot's row in `host`.
  // A batch with any registered slot runs its kernels through the tables, in
  // place on the callers' buffers over PCIe (indirect rows, xrs_plan.h).
  uint64_t* tab = nullptr;
  uint64_t* tab_dev = nullptr;
  hipStream_t stream = nullptr;
  volatile uint32_t* flag = nullptr;  // pinned host word the stream writes `launches` to
  uint32_t* flag_dev = nullptr;
  uint32_t launches = 0;
  // guarded by the queue mutex
  State state = FREE;
  int key = -1;  // 0: encode, 1 + k: reconst_one(k), 1 + d: update (any rows),
                 // 2 + d: reconst(pat_has, pat_need), 3 + d: replace(pat_has = rows)
  std::vector<int> pat_has, pat_need;  // Reconst pattern of the batch
  size_t reserved = 0;
  Clock::time_point opened, launched;
  // lock-free: slots staged / slots released, and the completion word (+1
  // when the batch's results are in staging; err and n are written first)
  std::atomic<uint32_t> filled{0}, released{0}, done{0};
  std::atomic<uint32_t> n_reg{0};  // slots whose vects are all in registered memory
  // Asynchronous registered slots (nothing to copy back): released by the
  // completion thread itself when the batch succeeds, so their batch is
  // recycled without waiting for the tickets' owners (auto_st[slot]: the
  // ticket's status word, else nullptr).
  std::vector<std::atomic<int>*> auto_st;
  std::atomic<uint32_t> n_auto{0};
  size_t n = 0;  // slots of the closed batch
  int err = 0;
};

}  // namespace

struct xrs_queue {
  const xrs_codec* codec = nullptr;
  int d = 0, p = 0, device = -1;
  size_t size = 0, stripe_bytes = 0, max_batch = 1, zc_max = 0;
  size_t bo = 0;  // staged stripes start at the odd-size base offset (b-halves aligned)
  size_t nrows = 0;     // staged rows per stripe (stripe_bytes / size)
  bool reg_ok = false;  // row tables allocated: registered callers skip the copies
  std::chrono::microseconds max_wait{50};
  Batch b[kBatches];
  uint32_t* flags = nullptr;  // pinned, mapped: kFlagStride words per batch
  int open = -1;
  int in_flight = 0;  // batches launching or in flight (guarded by mu)
  std::atomic<uint32_t> inflight_bits{0};  // bit i: batch i waits for its host word
  std::atomic<int> active{0};  // callers inside submit() (xrs_queue_free waits for 0)
  bool stop = false, comp_stop = false;
  // statistics (guarded by mu): batches run, stripes run, device time
  // (launch to completion seen) and queueing time (open to launch) summed
  // over batches, in ns
  uint64_t st_batches = 0, st_stripes = 0, st_run_ns = 0, st_wait_ns = 0;
  // batches run by stripe count (index n: n stripes; the last bucket: more)
  static constexpr int kHist = 65;
  static constexpr int kMaxRows = 258;  // staged rows per stripe: max(d + p, p + 2) <= 258
  uint64_t st_hist[kHist] = {};
  std::mutex mu;
  std::condition_variable cv_work, cv_free, cv_comp;
  std::thread worker[kMaxWorkers], completer;
  int n_workers = 1, n_batches = 6, max_inflight = 4;
  bool timer = false;        // XRS_QUEUE_POLICY=timer
  uint64_t spin_ns = 20000;  // launcher spin (staging fills) before yielding
  uint64_t comp_spin_ns = 200000;  // completion thread spin before yielding

  // One copy between a caller's buffer and its staged stripe: `len` bytes at
  // staging row `row` (row * size + off) <-> host + off.
  struct Piece {
    uint8_t* host;
    int row;
    size_t off, len;
  };

  int launch(Batch& bt);
  void work();
  void complete();
  void finish(int i, int err);
  void close_open() {  // (mu held)
    b[open].state = CLOSED;
    b[open].n = b[open].reserved;
    open = -1;
    cv_work.notify_one();
  }
  void leave() {
    if (active.fetch_sub(1, std::memory_order_acq_rel) == 1) {
      std::lock_guard<std::mutex> lk(mu);
      if (stop) cv_free.notify_all();
    }
  }
  // A staged call: its batch, slot and the batch's completion count when it
  // was reserved, and the pieces to copy back after the batch ran.
  struct Staged {
    Batch* bt = nullptr;
    size_t slot = 0;
    uint32_t seq = 0;
    bool reg = false;  // the call's vects are registered: no copies
    std::atomic<int>* status = nullptr;  // auto-released slot: 0 once done
    std::vector<Piece> out;
  };
  // Reserve a slot and stage the call (no wait).  nonblock: XRS_ERR_BUSY
  // instead of waiting for a free staging batch.
  int stage(int key, const std::vector<Piece>& in, const std::vector<Piece>& out, int row,
            const std::vector<int>* has, const std::vector<int>* need, bool nonblock, Staged* sc,
            std::atomic<int>* status = nullptr);
  // Wait for a staged call's batch, copy its outputs back, release the slot.
  int wait(Staged& sc);
  int submit(int key, const std::vector<Piece>& in, const std::vector<Piece>& out, int row = -1,
             const std::vector<int>* has = nullptr, const std::vector<int>* need = nullptr) {
    Staged sc;
    const int e = stage(key, in, out, row, has, need, false, &sc);
    return e ? e : wait(sc);
  }
  // The synchronous call (t == nullptr) or its asynchronous form (*t: a
  // ticket for xrs_queue_wait).
  int run(int key, const std::vector<Piece>& in, const std::vector<Piece>& out, int row,
          const std::vector<int>* has, const std::vector<int>* need, xrs_queue_ticket** t);
};

// An asynchronous call (xrs_queue_submit_*): staged in a batch, or already
// finished (st.bt == nullptr: a call the queue ran directly, status `err`).
struct xrs_queue_ticket {
  xrs_queue* q = nullptr;
  xrs_queue::Staged st;
  int err = 0;
  std::atomic<int> status{-1};  // (registered vects: set to 0 by the completion thread)
};

int xrs_queue::run(int key, const std::vector<Piece>& in, const std::vector<Piece>& out, int row,
                   const std::vector<int>* has, const std::vector<int>* need,
                   xrs_queue_ticket** t) {
  if (!t) return submit(key, in, out, row, has, need);
  *t = nullptr;
  auto* tk = new xrs_queue_ticket();
  tk->q = this;
  const int e = stage(key, in, out, row, has, need, true, &tk->st, &tk->status);
  if (e) {
    delete tk;
    return e;
  }
  *t = tk;
  return XRS_OK;
}

// Enqueue batch bt on its stream, ending with the write of its sequence
// number to its host word.  Returns an XRS error if anything failed to
// enqueue (then no host word write is pending).
int xrs_queue::launch(Batch& bt) {
  const size_t n = bt.n;
  // Encode: only the data rows go up and only the parity rows come back (one
  // 2-D copy each); ReconstOne: the whole staged stripe up, vect k back;
  // Update(row): parity rows, old and new up (rows [0, p+2)), parity back.
  const bool enc = bt.key == 0, upd = bt.key == 1 + d, rec = bt.key == 2 + d,
             rep = bt.key == 3 + d;
  const size_t up_off = 0;
  // Replace(rows): parity rows [0, p) and the n data rows [p, p+n) up, parity back.
  const size_t up_len = enc   ? static_cast<size_t>(d) * size
                        : upd ? static_cast<size_t>(p + 2) * size
                        : rep ? (p + bt.pat_has.size()) * size
                              : stripe_bytes;
  const size_t dn_off = enc ? static_cast<size_t>(d) * size
                            : upd || rec || rep ? 0 : static_cast<size_t>(bt.key - 1) * size;
  const size_t dn_len = enc || upd || rep ? static_cast<size_t>(p) * size
                                          : rec ? static_cast<size_t>(d + p) * size : size;
  // Registered callers: the kernels read and write the callers' own buffers
  // (and unregistered slots' pinned staging) through the row tables, in
  // place over PCIe, one launch as in zero-copy mode (XRS_QUEUE_REG=0: never).
  const bool table = reg_ok && bt.n_reg.load(std::memory_order_acquire) > 0;
  const bool zc = !table && bt.host_dev && n * stripe_bytes <= zc_max;
  uint8_t* base = (zc ? bt.host_dev : bt.dev) + bo;
  uint8_t *hst = bt.host + bo, *dst = bt.dev + bo;
  int e = 0;
  if (table) {
    const size_t ts = 2 * nrows * sizeof(uint64_t);
    if (enc)
      e = xrs_detail::encode_table(codec, bt.tab_dev, ts, size, n, bt.stream);
    else if (rep)
      e = xrs_detail::replace_table(codec, bt.tab_dev, ts, bt.pat_has.data(),
                                    static_cast<int>(bt.pat_has.size()), size, n, bt.stream);
    else if (rec)
      e = xrs_detail::reconst_table(codec, bt.tab_dev, ts, size, n, bt.pat_has.data(),
                                    static_cast<int>(bt.pat_has.size()), bt.pat_need.data(),
                                    static_cast<int>(bt.pat_need.size()), bt.stream);
    else if (upd)
      e = xrs_detail::update_rows_table(codec, bt.tab_dev, ts, size, bt.rows_dev, n, bt.stream);
    else
      e = xrs_detail::reconst_one_table(codec, bt.tab_dev, ts, size, n, bt.key - 1, bt.stream);
  } else {
    if (!zc)  // (odd sizes: rows start at an aligned word, codec.cpp copy_rows)
      e = xrs_detail::copy_rows_mirror(true, dst + up_off, hst + up_off, stripe_bytes, up_len, n,
                                       bt.stream);
    if (!e) {
      if (enc)
        e = xrs_detail::encode_dev(codec, base, size, size, stripe_bytes, n, bt.stream);
      else if (rep)
        e = xrs_replace_batched(codec, base + static_cast<size_t>(p) * size, size, stripe_bytes,
                                bt.pat_has.data(), static_cast<int>(bt.pat_has.size()), size, base,
                                size, stripe_bytes, n, bt.stream);
      else if (rec)
        e = xrs_reconst_batched(codec, base, size, size, stripe_bytes, n, bt.pat_has.data(),
                                static_cast<int>(bt.pat_has.size()), bt.pat_need.data(),
                                static_cast<int>(bt.pat_need.size()), bt.stream);
      else if (upd)  // one launch for every row: each stripe carries its own
        e = xrs_update_rows_batched(codec, base + static_cast<size_t>(p) * size, stripe_bytes,
                                    base + static_cast<size_t>(p + 1) * size, stripe_bytes, size,
                                    bt.rows_dev, base, size, stripe_bytes, n, bt.stream);
      else
        e = xrs_detail::reconst_one_dev(codec, base, size, size, stripe_bytes, n, bt.key - 1,
                                        bt.stream);
    }
    if (!e && !zc)
      e = xrs_detail::copy_rows_mirror(false, dst + dn_off, hst + dn_off, stripe_bytes, dn_len, n,
                                       bt.stream);
  }
  if (!e && hipStreamWriteValue32(bt.stream, bt.flag_dev, ++bt.launches, 0) != hipSuccess)
    e = XRS_ERR_HIP;
  if (e) (void)hipStreamSynchronize(bt.stream);  // nothing of it may still run
  return e;
}

// Batch i's results are in staging (or it failed): release its callers.
void xrs_queue::finish(int i, int err) {
  Batch& bt = b[i];
  const size_t n = bt.n;
  const uint32_t n_auto = err ? 0 : bt.n_auto.load(std::memory_order_relaxed);
  {
    std::lock_guard<std::mutex> lk(mu);
    bt.err = err;
    bt.state = DONE;
    --in_flight;
    ++st_batches;
    st_stripes += n;
    ++st_hist[std::min<size_t>(n, kHist - 1)];
    st_run_ns += ns_since(bt.launched);
    cv_work.notify_one();  // a launcher may wait for in_flight < max_inflight
  }
  if (n_auto)  // asynchronous registered calls: done, nothing to copy back
    for (size_t j = 0; j < n; ++j)
      if (bt.auto_st[j]) bt.auto_st[j]->store(0, std::memory_order_relaxed);
  bt.done.fetch_add(1, std::memory_order_release);
  futex_wake_all(&bt.done);
  // their slots are released here, after the completion count moved (a batch
  // recycled before it would wake the next calls' waiters), once per slot
  if (n_auto && bt.released.fetch_add(n_auto, std::memory_order_acq_rel) + n_auto == n) {
    std::lock_guard<std::mutex> lk(mu);
    bt.state = FREE;
    cv_free.notify_all();
  }
}

void xrs_queue::work() {
  if (device >= 0) (void)hipSetDevice(device);
  std::unique_lock<std::mutex> lk(mu);
  for (;;) {
    int pick = -1;
    bool pending = false;  // a batch some caller still waits on
    Clock::time_point next = Clock::now() + max_wait;
    for (int i = 0; i < n_batches && pick < 0; ++i) {
      Batch& bt = b[i];
      if (bt.state == OPEN || bt.state == CLOSED) pending = true;
      if (bt.state == CLOSED) pick = i;
      if (bt.state == OPEN && bt.reserved > 0) {
        // (stopping: drain, every caller already in gets its result)
        bool go = stop;
        if (!go && !timer) {
          go = in_flight < max_inflight;
        } else if (!go) {
          // timer: a small batch runs at once when nothing is in flight;
          // otherwise, and for large stripes (PCIe-bound, where bigger
          // batches measured faster), it grows until max_wait has passed.
          const auto due = bt.opened + max_wait;
          go = (in_flight == 0 && bt.reserved * stripe_bytes <= zc_max) || Clock::now() >= due;
          if (!go) next = std::min(next, due);
        }
        if (go) {
          close_open();
          pick = i;
        }
      }
    }
    if (pick < 0) {
      if (stop && !pending) break;
      cv_work.wait_until(lk, next);
      continue;
    }
    Batch& bt = b[pick];
    bt.state = LAUNCHING;
    ++in_flight;
    const size_t n = bt.n;
    lk.unlock();
    // the batch's callers are still copying in (a few us at 4 KiB)
    spin_until([&] { return bt.filled.load(std::memory_order_acquire) == n; }, spin_ns);
    bt.launched = Clock::now();
    const uint64_t waited = std::chrono::duration_cast<std::chrono::nanoseconds>(
                                bt.launched - bt.opened).count();
    const int e = launch(bt);
    lk.lock();
    st_wait_ns += waited;
    if (e) {
      lk.unlock();
      finish(pick, e);
      lk.lock();
      continue;
    }
    bt.state = INFLIGHT;
    inflight_bits.fetch_or(1u << pick, std::memory_order_release);
    cv_comp.notify_one();
  }
}

void xrs_queue::complete() {
  if (device >= 0) (void)hipSetDevice(device);
  for (;;) {
    {
      std::unique_lock<std::mutex> lk(mu);
      cv_comp.wait(lk, [&] {
        return inflight_bits.load(std::memory_order_acquire) != 0 || (comp_stop && in_flight == 0);
      });
      if (inflight_bits.load(std::memory_order_acquire) == 0) return;  // stopping, drained
    }
    // Spin on the host words of every batch in flight (new launches join the
    // mask as they happen) until none is left.  A failed stream never writes
    // its word, so a batch still waiting after kStuckNs gets hipStreamQuery
    // checks (which are not free: spinning on hipStreamQuery saw an empty
    // kernel done 5-9 us later than its host word, r03_queue_latency_probe).
    auto idle = Clock::now();
    bool slept = false;
    for (uint32_t it = 1;; ++it) {
      uint32_t bits = inflight_bits.load(std::memory_order_acquire);
      if (!bits) break;
      bool any = false;
      const bool poll = slept || (it & 1023) == 0;
      slept = false;
      for (uint32_t m = bits; m; m &= m - 1) {
        const int i = __builtin_ctz(m);
        Batch& bt = b[i];
        int err = -1;
        if (*bt.flag == bt.launches) {
          err = 0;
        } else if (poll && ns_since(bt.launched) > kStuckNs) {
          const hipError_t q = hipStreamQuery(bt.stream);
          if (q == hipSuccess) err = *bt.flag == bt.launches ? 0 : XRS_ERR_HIP;
          else if (q != hipErrorNotReady) err = XRS_ERR_HIP;
        }
        if (err < 0) continue;
        std::atomic_thread_fence(std::memory_order_acquire);  // staging after the word
        inflight_bits.fetch_and(~(1u << i), std::memory_order_acq_rel);
        finish(i, err);
        any = true;
      }
      if (any) {
        idle = Clock::now();
      } else if (ns_since(idle) > comp_spin_ns) {
        // a long batch (large stripes over PCIe): sleep between polls instead
        // of burning a core.  A 20 us sleep lasts 70-80 us under Linux's
        // default 50 us timer slack, which a batch that already ran > 200 us
        // can absorb; the stuck-stream check runs on every sleeping pass.
        std::this_thread::sleep_for(std::chrono::microseconds(20));
        slept = true;
      } else {
        _mm_pause();
      }
    }
  }
}

int xrs_queue::stage(int key, const std::vector<Piece>& in, const std::vector<Piece>& out, int row,
                     const std::vector<int>* has, const std::vector<int>* need, bool nonblock,
                     Staged* sc, std::atomic<int>* status) {
  auto same_pattern = [&](const Batch& bt) {
    return !has || (bt.pat_has == *has && bt.pat_need == *need);
  };
  // Device address of each staged row's vect when every vect of the call lies
  // in registered host memory (hostreg.h): then no copy on this thread.
  uint64_t regdev[xrs_queue::kMaxRows];
  bool reg = reg_ok;
  if (reg) {
    const xrs_detail::HostRangesView ranges;
    for (const auto* ps : {&in, &out})
      for (const Piece& pc : *ps)
        if (reg) {
          const uint64_t a = ranges.device(pc.host, size);
          reg = a != 0 && pc.row >= 0 && static_cast<size_t>(pc.row) < nrows;
          if (reg) regdev[pc.row] = a;
        }
  }
  Batch* bp;
  size_t slot;
  uint32_t seq;
  {
    std::unique_lock<std::mutex> lk(mu);
    if (stop) return XRS_ERR_INVALID_ARG;
    active.fetch_add(1, std::memory_order_relaxed);
    for (;;) {
      if (stop) {
        lk.unlock();
        leave();
        return XRS_ERR_INVALID_ARG;
      }
      if (open >= 0 && b[open].key == key && b[open].reserved < max_batch && same_pattern(b[open]))
        break;
      if (open >= 0) close_open();  // different op or full: a launcher runs it
      int f = -1;
      for (int i = 0; i < n_batches && f < 0; ++i)
        if (b[i].state == FREE) f = i;
      if (f < 0) {
        if (nonblock) {  // (xrs_queue_submit_*: the caller waits on a ticket first)
          lk.unlock();
          leave();
          return XRS_ERR_BUSY;
        }
        cv_free.wait(lk);
        continue;
      }
      Batch& nb = b[f];
      nb.state = OPEN;
      nb.key = key;
      nb.reserved = nb.n = 0;
      nb.filled.store(0, std::memory_order_relaxed);
      nb.released.store(0, std::memory_order_relaxed);
      nb.err = 0;
      nb.n_reg.store(0, std::memory_order_relaxed);
      nb.n_auto.store(0, std::memory_order_relaxed);
      nb.opened = Clock::now();
      if (has) {
        nb.pat_has = *has;
        nb.pat_need = *need;
      }
      open = f;
      if (!timer) cv_work.notify_one();  // a free launcher takes it at once
    }
    bp = &b[open];
    slot = bp->reserved++;
    seq = bp->done.load(std::memory_order_relaxed);
    if (bp->reserved == max_batch) close_open();
  }
  Batch& bt = *bp;
  uint8_t* st = bt.host + bo + slot * stripe_bytes;
  if (row >= 0) bt.rows[slot] = row;
  if (reg_ok) {  // the slot's row table: a- and b-half of every row it uses
    uint64_t* tb = bt.tab + slot * 2 * nrows;
    const uint64_t sd = reinterpret_cast<uint64_t>(bt.host_dev + bo + slot * stripe_bytes);
    for (const auto* ps : {&in, &out})
      for (const Piece& pc : *ps) {
        const uint64_t a = reg ? regdev[pc.row] : sd + static_cast<uint64_t>(pc.row) * size;
        tb[2 * pc.row] = a;
        tb[2 * pc.row + 1] = a + size / 2;
      }
    if (reg) bt.n_reg.fetch_add(1, std::memory_order_relaxed);
  }
  // (every reservation sets its entry: the vector keeps entries of earlier batches)
  bt.auto_st[slot] = reg && status ? status : nullptr;
  if (reg && status) bt.n_auto.fetch_add(1, std::memory_order_relaxed);
  if (!reg)
    for (const Piece& pc : in)
      std::memcpy(st + static_cast<size_t>(pc.row) * size + pc.off, pc.host + pc.off, pc.len);
  bt.filled.fetch_add(1, std::memory_order_release);
  if (timer) {
    // the timer policy's launcher may be asleep on a batch that is now staged
    std::lock_guard<std::mutex> lk(mu);
    cv_work.notify_one();
  }
  sc->bt = &bt;
  sc->slot = slot;
  sc->seq = seq;
  sc->reg = reg;
  sc->status = reg && status ? status : nullptr;
  sc->out = out;
  return XRS_OK;
}

int xrs_queue::wait(Staged& sc) {
  Batch& bt = *sc.bt;
  const uint32_t seq = sc.seq;
  const bool reg = sc.reg;
  const std::vector<Piece>& out = sc.out;
  uint8_t* st = bt.host + bo + sc.slot * stripe_bytes;
  while (bt.done.load(std::memory_order_acquire) == seq) futex_wait(&bt.done, seq);
  if (sc.status && sc.status->load(std::memory_order_acquire) == 0) {
    // released by the completion thread (the batch may be running new calls
    // already): nothing of it is touched here
    leave();
    return XRS_OK;
  }
  // The batch cannot be recycled before this caller's own release below, so
  // its slot count and status are read here, once: after the release another
  // caller may free the batch and a new submit() reopen it (n = 0).
  const size_t n_slots = bt.n;
  const int err = bt.err;
  if (!err && !reg)
    for (const Piece& pc : out)
      std::memcpy(pc.host + pc.off, st + static_cast<size_t>(pc.row) * size + pc.off, pc.len);
  if (bt.released.fetch_add(1, std::memory_order_acq_rel) + 1 == n_slots) {
    std::lock_guard<std::mutex> lk(mu);
    bt.state = FREE;
    cv_free.notify_all();
  }
  leave();
  return err;
}

extern "C" {

int xrs_queue_new(const xrs_codec* codec, size_t size, size_t max_batch_stripes, int max_wait_us,
                  xrs_queue** out) {
  if (!codec || !out || (size & 1) || size == 0 || max_wait_us < 0) return XRS_ERR_INVALID_ARG;
  *out = nullptr;
  const int dev = xrs_detail::codec_device(codec);
  if (dev < 0) return XRS_ERR_NO_DEVICE;
  auto* q = new xrs_queue();
  q->codec = codec;
  q->d = xrs_detail::codec_d(codec);
  q->p = xrs_detail::codec_p(codec);
  q->device = dev;
  q->size = size;
  // A staged stripe holds d+p vects (Encode, ReconstOne) or p parity + old +
  // new (Update): p+2 rows, more than d+p only when d == 1.
  q->stripe_bytes = static_cast<size_t>(std::max(q->d + q->p, q->p + 2)) * size;
  // xrs_batch_layout's base offset: with an odd half (size % 32 != 0) every
  // staged b-half is as aligned as in a recommended device batch
  q->bo = (16 - (size / 2) % 16) % 16;
  q->nrows = q->stripe_bytes / size;
  q->max_batch = std::max<size_t>(
      1, std::min(max_batch_stripes ? max_batch_stripes : SIZE_MAX, kMaxBatchBytes / q->stripe_bytes));
  q->max_wait = std::chrono::microseconds(max_wait_us);
  const char* zv = std::getenv("XRS_QUEUE_ZC_MAX");
  q->zc_max = (zv && *zv) ? static_cast<size_t>(std::strtoull(zv, nullptr, 0)) : (4u << 20);
  auto env_int = [](const char* v, int lo, int hi, int def) {
    const char* e = std::getenv(v);
    return (e && *e) ? std::max(lo, std::min(hi, std::atoi(e))) : def;
  };
  q->n_workers = env_int("XRS_QUEUE_WORKERS", 1, kMaxWorkers, 1);
  q->max_inflight = env_int("XRS_QUEUE_INFLIGHT", 1, kBatches - 1, 4);
  q->n_batches = env_int("XRS_QUEUE_BATCHES", 2, kBatches, std::min(kBatches, q->max_inflight + 2));
  const char* pv = std::getenv("XRS_QUEUE_POLICY");
  q->timer = pv && std::strcmp(pv, "timer") == 0;
  const char* nv = std::getenv("XRS_QUEUE_SPIN_NS");
  if (nv && *nv) q->spin_ns = std::strtoull(nv, nullptr, 0);
  const char* rv = std::getenv("XRS_QUEUE_REG");
  q->reg_ok = !(rv && rv[0] == '0');
  int prev = -1;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(dev);
  int e = XRS_OK;
  void* fp = nullptr;
  if (hipHostMalloc(reinterpret_cast<void**>(&q->flags), kBatches * kFlagStride * sizeof(uint32_t),
                    hipHostMallocMapped) != hipSuccess ||
      hipHostGetDevicePointer(&fp, q->flags, 0) != hipSuccess)
    e = XRS_ERR_HIP;
  for (int i = 0; i < q->n_batches && !e; ++i) {
    Batch& bt = q->b[i];
    bt.flag = q->flags + i * kFlagStride;
    *bt.flag = 0;
    bt.flag_dev = static_cast<uint32_t*>(fp) + i * kFlagStride;
    if (hipHostMalloc(&bt.host, q->max_batch * q->stripe_bytes + q->bo, hipHostMallocMapped) != hipSuccess ||
        hipMalloc(&bt.dev, q->max_batch * q->stripe_bytes + q->bo) != hipSuccess ||
        hipStreamCreateWithFlags(&bt.stream, hipStreamNonBlocking) != hipSuccess) {
      e = XRS_ERR_HIP;
      break;
    }
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, bt.host, 0) == hipSuccess) bt.host_dev = static_cast<uint8_t*>(dp);
    if (hipHostMalloc(&bt.rows, q->max_batch * sizeof(int32_t), hipHostMallocMapped) != hipSuccess ||
        hipHostGetDevicePointer(&dp, bt.rows, 0) != hipSuccess) {
      e = XRS_ERR_HIP;
      break;
    }
    bt.rows_dev = static_cast<int32_t*>(dp);
    bt.auto_st.assign(q->max_batch, nullptr);
    // row tables for registered callers (at most 16 MiB per batch, else the
    // queue copies every call through `host`; XRS_QUEUE_REG=0: always)
    const size_t tb = q->max_batch * 2 * q->nrows * sizeof(uint64_t);
    if (q->reg_ok && tb <= (16u << 20) &&
        hipHostMalloc(reinterpret_cast<void**>(&bt.tab), tb, hipHostMallocMapped) == hipSuccess &&
        hipHostGetDevicePointer(&dp, bt.tab, 0) == hipSuccess && bt.host_dev) {
      bt.tab_dev = static_cast<uint64_t*>(dp);
    } else {
      (void)hipGetLastError();
      q->reg_ok = false;
    }
  }
  if (prev >= 0) (void)hipSetDevice(prev);
  if (e) {
    xrs_queue_free(q);
    return e;
  }
  q->completer = std::thread([q] { q->complete(); });
  for (int i = 0; i < q->n_workers; ++i) q->worker[i] = std::thread([q] { q->work(); });
  *out = q;
  return XRS_OK;
}

void xrs_queue_free(xrs_queue* q) {
  if (!q) return;
  {
    // New calls fail from here on; calls already holding a slot complete
    // (the launchers drain every open batch before they exit, the completion
    // thread every batch in flight), and the queue
    // is torn down only after the last caller has left submit().
    std::unique_lock<std::mutex> lk(q->mu);
    q->stop = true;
    q->cv_work.notify_all();
    q->cv_free.notify_all();
    q->cv_free.wait(lk, [q] { return q->active.load() == 0; });
  }
  for (auto& w : q->worker)
    if (w.joinable()) w.join();
  {
    std::lock_guard<std::mutex> lk(q->mu);
    q->comp_stop = true;
    q->cv_comp.notify_all();
  }
  if (q->completer.joinable()) q->completer.join();
  int prev = -1;
  (void)hipGetDevice(&prev);
  if (q->device >= 0) (void)hipSetDevice(q->device);
  for (Batch& bt : q->b) {
    if (bt.stream) (void)hipStreamDestroy(bt.stream);
    if (bt.dev) (void)hipFree(bt.dev);
    if (bt.host) (void)hipHostFree(bt.host);
    if (bt.rows) (void)hipHostFree(bt.rows);
    if (bt.tab) (void)hipHostFree(bt.tab);
  }
  if (q->flags) (void)hipHostFree(q->flags);
  if (prev >= 0) (void)hipSetDevice(prev);
  delete q;
}

// xrs.go:103 Encode, coalesced with concurrent callers: data rows in,
// parity rows out.
static int queue_encode(xrs_queue* q, uint8_t* const* vects, int n, xrs_queue_ticket** t) {
  if (!q) return XRS_ERR_INVALID_ARG;
  if (!vects || n != q->d + q->p) return XRS_ERR_ILLEGAL_VECTS;
  for (int i = 0; i < n; ++i)
    if (!vects[i]) return XRS_ERR_INVALID_ARG;
  std::vector<xrs_queue::Piece> in, out;
  for (int j = 0; j < q->d; ++j) in.push_back({vects[j], j, 0, q->size});
  for (int r = 0; r < q->p; ++r) out.push_back({vects[q->d + r], q->d + r, 0, q->size});
  return q->run(0, in, out, -1, nullptr, nullptr, t);
}

// xrs.go:175 ReconstOne, coalesced: only the GetNeedVects set is copied in
// (b-halves of the d survivors and of parity bi, a-halves of aNeed), vect k
// out.
static int queue_reconst_one(xrs_queue* q, uint8_t* const* vects, int n, int k, xrs_queue_ticket** t) {
  if (!q) return XRS_ERR_INVALID_ARG;
  if (k < 0 || k >= q->d) return XRS_ERR_ILLEGAL_DATA_INDEX;
  if (!vects || n != q->d + q->p) return XRS_ERR_ILLEGAL_VECTS;
  for (int i = 0; i < n; ++i)
    if (!vects[i]) return XRS_ERR_INVALID_ARG;
  std::vector<int> a_need;
  int bi = 0;
  const int e = xrs_detail::need_set(q->codec, k, &a_need, &bi);
  if (e) return e;
  const size_t half = q->size / 2;
  std::vector<xrs_queue::Piece> in, out;
  for (int m = 0; m < q->d; ++m) {
    const int h = m == k ? q->d : m;
    in.push_back({vects[h], h, half, half});
  }
  in.push_back({vects[bi], bi, half, half});
  for (int a : a_need) in.push_back({vects[a], a, 0, half});
  out.push_back({vects[k], k, 0, q->size});
  return q->run(1 + k, in, out, -1, nullptr, nullptr, t);
}

// xrs.go:324 Update(oldData, newData, row, parity), coalesced across rows
// (each staged stripe carries its own row: update_rows kernel): staged rows
// [0, p) parity, p old, p+1 new; parity out.
static int queue_update(xrs_queue* q, const uint8_t* old_data, const uint8_t* new_data, int row,
                         uint8_t* const* parity, int n_parity, xrs_queue_ticket** t) {
  if (!q) return XRS_ERR_INVALID_ARG;
  if (row < 0 || row >= q->d) return XRS_ERR_ILLEGAL_DATA_INDEX;
  if (!parity || n_parity != q->p) return XRS_ERR_ILLEGAL_VECTS;
  if (!old_data || !new_data) return XRS_ERR_INVALID_ARG;
  for (int r = 0; r < n_parity; ++r)
    if (!parity[r]) return XRS_ERR_INVALID_ARG;
  std::vector<xrs_queue::Piece> in, out;
  for (int r = 0; r < q->p; ++r) {
    in.push_back({parity[r], r, 0, q->size});
    out.push_back({parity[r], r, 0, q->size});
  }
  in.push_back({const_cast<uint8_t*>(old_data), q->p, 0, q->size});
  in.push_back({const_cast<uint8_t*>(new_data), q->p + 1, 0, q->size});
  return q->run(1 + q->d, in, out, row, nullptr, nullptr, t);
}

// xrs.go:236 Reconst(vects, dpHas, needReconst), coalesced: calls with the
// same (dpHas, needReconst) share a batch.  The survivors go up whole, and
// every half the reference writes comes back: the a-halves of every vect not
// in dpHas, the b-halves of surviving piggybacked parity (retrieveRS,
// xrs.go:305-320) and of every needed vect.  A call whose indexes are not all
// valid and distinct, or whose need overlaps dpHas, runs as a plain
// xrs_reconst (the reference's partial side effects and toggling).
static int queue_reconst(xrs_queue* q, uint8_t* const* vects, int n, const int* dp_has, int n_has,
                          const int* need, int n_need, xrs_queue_ticket** t) {
  if (!q) return XRS_ERR_INVALID_ARG;
  if (n_has < 0 || n_need < 0 || (n_has && !dp_has) || (n_need && !need))
    return XRS_ERR_INVALID_ARG;
  if (n_need == 1 && need[0] < q->d)  // xrs.go:238-240 (a negative k is rejected there)
    return queue_reconst_one(q, vects, n, need[0], t);
  const int d = q->d, m = q->d + q->p;
  if (!vects || n != m) return XRS_ERR_ILLEGAL_VECTS;
  for (int i = 0; i < n; ++i)
    if (!vects[i]) return XRS_ERR_INVALID_ARG;
  std::vector<int> in_has(m, 0), in_need(m, 0);
  bool clean = n_has >= d;
  for (int i = 0; i < n_has && clean; ++i) {
    clean = dp_has[i] >= 0 && dp_has[i] < m && !in_has[dp_has[i]];
    if (clean) in_has[dp_has[i]] = 1;
  }
  for (int u = 0; u < n_need && clean; ++u) {
    clean = need[u] >= 0 && need[u] < m && !in_has[need[u]] && !in_need[need[u]];
    if (clean) in_need[need[u]] = 1;
  }
  if (!clean) {  // runs now; an asynchronous caller gets a finished ticket
    const int e = xrs_detail::reconst_direct(q->codec, vects, n, q->size, dp_has, n_has, need, n_need);
    if (!t) return e;
    *t = new xrs_queue_ticket();
    (*t)->q = q;
    (*t)->err = e;
    return XRS_OK;
  }
  const size_t half = q->size / 2;
  std::vector<xrs_queue::Piece> in, out;
  for (int i = 0; i < m; ++i) {
    if (in_has[i]) {
      in.push_back({vects[i], i, 0, q->size});
      int idx[256], len = 0;
      if (i > d && xrs_xorset(q->codec, i, idx, 256, &len) == XRS_OK && len > 0)
        out.push_back({vects[i], i, half, half});  // retrieveRS side effect
    } else {
      out.push_back({vects[i], i, 0, half});  // every lost a-half is rebuilt
      if (in_need[i]) out.push_back({vects[i], i, half, half});
    }
  }
  const std::vector<int> has(dp_has, dp_has + n_has), nd(need, need + n_need);
  return q->run(2 + d, in, out, -1, &has, &nd, t);
}

// xrs.go:363 Replace(data, replaceRows, parity), coalesced: calls with the
// same rows share a batch (staged rows [0, p) parity, [p, p+n) data);
// parity out.
static int queue_replace(xrs_queue* q, uint8_t* const* data, const int* rows, int n,
                          uint8_t* const* parity, int n_parity, xrs_queue_ticket** t) {
  if (!q) return XRS_ERR_INVALID_ARG;
  if (n < 1 || n > q->d) return XRS_ERR_ILLEGAL_VECTS;
  if (!rows) return XRS_ERR_INVALID_ARG;
  for (int i = 0; i < n; ++i)
    if (rows[i] < 0 || rows[i] >= q->d) return XRS_ERR_ILLEGAL_DATA_INDEX;
  if (!parity || n_parity != q->p) return XRS_ERR_ILLEGAL_VECTS;
  if (!data) return XRS_ERR_INVALID_ARG;
  for (int i = 0; i < n; ++i)
    if (!data[i]) return XRS_ERR_INVALID_ARG;
  for (int r = 0; r < n_parity; ++r)
    if (!parity[r]) return XRS_ERR_INVALID_ARG;
  std::vector<xrs_queue::Piece> in, out;
  for (int r = 0; r < q->p; ++r) {
    in.push_back({parity[r], r, 0, q->size});
    out.push_back({parity[r], r, 0, q->size});
  }
  for (int i = 0; i < n; ++i) in.push_back({data[i], q->p + i, 0, q->size});
  const std::vector<int> rv(rows, rows + n), none;
  return q->run(3 + q->d, in, out, -1, &rv, &none, t);
}

int xrs_queue_encode(xrs_queue* q, uint8_t* const* vects, int n) {
  return queue_encode(q, vects, n, nullptr);
}
int xrs_queue_reconst_one(xrs_queue* q, uint8_t* const* vects, int n, int k) {
  return queue_reconst_one(q, vects, n, k, nullptr);
}
int xrs_queue_update(xrs_queue* q, const uint8_t* old_data, const uint8_t* new_data, int row,
                     uint8_t* const* parity, int n_parity) {
  return queue_update(q, old_data, new_data, row, parity, n_parity, nullptr);
}
int xrs_queue_reconst(xrs_queue* q, uint8_t* const* vects, int n, const int* dp_has, int n_has,
                      const int* need, int n_need) {
  return queue_reconst(q, vects, n, dp_has, n_has, need, n_need, nullptr);
}
int xrs_queue_replace(xrs_queue* q, uint8_t* const* data, const int* rows, int n,
                      uint8_t* const* parity, int n_parity) {
  return queue_replace(q, data, rows, n, parity, n_parity, nullptr);
}

// ---- asynchronous forms: stage now, xrs_queue_wait later ----------------
// A submit that finds no free staging batch returns XRS_ERR_BUSY with nothing
// staged (a blocking wait there could deadlock a thread whose own tickets
// hold every batch); the caller waits on one of its tickets and submits again.
#define XRS_SUBMIT(call)             \
  if (!t) return XRS_ERR_INVALID_ARG; \
  *t = nullptr;                      \
  return call
int xrs_queue_submit_encode(xrs_queue* q, uint8_t* const* vects, int n, xrs_queue_ticket** t) {
  XRS_SUBMIT(queue_encode(q, vects, n, t));
}
int xrs_queue_submit_reconst_one(xrs_queue* q, uint8_t* const* vects, int n, int k,
                                 xrs_queue_ticket** t) {
  XRS_SUBMIT(queue_reconst_one(q, vects, n, k, t));
}
int xrs_queue_submit_update(xrs_queue* q, const uint8_t* old_data, const uint8_t* new_data,
                            int row, uint8_t* const* parity, int n_parity, xrs_queue_ticket** t) {
  XRS_SUBMIT(queue_update(q, old_data, new_data, row, parity, n_parity, t));
}
int xrs_queue_submit_reconst(xrs_queue* q, uint8_t* const* vects, int n, const int* dp_has,
                             int n_has, const int* need, int n_need, xrs_queue_ticket** t) {
  XRS_SUBMIT(queue_reconst(q, vects, n, dp_has, n_has, need, n_need, t));
}
int xrs_queue_submit_replace(xrs_queue* q, uint8_t* const* data, const int* rows, int n,
                             uint8_t* const* parity, int n_parity, xrs_queue_ticket** t) {
  XRS_SUBMIT(queue_replace(q, data, rows, n, parity, n_parity, t));
}
#undef XRS_SUBMIT

int xrs_queue_poll(const xrs_queue_ticket* t) {
  if (!t) return XRS_ERR_INVALID_ARG;
  if (!t->st.bt) return 1;
  return t->st.bt->done.load(std::memory_order_acquire) != t->st.seq ? 1 : 0;
}

int xrs_queue_wait(xrs_queue_ticket* t) {
  if (!t) return XRS_ERR_INVALID_ARG;
  const int e = t->st.bt ? t->q->wait(t->st) : t->err;
  delete t;
  return e;
}

size_t xrs_queue_batch_stripes(const xrs_queue* q) { return q ? q->max_batch : 0; }

int xrs_queue_stats(xrs_queue* q, uint64_t out[4]) {
  if (!q || !out) return XRS_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(q->mu);
  out[0] = q->st_batches;
  out[1] = q->st_stripes;
  out[2] = q->st_run_ns;
  out[3] = q->st_wait_ns;
  return XRS_OK;
}

int xrs_queue_batch_sizes(xrs_queue* q, uint64_t* counts, int cap) {
  if (!q || !counts || cap < 1) return XRS_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(q->mu);
  for (int i = 0; i < cap; ++i) counts[i] = 0;
  for (int n = 0; n < xrs_queue::kHist; ++n) counts[std::min(n, cap - 1)] += q->st_hist[n];
  return XRS_OK;
}

size_t xrs_queue_dump(xrs_queue* q, char* buf, size_t cap) {
  if (!q) return 0;
  std::unique_lock<std::mutex> lk(q->mu, std::defer_lock);
  for (int i = 0; i < 100 && !lk.try_lock(); ++i) std::this_thread::sleep_for(std::chrono::microseconds(100));
  static const char* names[] = {"FREE", "OPEN", "CLOSED", "LAUNCHING", "INFLIGHT", "DONE"};
  std::string out;
  char line[256];
  std::snprintf(line, sizeof line, "lock %s open %d in_flight %d bits 0x%x active %d stop %d\n",
                lk.owns_lock() ? "taken" : "BUSY", q->open, q->in_flight, q->inflight_bits.load(),
                q->active.load(), q->stop ? 1 : 0);
  out += line;
  for (int i = 0; i < q->n_batches; ++i) {
    const Batch& bt = q->b[i];
    std::snprintf(line, sizeof line,
                  "batch %d %s key %d reserved %zu n %zu filled %u released %u done %u launches %u "
                  "flag %u err %d\n",
                  i, names[bt.state], bt.key, bt.reserved, bt.n, bt.filled.load(), bt.released.load(),
                  bt.done.load(), bt.launches, bt.flag ? *bt.flag : 0u, bt.err);
    out += line;
  }
  if (buf && cap) {
    const size_t n = std::min(out.size(), cap - 1);
    std::memcpy(buf, out.data(), n);
    buf[n] = 0;
  }
  return out.size();
}

}  // extern "C"
