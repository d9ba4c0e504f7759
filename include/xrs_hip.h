/*
 * xrs_hip.h -- C ABI of the MI355X-native X-Reed-Solomon codec (libxrs_hip.so).
 *
 * This is the drop-in boundary for templexxx/xrs.  The reference has no FFI:
 * its plugin surface is the Go method set of *XRS (/root/reference/xrs.go).
 * Each entry point below names the Go symbol it replaces (file:line).  A cgo
 * shim that keeps the Go method set on top of these calls is in INTEGRATION.md.
 *
 * Conventions (mirroring the reference):
 *  - Shards ("vects") are caller-owned; outputs are written in place; the
 *    library retains no pointer after a call returns (sync calls) or after
 *    the stream reaches the call (async calls).
 *  - Every function returns an int status: 0 = OK, negative = error.
 *    xrs_strerror() gives the text; xrs_format_error() rebuilds the exact Go
 *    message (e.g. "vect size not even: 3") from the code and its argument.
 *  - The codec is immutable after xrs_new() and safe to share across threads.
 *  - Sync calls take HOST pointers (like Go []byte) and block until done.
 *  - *_batched calls take DEVICE pointers to many stripes and are async on the
 *    given stream (a hipStream_t passed as void*; NULL = default stream).
 *    Stripe s, shard i lives at base + s*stripe_stride + i*shard_stride.
 *    This is the performance path.
 *  - No torch/HIP types appear in any signature.
 */
#ifndef XRS_HIP_H
#define XRS_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---------------------------------------------------- */
#define XRS_OK 0
#define XRS_ERR_ILLEGAL_PARITY (-1)     /* xrs.go:57  "illegal parity"            */
#define XRS_ERR_SIZE_NOT_EVEN (-2)      /* xrs.go:133 "vect size not even: %d"    */
#define XRS_ERR_ILLEGAL_DATA_INDEX (-3) /* xrs.go:149 "illegal data index: %d"    */
#define XRS_ERR_ILLEGAL_VECTS (-4)      /* reedsolomon [dep]: bad d/p or vect count */
#define XRS_ERR_TOO_FEW_SURVIVORS (-5)  /* reedsolomon [dep]: len(dpHas) < d      */
#define XRS_ERR_ILLEGAL_INDEX (-6)      /* reedsolomon [dep]: index out of range  */
#define XRS_ERR_SINGULAR (-7)           /* reedsolomon [dep]: singular survivors  */
#define XRS_ERR_HIP (-8)                /* HIP runtime failure                    */
#define XRS_ERR_INVALID_ARG (-9)        /* NULL pointer / bad layout argument     */
#define XRS_ERR_NO_DEVICE (-10)         /* no GPU visible                         */
#define XRS_ERR_BUSY (-11)              /* xrs_queue_submit_*: no staging batch free */

typedef struct xrs_codec xrs_codec;

/* Text for a status code (static storage). */
const char *xrs_strerror(int code);
/* Go-identical message for (code, arg): arg is the size for SIZE_NOT_EVEN and
 * the index for ILLEGAL_DATA_INDEX.  Returns the number of bytes written. */
int xrs_format_error(int code, long long arg, char *buf, size_t buflen);
/* Library version string, and the gfx target the kernels were built for. */
const char *xrs_version(void);
/* Diagnostics (no reference counterpart): record which kernel instantiations
 * the library launches, process-wide.  xrs_trace_kernels(1) clears the record
 * and starts it, (0) stops it.  xrs_traced_kernels writes one "name count"
 * line per kernel, in first-launch order, NUL-terminated and truncated to
 * cap, and returns the full length.  smoke() and the dispatch tests use it. */
int xrs_trace_kernels(int on);
size_t xrs_traced_kernels(char *buf, size_t cap);

/* ---- codec ----------------------------------------------------------- */
/* xrs.go:55 New(dataNum, parityNum).  Builds the systematic Cauchy generator
 * over GF(2^8)/0x11d, the XORSet (xrs.go:77-100) and every per-operation
 * coefficient plan on the host; binds the codec to the current HIP device. */
int xrs_new(int data_num, int parity_num, xrs_codec **out);
void xrs_free(xrs_codec *codec);
/* x.RS.DataNum / x.RS.ParityNum (xrs.go:147, :254). */
int xrs_data_num(const xrs_codec *codec);
int xrs_parity_num(const xrs_codec *codec);
/* x.RS encode matrix (generator), (d+p) x d bytes, row-major. */
int xrs_gen_matrix(const xrs_codec *codec, uint8_t *out, size_t cap);
/* x.XORSet[parity_index] (xrs.go:49): data indexes piggybacked on that
 * parity's b-half, ascending.  *len = 0 if the key is absent. */
int xrs_xorset(const xrs_codec *codec, int parity_index, int *data_idx, int cap, int *len);
/* xrs.go:146 GetNeedVects(needReconst) -> aNeed (a-vector indexes, ascending,
 * excluding k), bNeed = {DataNum, parity index}. a_need needs room for d ints. */
int xrs_get_need_vects(const xrs_codec *codec, int k, int *a_need, int *a_len, int b_need[2]);

/* ---- synchronous per-stripe calls (host memory, Go-identical semantics) -- *
 * A codec may be shared across threads.  A call (Encode, ReconstOne,
 * Reconst, Update, Replace) of up to 1 MiB vects that finds its codec busy
 * with another call is batched with its concurrent peers through an
 * internal xrs_queue for its vect size (same results and errors; up to four
 * sizes per codec, each holding six staging batches of max(4 MiB, one
 * stripe) in pinned host and in device memory until xrs_free: 24 MiB each
 * at 4 KiB vects, 96 MiB each at 1 MiB; a vect size whose staged stripe
 * exceeds 16 MiB is never queued, so a codec holds at most 384 MiB pinned
 * plus 384 MiB device staging; a queue that could not be created is not
 * retried); XRS_AUTO_QUEUE=0 in the environment turns this off.
 * Concurrent calls on one codec may run in one device batch, each on its own
 * staged copy of its vects: concurrent calls must not share OUTPUT buffers
 * (two Update or Replace calls on the same parity vects at once each apply
 * their delta to their own copy and the last copy-back wins; the Go
 * reference leaves this a data race too).  Calls on disjoint stripes, and
 * any number of readers of shared inputs, are safe. */
/* xrs.go:103 Encode(vects): n == d+p vects of `size` bytes; parity written. */
int xrs_encode(const xrs_codec *codec, uint8_t *const *vects, int n, size_t size);
/* xrs.go:175 ReconstOne(vects, needReconst): rebuilds data vect k from the
 * GetNeedVects set only (other vects are not read). */
int xrs_reconst_one(const xrs_codec *codec, uint8_t *const *vects, int n, size_t size, int k);
/* xrs.go:236 Reconst(vects, dpHas, needReconst), including the reference's
 * side effects: a-halves of every vect not in dpHas are rebuilt, and the
 * b-halves of surviving parity > d are left in plain-RS form (xrs.go:265). */
int xrs_reconst(const xrs_codec *codec, uint8_t *const *vects, int n, size_t size,
                const int *dp_has, int n_has, const int *need, int n_need);
/* xrs.go:324 Update(oldData, newData, row, parity): parity = p vects. */
int xrs_update(const xrs_codec *codec, const uint8_t *old_data, const uint8_t *new_data,
               size_t size, int row, uint8_t *const *parity, int n_parity);
/* xrs.go:363 Replace(data, replaceRows, parity). */
int xrs_replace(const xrs_codec *codec, uint8_t *const *data, const int *rows, int n,
                size_t size, uint8_t *const *parity, int n_parity);

/* ---- batched, device-resident, async (the performance path) ----------- */
/* Recommended device layout for a batch of stripes of n_shards vects of
 * `size` bytes: shard stride (size itself below 32 KiB, else size rounded
 * up to 16; plus a 4 KiB + 256 B pad from 4 MiB up) and stripe
 * stride (n_shards shard strides, rounded up to a power of two when that
 * costs at most 1/7 more).  Any layout works; this one streams fastest on
 * MI355X. */
int xrs_batch_strides(size_t size, int n_shards, size_t *shard_stride, size_t *stripe_stride);
/* xrs_batch_strides plus a base offset (0..15 bytes): place the batch at
 * (16-B-aligned allocation) + base_offset, so that the b-half of every shard
 * (vect[S/2:]) is aligned when S/2 is not a multiple of 16 (odd vect sizes:
 * 0 for sizes that are multiples of 32).  A batch of n stripes needs
 * base_offset + n * stripe_stride bytes (stripe_stride may exceed
 * n_shards * shard_stride).  Any layout is correct; this one streams fastest
 * ("Any size, any alignment"). */
int xrs_batch_layout(size_t size, int n_shards, size_t *shard_stride, size_t *stripe_stride,
                     size_t *base_offset);
/* Encode n_stripes stripes in place.  One fused pass: RS + piggyback. */
int xrs_encode_batched(const xrs_codec *codec, uint8_t *base, size_t size,
                       size_t shard_stride, size_t stripe_stride, size_t n_stripes,
                       void *stream);
/* ReconstOne(k) for every stripe (reads only the GetNeedVects set). */
int xrs_reconst_one_batched(const xrs_codec *codec, uint8_t *base, size_t size,
                            size_t shard_stride, size_t stripe_stride, size_t n_stripes,
                            int k, void *stream);
/* Reconst(dpHas, need) for every stripe (same survivor pattern). */
int xrs_reconst_batched(const xrs_codec *codec, uint8_t *base, size_t size,
                        size_t shard_stride, size_t stripe_stride, size_t n_stripes,
                        const int *dp_has, int n_has, const int *need, int n_need,
                        void *stream);
/* Update(old, new, row, parity) for every stripe: old/new rows at
 * old_base + s*old_stripe_stride (same for new); parity shard r of stripe s at
 * parity_base + s*parity_stripe_stride + r*parity_shard_stride. */
int xrs_update_batched(const xrs_codec *codec, const uint8_t *old_base, size_t old_stripe_stride,
                       const uint8_t *new_base, size_t new_stripe_stride, size_t size, int row,
                       uint8_t *parity_base, size_t parity_shard_stride,
                       size_t parity_stripe_stride, size_t n_stripes, void *stream);
/* Update with one data row per stripe -- a batch of small writes to different
 * data shards: stripe s applies Update(old_s, new_s, rows[s], parity_s).
 * rows: n_stripes int32 in device-readable memory (device or host-mapped);
 * a stripe whose row is not in [0, d) is left untouched. */
int xrs_update_rows_batched(const xrs_codec *codec, const uint8_t *old_base,
                            size_t old_stripe_stride, const uint8_t *new_base,
                            size_t new_stripe_stride, size_t size, const int32_t *rows,
                            uint8_t *parity_base, size_t parity_shard_stride,
                            size_t parity_stripe_stride, size_t n_stripes, void *stream);
/* Replace(data, rows, parity) for every stripe: data i of stripe s at
 * data_base + s*data_stripe_stride + i*data_shard_stride. */
int xrs_replace_batched(const xrs_codec *codec, const uint8_t *data_base,
                        size_t data_shard_stride, size_t data_stripe_stride, const int *rows,
                        int n, size_t size, uint8_t *parity_base, size_t parity_shard_stride,
                        size_t parity_stripe_stride, size_t n_stripes, void *stream);

/* ---- per-shard pointer tables (device memory, async) -------------------- *
 * shards[i] = base of shard i; stripe s of shard i at shards[i] + s*stripe_stride.
 * For shards held in separate allocations (e.g. one buffer per disk), or on
 * peer GPUs: with xrs_enable_peer_access(device, peer) the kernels read (and
 * write) peer HBM directly over xGMI (cross-GPU repair). */
int xrs_encode_shards(const xrs_codec *codec, uint8_t *const *shards, size_t stripe_stride,
                      size_t size, size_t n_stripes, void *stream);
/* Only shards in the GetNeedVects set and shard k are dereferenced (others may be NULL). */
int xrs_reconst_one_shards(const xrs_codec *codec, uint8_t *const *shards, size_t stripe_stride,
                           size_t size, size_t n_stripes, int k, void *stream);
int xrs_reconst_shards(const xrs_codec *codec, uint8_t *const *shards, size_t stripe_stride,
                       size_t size, size_t n_stripes, const int *dp_has, int n_has,
                       const int *need, int n_need, void *stream);
/* Let kernels running on `device` access HBM of `peer` (idempotent). */
int xrs_enable_peer_access(int device, int peer);

/* ---- host-resident batches (synchronous) ------------------------------- *
 * The real caller's path (shards start and end in host memory, e.g. disk or
 * NIC buffers).  Host layout as for *_batched.  A batch inside pinned, mapped
 * memory (xrs_host_alloc / xrs_host_register) runs in place: the kernels read
 * and write it over PCIe.  Pageable memory (or XRS_HOST_ZC=0) is moved in
 * chunks through device slots on three streams so H2D, kernel and D2H
 * overlap. */
int xrs_encode_host(const xrs_codec *codec, uint8_t *host_base, size_t size, size_t shard_stride,
                    size_t stripe_stride, size_t n_stripes);
/* ReconstOne(k) per stripe; only the GetNeedVects halves cross PCIe. */
int xrs_reconst_one_host(const xrs_codec *codec, uint8_t *host_base, size_t size,
                         size_t shard_stride, size_t stripe_stride, size_t n_stripes, int k);
/* xrs.go:236 Reconst(dpHas, need) over a host-resident batch (same layout
 * rules; a clean call moves only the survivors up and the written halves
 * back, with the reference's side effects). */
int xrs_reconst_host(const xrs_codec *codec, uint8_t *host_base, size_t size, size_t shard_stride,
                     size_t stripe_stride, size_t n_stripes, const int *dp_has, int n_has,
                     const int *need, int n_need);
/* xrs.go:324 Update over host-resident rows (layout as xrs_update_batched,
 * host addresses; in place over PCIe when every buffer is pinned and mapped). */
int xrs_update_host(const xrs_codec *codec, const uint8_t *old_base, size_t old_stripe_stride,
                    const uint8_t *new_base, size_t new_stripe_stride, size_t size, int row,
                    uint8_t *parity_base, size_t parity_shard_stride,
                    size_t parity_stripe_stride, size_t n_stripes);
/* xrs.go:363 Replace over host-resident rows (layout as xrs_replace_batched). */
int xrs_replace_host(const xrs_codec *codec, const uint8_t *data_base, size_t data_shard_stride,
                     size_t data_stripe_stride, const int *rows, int n, size_t size,
                     uint8_t *parity_base, size_t parity_shard_stride,
                     size_t parity_stripe_stride, size_t n_stripes);
/* Pinned, device-mapped host memory.  Per-stripe calls (xrs_encode ...,
 * xrs_queue_* and xrs_queue_submit_*) whose every vect lies in such memory
 * do not copy: the kernels read and write the caller's buffers IN PLACE over
 * PCIe (codec.cpp reg_vects, queue.cpp table mode), host-resident batches
 * (*_host) likewise.  Lifetime contract: xrs_host_free / xrs_host_unregister
 * only when no call on vects inside the range is in flight (a synchronous
 * call has returned; every ticket of an asynchronous one has been waited
 * on).  After unregister the pages are ordinary pageable memory again: they
 * may be freed and reused (tests/cpp/xrs_test.cpp
 * TestRegistered_UnregisterFreeReuse,
 * tests/gpu_registered_cases.py::test_unregister_free_reuse_then_pageable_copy).
 * Caution: late in a long process the HIP runtime's own pageable copies of
 * such reused pages have met an illegal-address error inside its user-page
 * pinning (never with GPU_PINNED_MIN_XFER_SIZE=1048576 set).
 * Registering is a pin and a map (tens of us per MiB), so a buffer pool that
 * registers once and lives for the process is the intended use
 * (INTEGRATION.md). */
void *xrs_host_alloc(size_t bytes);           /* pinned host memory mapped to every GPU (NULL on failure) */
void xrs_host_free(void *p);
int xrs_host_register(void *p, size_t bytes); /* pin (and map) existing host memory */
int xrs_host_unregister(void *p);             /* p: the pointer given to xrs_host_register */
/* Device address of pinned, mapped host memory (from xrs_host_alloc or
 * xrs_host_register), or NULL.  It may be passed as the base of the
 * *_batched calls: the kernels then read and write host memory over PCIe
 * (zero copy). */
void *xrs_host_device_pointer(void *host);

/* ---- one process, several GPUs ----------------------------------------- *
 * A group holds one codec per listed device.  Host-resident batches are split
 * into contiguous stripe ranges, one per member, run concurrently (one host
 * thread per GPU, each GPU on its own PCIe link); no data moves between GPUs.
 * A device may be listed more than once.  Device-resident batches already on
 * each GPU take the member codecs' *_batched calls directly. */
typedef struct xrs_group xrs_group;
int xrs_group_new(int data_num, int parity_num, const int *devices, int n_devices,
                  xrs_group **out);
void xrs_group_free(xrs_group *g);
int xrs_group_size(const xrs_group *g);
const xrs_codec *xrs_group_codec(const xrs_group *g, int i);
int xrs_group_encode_host(xrs_group *g, uint8_t *host_base, size_t size, size_t shard_stride,
                          size_t stripe_stride, size_t n_stripes);
int xrs_group_reconst_one_host(xrs_group *g, uint8_t *host_base, size_t size,
                               size_t shard_stride, size_t stripe_stride, size_t n_stripes,
                               int k);
/* xrs.go:236 Reconst(dpHas, need) over a host-resident batch, split across the group. */
int xrs_group_reconst_host(xrs_group *g, uint8_t *host_base, size_t size, size_t shard_stride,
                           size_t stripe_stride, size_t n_stripes, const int *dp_has, int n_has,
                           const int *need, int n_need);
/* xrs.go:324 Update / :363 Replace over host-resident rows, split across the group. */
int xrs_group_update_host(xrs_group *g, const uint8_t *old_base, size_t old_stripe_stride,
                          const uint8_t *new_base, size_t new_stripe_stride, size_t size, int row,
                          uint8_t *parity_base, size_t parity_shard_stride,
                          size_t parity_stripe_stride, size_t n_stripes);
int xrs_group_replace_host(xrs_group *g, const uint8_t *data_base, size_t data_shard_stride,
                           size_t data_stripe_stride, const int *rows, int n, size_t size,
                           uint8_t *parity_base, size_t parity_shard_stride,
                           size_t parity_stripe_stride, size_t n_stripes);

/* ---- batching queue (per-stripe calls from many threads) --------------- *
 * Coalesces concurrent per-stripe calls (Go: many goroutines calling
 * x.Encode / x.ReconstOne / x.Update ...) into device batches of up to
 * max_batch_stripes (capped at 64 MiB of staging); a batch holds calls of
 * one kind (Encode, ReconstOne of one k, Reconst of one (dpHas, need)
 * pattern, Replace of one rows set, or Update of any rows).  The open batch
 * runs as soon as fewer than XRS_QUEUE_INFLIGHT (default 4) batches are in
 * flight, or when full (XRS_QUEUE_POLICY=timer: when full, when the GPU is
 * idle, or max_wait_us after it opened).  Batches of up to XRS_QUEUE_ZC_MAX
 * bytes (default 4 MiB) are processed in place in pinned host memory over
 * PCIe, larger ones with one H2D, one kernel and one D2H.  Each call blocks
 * until its own stripe is done and has the semantics of the matching
 * synchronous call for vects of the queue's `size`.  Thread-safe; one queue
 * per (codec, vect size).  A queue holds XRS_QUEUE_BATCHES (default 6)
 * staging batches, each max_batch_stripes stripes (<= 64 MiB) of pinned host
 * and of device memory, one launcher and one completion thread.
 * xrs_queue_free: later calls fail; calls in flight complete first. */
typedef struct xrs_queue xrs_queue;
int xrs_queue_new(const xrs_codec *codec, size_t size, size_t max_batch_stripes, int max_wait_us,
                  xrs_queue **out);
void xrs_queue_free(xrs_queue *q);
int xrs_queue_encode(xrs_queue *q, uint8_t *const *vects, int n);
int xrs_queue_reconst_one(xrs_queue *q, uint8_t *const *vects, int n, int k);
/* xrs.go:236 Reconst(vects, dpHas, needReconst), coalesced: calls with the
 * same (dpHas, needReconst) share a batch, with the side effects of
 * xrs_reconst; calls with invalid, repeated or overlapping indexes run as a
 * plain xrs_reconst. */
int xrs_queue_reconst(xrs_queue *q, uint8_t *const *vects, int n, const int *dp_has, int n_has,
                      const int *need, int n_need);
/* xrs.go:363 Replace(data, replaceRows, parity), coalesced per rows set. */
int xrs_queue_replace(xrs_queue *q, uint8_t *const *data, const int *rows, int n,
                      uint8_t *const *parity, int n_parity);
/* xrs.go:324 Update(oldData, newData, row, parity), coalesced. */
int xrs_queue_update(xrs_queue *q, const uint8_t *old_data, const uint8_t *new_data, int row,
                     uint8_t *const *parity, int n_parity);
/* Asynchronous forms (one caller thread -- one cgo call site -- keeps several
 * stripes in flight; reference call pattern xrs_test.go:498-521, one
 * x.Encode per stripe).  A submit validates like the synchronous call, stages
 * the stripe into the open batch and returns at once with *ticket set;
 * xrs_queue_wait(ticket) blocks until that stripe is done, copies its outputs
 * back (vects outside registered memory), frees the ticket and returns the
 * call's status.  The vects must stay valid and must not be touched until the
 * wait returns.  Every ticket is waited on exactly once, before
 * xrs_queue_free.  A submit never blocks: with no staging batch free it
 * returns XRS_ERR_BUSY and stages nothing -- wait on one of your tickets
 * (e.g. the oldest) and submit again.  A Reconst the queue cannot batch
 * (see xrs_queue_reconst) runs at once and returns a finished ticket. */
typedef struct xrs_queue_ticket xrs_queue_ticket;
int xrs_queue_submit_encode(xrs_queue *q, uint8_t *const *vects, int n, xrs_queue_ticket **ticket);
int xrs_queue_submit_reconst_one(xrs_queue *q, uint8_t *const *vects, int n, int k,
                                 xrs_queue_ticket **ticket);
int xrs_queue_submit_reconst(xrs_queue *q, uint8_t *const *vects, int n, const int *dp_has,
                             int n_has, const int *need, int n_need, xrs_queue_ticket **ticket);
int xrs_queue_submit_replace(xrs_queue *q, uint8_t *const *data, const int *rows, int n,
                             uint8_t *const *parity, int n_parity, xrs_queue_ticket **ticket);
int xrs_queue_submit_update(xrs_queue *q, const uint8_t *old_data, const uint8_t *new_data,
                            int row, uint8_t *const *parity, int n_parity,
                            xrs_queue_ticket **ticket);
/* 1 when the ticket's stripe is done (xrs_queue_wait will not block), else 0. */
int xrs_queue_poll(const xrs_queue_ticket *ticket);
int xrs_queue_wait(xrs_queue_ticket *ticket);
size_t xrs_queue_batch_stripes(const xrs_queue *q);
/* Counters since xrs_queue_new: out[0] batches run, out[1] stripes run,
 * out[2] ns from each batch's launch to its completion, out[3] ns each batch
 * waited between opening and launch (summed over batches). */
int xrs_queue_stats(xrs_queue *q, uint64_t out[4]);
/* Batches run since xrs_queue_new by stripe count: counts[n] = batches of n
 * stripes for n < cap - 1, counts[cap - 1] = batches of cap - 1 or more
 * (stripe counts past 64 are kept as 64). */
int xrs_queue_batch_sizes(xrs_queue *q, uint64_t *counts, int cap);
/* Diagnostics: the queue's state (per staging batch: state, slots reserved /
 * staged / released, launches and the completion word) as text into buf
 * (NUL-terminated, truncated to cap); returns the full length.  Takes the
 * queue lock only if it is free within 10 ms. */
size_t xrs_queue_dump(xrs_queue *q, char *buf, size_t cap);

#ifdef __cplusplus
}
#endif
#endif /* XRS_HIP_H */
