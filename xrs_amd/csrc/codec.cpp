// codec.cpp -- host side of the MI355X X-Reed-Solomon codec and its C ABI.
//
// The host owns what xrs.go does on the CPU that is not byte arithmetic:
// argument checks (xrs.go:130-136, :146-151), the XORSet (xrs.go:77-100),
// survivor selection and the GF(2^8) matrix inverses of the RS dependency,
// composition of every operation into one or a few "pair"/"rows" kernel plans
// (xrs_plan.h), and the per-stripe synchronous API that moves host vects
// through device staging.  Every byte of shard arithmetic runs in kernels.hip.
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "gf256.h"
#include "hostreg.h"
#include "xrs_hip.h"
#include "xrs_plan.h"

using xrs::GF;
using xrs::GfTab;
using xrs::RowRef;

struct xrs_codec {
  int d = 0, p = 0;
  int device = -1;
  std::vector<uint8_t> gen;          // (d+p) x d systematic generator
  std::vector<std::vector<int>> xs;  // xs[h] = XORSet[h] (empty if no such key)
  std::vector<int> bi_of;            // data j -> parity index whose b-half carries a_j
  // ReconstOne(k) plans (xrs.go:175-221): survivors has_k = [0..d-1] with k -> d;
  // r1_bk[k][m] rebuilds b_k, r1_brs[k][m] rebuilds the RS-form b of parity bi.
  // Built on first use of k (a d x d inverse each), then immutable.
  mutable std::mutex plan_mu;
  mutable std::vector<std::vector<uint8_t>> r1_bk, r1_brs;

  // sync-API state (lazy; guarded by mu)
  mutable std::mutex mu;
  mutable uint8_t* staging = nullptr;
  mutable size_t staging_cap = 0;
  mutable uint8_t* hstaging = nullptr;  // pinned, mapped host mirror of `staging` (small calls)
  mutable uint8_t* hstaging_dev = nullptr;  // its device address (zero-copy kernels)
  mutable size_t hstaging_cap = 0;
  mutable hipStream_t stream = nullptr;
  // completion word of the sync calls: the stream writes ++done_seq into
  // pinned host memory after a call's work, and the caller spins on it
  mutable uint32_t* done_word = nullptr;
  mutable uint32_t* done_word_dev = nullptr;
  mutable uint32_t done_seq = 0;
  // batching queues of concurrent per-stripe calls, one per vect size
  // (auto_queue; guarded by aq_mu)
  mutable std::mutex aq_mu;
  mutable std::vector<std::pair<size_t, xrs_queue*>> aq;

  // host-resident pipeline state (lazy; guarded by pipe_mu): kPipe device
  // slots, one stream each, so chunk i+1's H2D, chunk i's kernel and chunk
  // i-1's D2H overlap.
  static constexpr int kPipe = 3;
  mutable std::mutex pipe_mu;
  mutable uint8_t* slot[kPipe] = {nullptr, nullptr, nullptr};
  mutable size_t slot_cap = 0;
  mutable hipStream_t pstream[kPipe] = {nullptr, nullptr, nullptr};
  mutable uint8_t* bounce[kPipe] = {nullptr, nullptr, nullptr};  // pinned (HeadBounce)
  mutable size_t bounce_cap = 0;

  uint8_t g(int row, int col) const { return gen[static_cast<size_t>(row) * d + col]; }
};

namespace {

int hip_err(hipError_t e) { return e == hipSuccess ? XRS_OK : XRS_ERR_HIP; }

// ---------------------------------------------------------------- planning
struct MulSrc {
  RowRef row;
  std::vector<uint8_t> coef;  // one per output
  int pb;                     // pair kernel: output whose b-half takes this a-half, or -1
};
struct XorSrc {
  RowRef row;
  std::vector<int> outs;  // outputs this row is XORed into
};

// Pair plans: outputs in groups of kMaxOut, sources in chunks of kMaxSrc; the
// first chunk of each group writes (or accumulates if acc), later chunks add.
int run_pair(const std::vector<RowRef>& dst, const std::vector<MulSrc>& src, bool acc,
             bool encode, uint64_t half, uint64_t n_stripes, hipStream_t stream) {
  if (half == 0 || n_stripes == 0 || dst.empty()) return XRS_OK;
  const GF& gf = GF::get();
  const int np = static_cast<int>(dst.size()), ns = static_cast<int>(src.size());
  xrs::PairPlan plan;
  for (int g0 = 0; g0 < np; g0 += xrs::kMaxOut) {
    const int P = std::min(xrs::kMaxOut, np - g0);
    int c0 = 0;
    do {
      const int C = std::min(xrs::kMaxSrc, ns - c0);
      std::memset(&plan, 0, sizeof(plan));
      plan.P = P;
      plan.C = C;
      plan.acc = acc || c0 > 0;
      // one launch covers the whole Encode: source c = data c, piggyback
      // target 1 + c % (p-1) (makeXORSet, xrs.go:77-100)
      plan.encode_xs = encode && np <= xrs::kMaxOut && ns <= xrs::kMaxSrc && np >= 2;
      // ... and only with sources in makeXORSet order: the compile-time
      // kernels hard-code that piggyback target and ignore plan.pb
      for (int c = 0; c < C && plan.encode_xs; ++c)
        plan.encode_xs = src[c0 + c].pb == 1 + c % (np - 1);
      plan.half = half;
      plan.n_stripes = n_stripes;
      for (int r = 0; r < P; ++r) plan.dst[r] = dst[g0 + r];
      for (int c = 0; c < C; ++c) {
        const MulSrc& s = src[c0 + c];
        plan.src[c] = s.row;
        for (int r = 0; r < P; ++r) plan.tab[c][r] = gf.tab(s.coef[g0 + r]);
        plan.pb[c] = (s.pb >= g0 && s.pb < g0 + P) ? static_cast<int8_t>(s.pb - g0) : -1;
      }
      const int e = xrs::launch_pair(plan, stream);
      if (e != 0) return XRS_ERR_HIP;
      c0 += C;
    } while (c0 < ns);
  }
  return XRS_OK;
}

// Rows plans: outputs in groups of kMaxOut; GF and XOR sources in chunks.
int run_rows(const std::vector<RowRef>& dst, const std::vector<MulSrc>& msrc,
             const std::vector<XorSrc>& xsrc, bool acc, uint64_t len, uint64_t n_stripes,
             hipStream_t stream) {
  if (len == 0 || n_stripes == 0 || dst.empty()) return XRS_OK;
  const GF& gf = GF::get();
  const int nr = static_cast<int>(dst.size());
  xrs::RowsPlan plan;
  for (int g0 = 0; g0 < nr; g0 += xrs::kMaxOut) {
    const int R = std::min(xrs::kMaxOut, nr - g0);
    // XOR sources that touch this group, with their group-relative masks
    std::vector<std::pair<RowRef, uint32_t>> xs;
    for (const XorSrc& x : xsrc) {
      uint32_t m = 0;
      for (int o : x.outs)
        if (o >= g0 && o < g0 + R) m ^= 1u << (o - g0);  // ^=: a repeated target cancels
      if (m) xs.push_back({x.row, m});
    }
    const int nm = static_cast<int>(msrc.size()), nx = static_cast<int>(xs.size());
    int m0 = 0, x0 = 0;
    bool first = true;
    do {
      const int NM = std::min(xrs::kMaxSrc, nm - m0), NX = std::min(xrs::kMaxXor, nx - x0);
      std::memset(&plan, 0, sizeof(plan));
      plan.R = R;
      plan.NM = NM;
      plan.NX = NX;
      plan.acc = acc || !first;
      plan.len = len;
      plan.n_stripes = n_stripes;
      for (int r = 0; r < R; ++r) plan.dst[r] = dst[g0 + r];
      for (int m = 0; m < NM; ++m) {
        plan.msrc[m] = msrc[m0 + m].row;
        for (int r = 0; r < R; ++r) plan.tab[m][r] = gf.tab(msrc[m0 + m].coef[g0 + r]);
      }
      for (int x = 0; x < NX; ++x) {
        plan.xsrc[x] = xs[x0 + x].first;
        plan.xmask[x] = xs[x0 + x].second;
      }
      const int e = xrs::launch_rows(plan, stream);
      if (e != 0) return XRS_ERR_HIP;
      m0 += NM;
      x0 += NX;
      first = false;
    } while (m0 < nm || x0 < nx);
  }
  return XRS_OK;
}

// Device layout of a batch of stripes: shard i of stripe s at
// base + s*stripe_stride + i*shard_stride, or, with a per-shard pointer table,
// at table[i] + s*stripe_stride (shards in separate allocations, or on peer
// GPUs reached over xGMI).
//
// Or, with `ind` (the batching queue's callers' own buffers), every row is
// indirect (xrs_plan.h kRowInd): stripe s has a table of two device-readable
// entries per shard, the addresses of its a-half and b-half, at
// ind + s * ind_stride bytes; row(shard, off) takes off = 0 or S/2.
struct Layout {
  uint8_t* base;
  size_t shard_stride, stripe_stride;
  const uint64_t* table = nullptr;
  const uint64_t* ind = nullptr;
  uint64_t ind_stride = 0;
  RowRef row(int shard, size_t off) const {
    if (ind)
      return {reinterpret_cast<uint64_t>(ind + 2 * shard + (off ? 1 : 0)), ind_stride | xrs::kRowInd};
    const uint64_t b = table ? table[shard]
                             : reinterpret_cast<uint64_t>(base) +
                                   static_cast<uint64_t>(shard) * shard_stride;
    return {b + off, static_cast<uint64_t>(stripe_stride)};
  }
};

int check_size(size_t size) { return (size & 1) ? XRS_ERR_SIZE_NOT_EVEN : XRS_OK; }

int need_vects(const xrs_codec* x, int k, std::vector<int>* a_need, int* bi) {
  if (k < 0 || k >= x->d) return XRS_ERR_ILLEGAL_DATA_INDEX;  // xrs.go:148-151
  *bi = x->bi_of[k];
  a_need->clear();
  for (int i : x->xs[*bi])
    if (i != k) a_need->push_back(i);
  return XRS_OK;
}

// Rebuild rows `out` from survivors dp_has[:d] (reedsolomon Reconst [dep]):
// coefficient row for t = gen[t] * inv(gen[has]).  Validation order follows
// oracle/xrs_oracle.c oxrs_rs_reconst.
int survivor_rows(const xrs_codec* x, const int* dp_has, int n_has, const std::vector<int>& out,
                  std::vector<std::vector<uint8_t>>* coef) {
  const int d = x->d, n = x->d + x->p;
  if (out.empty()) return XRS_OK;
  if (n_has < d) return XRS_ERR_TOO_FEW_SURVIVORS;
  for (int i = 0; i < n_has; ++i)
    if (dp_has[i] < 0 || dp_has[i] >= n) return XRS_ERR_ILLEGAL_INDEX;
  for (int t : out)
    if (t < 0 || t >= n) return XRS_ERR_ILLEGAL_INDEX;
  const GF& gf = GF::get();
  std::vector<uint8_t> e(static_cast<size_t>(d) * d);
  for (int i = 0; i < d; ++i)
    for (int j = 0; j < d; ++j) e[static_cast<size_t>(i) * d + j] = x->g(dp_has[i], j);
  if (!gf.invert(e, d)) return XRS_ERR_SINGULAR;
  coef->assign(out.size(), std::vector<uint8_t>(d, 0));
  for (size_t q = 0; q < out.size(); ++q)
    for (int i = 0; i < d; ++i) {
      uint8_t c = 0;
      for (int j = 0; j < d; ++j) c ^= gf.mul(x->g(out[q], j), e[static_cast<size_t>(j) * d + i]);
      (*coef)[q][i] = c;
    }
  return XRS_OK;
}

// ReconstOne(k) coefficient rows, built once per (codec, k).
int reconst_one_plan(const xrs_codec* x, int k, std::vector<uint8_t>* bk,
                     std::vector<uint8_t>* brs) {
  std::lock_guard<std::mutex> lk(x->plan_mu);
  if (x->r1_bk[k].empty()) {
    std::vector<int> has(x->d);
    for (int m = 0; m < x->d; ++m) has[m] = m;
    has[k] = x->d;  // xrs.go:195-199
    std::vector<std::vector<uint8_t>> coef;
    const int e = survivor_rows(x, has.data(), x->d, {k, x->bi_of[k]}, &coef);
    if (e) return e;
    x->r1_bk[k] = coef[0];
    x->r1_brs[k] = coef[1];
  }
  *bk = x->r1_bk[k];
  *brs = x->r1_brs[k];
  return XRS_OK;
}

// Halves written by a batched op (for the sync API's copy-back).
struct Written {
  std::vector<std::pair<int, int>> halves;  // (shard, 0 = a-half / 1 = b-half)
  void add(int shard, int h) { halves.push_back({shard, h}); }
};

// ------------------------------------------------------------ batched ops
int encode_impl(const xrs_codec* x, const Layout& L, size_t size, size_t n_stripes,
                hipStream_t s) {
  const int d = x->d, p = x->p;
  const size_t half = size / 2;
  std::vector<RowRef> dst;
  for (int r = 0; r < p; ++r) dst.push_back(L.row(d + r, 0));
  std::vector<MulSrc> src(d);
  for (int j = 0; j < d; ++j) {
    src[j].row = L.row(j, 0);
    src[j].coef.resize(p);
    for (int r = 0; r < p; ++r) src[j].coef[r] = x->g(d + r, j);
    src[j].pb = x->bi_of[j] - d;  // xrs.go:118-126 piggyback target
  }
  return run_pair(dst, src, false, true, half, n_stripes, s);
}

int reconst_one_impl(const xrs_codec* x, const Layout& L, size_t size, size_t n_stripes, int k,
                     hipStream_t s) {
  const int d = x->d;
  const size_t half = size / 2;
  std::vector<int> a_need;
  int bi = 0;
  int e = need_vects(x, k, &a_need, &bi);
  if (e) return e;
  // b_k = sum_m r1_bk[k][m] * b(has_m);  a_k = b(bi) ^ bRS ^ XOR a(aNeed),
  // bRS = sum_m r1_brs[k][m] * b(has_m)   (xrs.go:205, :213-219)
  std::vector<uint8_t> bk, brs;
  if ((e = reconst_one_plan(x, k, &bk, &brs))) return e;
  std::vector<RowRef> dst = {L.row(k, half), L.row(k, 0)};
  std::vector<MulSrc> ms(d);
  for (int m = 0; m < d; ++m) {
    const int h = (m == k) ? d : m;
    ms[m].row = L.row(h, half);
    ms[m].coef = {bk[m], brs[m]};
    ms[m].pb = -1;
  }
  std::vector<XorSrc> xs;
  xs.push_back({L.row(bi, half), {1}});
  for (int i : a_need) xs.push_back({L.row(i, 0), {1}});
  return run_rows(dst, ms, xs, false, half, n_stripes, s);
}

// General Reconst (xrs.go:236-301) as ONE staged-kernel pass (xrs_plan.h
// StagedPlan): stage 1 rebuilds the lost a-halves, stage 2 is retrieveRS on
// the surviving piggybacked parity, stage 3+4 rebuild the needed b-halves and
// re-piggyback them, all from registers.  Applies when the call is "clean":
// every index valid and distinct, need disjoint from dpHas, both inverses
// exist, and the plan fits kStSrc/kStOut.  Otherwise returns 1 and the caller
// runs the step-by-step plan, which reproduces the reference's partial side
// effects on errors and its toggling on repeated indexes.
int reconst_staged(const xrs_codec* x, const Layout& L, size_t size, size_t n_stripes,
                   const int* dp_has, int n_has, const int* need, int n_need, hipStream_t s,
                   Written* w) {
  const int d = x->d, n = x->d + x->p;
  if (d > xrs::kStSrc || n_has < d || n_need > xrs::kStOut) return 1;
  std::vector<int> in_has(n, 0), lost_q(n, -1), apos(n, -1), bpos(n, -1);
  for (int i = 0; i < n_has; ++i) {
    if (dp_has[i] < 0 || dp_has[i] >= n || in_has[dp_has[i]]) return 1;
    in_has[dp_has[i]] = 1;
  }
  std::vector<int> seen(n, 0);
  for (int u = 0; u < n_need; ++u) {
    if (need[u] < 0 || need[u] >= n || in_has[need[u]] || seen[need[u]]) return 1;
    seen[need[u]] = 1;
  }
  std::vector<int> a_lost;
  for (int i = 0; i < n; ++i)
    if (!in_has[i]) a_lost.push_back(i);
  if (static_cast<int>(a_lost.size()) > xrs::kStOut) return 1;
  std::vector<std::vector<uint8_t>> acoef, bcoef;
  if (survivor_rows(x, dp_has, n_has, a_lost, &acoef) != XRS_OK) return 1;
  const std::vector<int> outs(need, need + n_need);
  if (survivor_rows(x, dp_has, n_has, outs, &bcoef) != XRS_OK) return 1;
  for (size_t q = 0; q < a_lost.size(); ++q) lost_q[a_lost[q]] = static_cast<int>(q);

  xrs::StagedPlan plan;
  std::memset(&plan, 0, sizeof(plan));
  const size_t half = size / 2;
  plan.nd = d;
  for (int m = 0; m < d; ++m) {
    plan.asrc[m] = L.row(dp_has[m], 0);
    plan.bsrc[m] = L.row(dp_has[m], half);
    apos[dp_has[m]] = bpos[dp_has[m]] = m;
  }
  plan.na = plan.nb = d;
  bool fits = true;
  // abar(XS[h]): surviving members from their a-rows (extra rows appended),
  // lost members from the stage-1 registers.
  auto abar = [&](int h) {
    uint32_t mask = 0;
    for (int j : x->xs[h]) {
      if (!in_has[j]) {
        mask ^= 1u << (xrs::kStSrc + lost_q[j]);
        continue;
      }
      if (apos[j] < 0) {
        if (plan.na == xrs::kStSrc) {
          fits = false;
          continue;
        }
        apos[j] = plan.na;
        plan.asrc[plan.na++] = L.row(j, 0);
      }
      mask ^= 1u << apos[j];
    }
    return mask;
  };
  plan.nl = static_cast<int>(a_lost.size());
  for (int q = 0; q < plan.nl; ++q) {
    plan.adst[q] = L.row(a_lost[q], 0);
    for (int m = 0; m < d; ++m) plan.acoef[m][q] = acoef[q][m];
  }
  for (int h = d + 1; h < n; ++h) {  // xrs.go:305-320: h in dpHas, h > d
    if (!in_has[h] || x->xs[h].empty()) continue;
    if (bpos[h] < 0) {
      if (plan.nb == xrs::kStB) return 1;
      bpos[h] = plan.nb;
      plan.bsrc[plan.nb++] = L.row(h, half);
    }
    plan.bret[bpos[h]] = abar(h);
    plan.bstore |= 1u << bpos[h];
  }
  plan.nn = n_need;
  for (int u = 0; u < n_need; ++u) {
    plan.bdst[u] = L.row(need[u], half);
    for (int m = 0; m < d; ++m) plan.bcoef[m][u] = bcoef[u][m];
    if (need[u] > d) plan.nmask[u] = abar(need[u]);  // xrs.go:283-297
  }
  if (!fits) return 1;
  plan.half = half;
  plan.n_stripes = n_stripes;
  if (half > 0 && n_stripes > 0) {
    const int e = xrs::launch_staged(plan, s);
    if (e == xrs::kStagedDecline) return 1;  // nothing launched: the step plan runs
    if (e != 0) return XRS_ERR_HIP;
  }
  for (int t : a_lost) w->add(t, 0);
  for (int h = d + 1; h < n; ++h)
    if (in_has[h] && !x->xs[h].empty()) w->add(h, 1);
  for (int u = 0; u < n_need; ++u) w->add(need[u], 1);
  return XRS_OK;
}

// xrs.go:236-301 general Reconst: four steps, in the reference's order.
int reconst_impl(const xrs_codec* x, const Layout& L, size_t size, size_t n_stripes,
                 const int* dp_has, int n_has, const int* need, int n_need, hipStream_t s,
                 Written* w) {
  const int d = x->d, p = x->p;
  const size_t half = size / 2;
  // One staged pass when the call is clean; XRS_RECONST=steps forces the
  // step-by-step plan (tests run both).
  const char* mode = std::getenv("XRS_RECONST");
  if (!(mode && std::strcmp(mode, "steps") == 0)) {
    const int e = reconst_staged(x, L, size, n_stripes, dp_has, n_has, need, n_need, s, w);
    if (e <= 0) return e;  // handled (or failed); 1 = not applicable
  }
  // Step 1: a-halves of every vect not in dpHas (xrs.go:247-262).
  std::vector<int> a_lost;
  for (int i = 0; i < d + p; ++i)
    if (std::find(dp_has, dp_has + n_has, i) == dp_has + n_has) a_lost.push_back(i);
  std::vector<std::vector<uint8_t>> coef;
  int e = survivor_rows(x, dp_has, n_has, a_lost, &coef);
  if (e) return e;
  if (!a_lost.empty()) {
    std::vector<RowRef> dst;
    for (int t : a_lost) dst.push_back(L.row(t, 0));
    std::vector<MulSrc> ms(d);
    for (int m = 0; m < d; ++m) {
      ms[m].row = L.row(dp_has[m], 0);
      ms[m].coef.resize(a_lost.size());
      for (size_t q = 0; q < a_lost.size(); ++q) ms[m].coef[q] = coef[q][m];
      ms[m].pb = -1;
    }
    e = run_rows(dst, ms, {}, false, half, n_stripes, s);
    if (e) return e;
    for (int t : a_lost) w->add(t, 0);
  }
  // Step 2: retrieveRS, surviving parity h > d back to RS form (xrs.go:305-320).
  // A repeated h in dpHas is applied repeatedly by the reference: parity of count.
  {
    std::vector<int> cnt(d + p, 0);
    for (int i = 0; i < n_has; ++i)
      if (dp_has[i] > d && dp_has[i] < d + p) cnt[dp_has[i]] ^= 1;
    std::vector<RowRef> dst;
    std::vector<XorSrc> xs;
    for (int h = d + 1; h < d + p; ++h) {
      if (!cnt[h] || x->xs[h].empty()) continue;
      const int o = static_cast<int>(dst.size());
      dst.push_back(L.row(h, half));
      for (int ai : x->xs[h]) xs.push_back({L.row(ai, 0), {o}});
      w->add(h, 1);
    }
    if (!dst.empty()) {
      e = run_rows(dst, {}, xs, true, half, n_stripes, s);
      if (e) return e;
    }
  }
  // Step 3 + 4: b-halves of need, then re-piggyback needed parity != d
  // (xrs.go:270-298).  Both write the same rows, so one plan per output.
  std::vector<int> outs(need, need + n_need);
  e = survivor_rows(x, dp_has, n_has, outs, &coef);
  if (e) return e;
  if (outs.empty()) return XRS_OK;
  std::vector<int> uniq;  // distinct need rows (a repeated need is rebuilt once)
  std::vector<int> rep;   // how many times each appears (re-piggyback count)
  std::vector<size_t> qidx;
  for (int q = 0; q < n_need; ++q) {
    auto it = std::find(uniq.begin(), uniq.end(), need[q]);
    if (it == uniq.end()) {
      uniq.push_back(need[q]);
      rep.push_back(1);
      qidx.push_back(q);
    } else {
      rep[it - uniq.begin()]++;
    }
  }
  // A need row that is one of the d GF sources (dp_has[:d]) rebuilds as
  // itself: its coefficient row is a unit vector.  It is kept out of the GF
  // plan, so no launch of a multi-launch plan (more than kMaxOut outputs, or
  // d > kMaxSrc chained launches) reads a source row an earlier launch of the
  // same plan already wrote; its re-piggyback XOR (if any) is applied after
  // every GF output is written.  The oracle computes all outputs before
  // writing any (oracle/xrs_oracle.c oxrs_rs_reconst), which this matches.
  std::vector<RowRef> dst, self_dst;
  std::vector<int> gf_u, self_u;
  for (size_t u = 0; u < uniq.size(); ++u) {
    const bool is_src = std::find(dp_has, dp_has + d, uniq[u]) != dp_has + d;
    (is_src ? self_u : gf_u).push_back(static_cast<int>(u));
  }
  std::vector<MulSrc> ms(d);
  for (int m = 0; m < d; ++m) {
    ms[m].row = L.row(dp_has[m], half);
    ms[m].pb = -1;
    for (int u : gf_u) ms[m].coef.push_back(coef[qidx[u]][m]);
  }
  std::vector<XorSrc> xs, self_xs;
  for (int u : gf_u) {
    const int o = static_cast<int>(dst.size()), t = uniq[u];
    dst.push_back(L.row(t, half));
    if (t <= d || (rep[u] & 1) == 0) continue;
    for (int ai : x->xs[t]) xs.push_back({L.row(ai, 0), {o}});
  }
  for (int u : self_u) {
    const int t = uniq[u];
    if (t <= d || (rep[u] & 1) == 0 || x->xs[t].empty()) continue;  // unchanged
    const int o = static_cast<int>(self_dst.size());
    self_dst.push_back(L.row(t, half));
    for (int ai : x->xs[t]) self_xs.push_back({L.row(ai, 0), {o}});
  }
  if (!dst.empty()) {
    e = run_rows(dst, ms, xs, false, half, n_stripes, s);
    if (e) return e;
  }
  if (!self_dst.empty()) {
    e = run_rows(self_dst, {}, self_xs, true, half, n_stripes, s);
    if (e) return e;
  }
  for (int t : uniq) w->add(t, 1);
  return XRS_OK;
}

int update_rows_impl(const xrs_codec* x, RowRef old_row, RowRef new_row, size_t size,
                     const int32_t* rows, int row, const Layout& P, size_t n_stripes,
                     hipStream_t s);

// xrs.go:324-346 Update.  Delta = old ^ new is linear: parity ^= gen[:, row] *
// delta (reedsolomon Update [dep], xrs.go:331) and the piggyback XOR of the
// delta's a-half (:340-344); the update_rows kernel forms the delta first, so
// it does one GF pass (the pair kernel with old and new as two sources would
// do two: measured 3% slower at 4 KiB, profiles/r01_bench_configs_rows.log).
int update_impl(const xrs_codec* x, RowRef old_row, RowRef new_row, size_t size, int row,
                const Layout& P, size_t n_stripes, hipStream_t s) {
  return update_rows_impl(x, old_row, new_row, size, nullptr, row, P, n_stripes, s);
}

// Update with a per-stripe data row (rows: device-readable int32 per stripe),
// or with one `row` for every stripe (rows == nullptr).  Per-stripe rows are
// covered in chunks of kMaxSrc per launch (the kernel skips stripes whose row
// is outside its chunk), outputs in groups of kMaxOut.
int update_rows_impl(const xrs_codec* x, RowRef old_row, RowRef new_row, size_t size,
                     const int32_t* rows, int row, const Layout& P, size_t n_stripes,
                     hipStream_t s) {
  const int d = x->d, p = x->p;
  if (size < 2 || n_stripes == 0) return XRS_OK;
  const GF& gf = GF::get();
  xrs::UpdRowsPlan plan;
  const int first = rows ? 0 : row, last = rows ? d : row + 1;
  for (int g0 = 0; g0 < p; g0 += xrs::kMaxOut) {
    for (int j0 = first; j0 < last; j0 += xrs::kMaxSrc) {
      std::memset(&plan, 0, sizeof(plan));
      plan.P = std::min(xrs::kMaxOut, p - g0);
      plan.row0 = j0;
      plan.nrows = std::min(xrs::kMaxSrc, last - j0);
      for (int j = 0; j < plan.nrows; ++j) {
        for (int q = 0; q < plan.P; ++q) plan.tab[j][q] = gf.tab(x->g(d + g0 + q, j0 + j));
        const int t = x->bi_of[j0 + j] - d - g0;  // xrs.go:340-344 piggyback target
        plan.pbq[j] = (t >= 0 && t < plan.P) ? static_cast<int8_t>(t) : -1;
      }
      plan.old_row = old_row;
      plan.new_row = new_row;
      for (int q = 0; q < plan.P; ++q) plan.dst[q] = P.row(g0 + q, 0);
      plan.rows = reinterpret_cast<uint64_t>(rows);
      plan.half = size / 2;
      plan.n_stripes = n_stripes;
      if (xrs::launch_update_rows(plan, s) != 0) return XRS_ERR_HIP;
    }
  }
  return XRS_OK;
}

int replace_impl(const xrs_codec* x, const Layout& D, const int* rows, int n, size_t size,
                 const Layout& P, size_t n_stripes, hipStream_t s) {
  const int d = x->d, p = x->p;
  std::vector<RowRef> dst;
  for (int r = 0; r < p; ++r) dst.push_back(P.row(r, 0));
  std::vector<MulSrc> src(n);
  for (int i = 0; i < n; ++i) {
    src[i].row = D.row(i, 0);
    src[i].coef.resize(p);
    for (int r = 0; r < p; ++r) src[i].coef[r] = x->g(d + r, rows[i]);  // xrs.go:370
    src[i].pb = x->bi_of[rows[i]] - d;                                   // xrs.go:375-385
  }
  return run_pair(dst, src, true, false, size / 2, n_stripes, s);
}

// Replace / Update argument checks (mirror oracle order; row checks before any write).
int check_replace(const xrs_codec* x, const int* rows, int n, size_t size) {
  if (n < 1) return XRS_ERR_ILLEGAL_VECTS;
  int e = check_size(size);
  if (e) return e;
  if (n > x->d) return XRS_ERR_ILLEGAL_VECTS;
  if (!rows) return XRS_ERR_INVALID_ARG;
  for (int i = 0; i < n; ++i)
    if (rows[i] < 0 || rows[i] >= x->d) return XRS_ERR_ILLEGAL_DATA_INDEX;
  return XRS_OK;
}

// ------------------------------------------------------------- sync API
class DeviceGuard {
 public:
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev_) != hipSuccess) prev_ = -1;
    if (dev >= 0 && dev != prev_) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev_ >= 0) (void)hipSetDevice(prev_);
  }

 private:
  int prev_ = -1;
};

// Ensure the sync stream + `bytes` of staging (caller holds x->mu).
int ensure_staging(const xrs_codec* x, size_t bytes) {
  if (x->device < 0) return XRS_ERR_NO_DEVICE;
  if (!x->stream) {
    if (hipStreamCreateWithFlags(&x->stream, hipStreamNonBlocking) != hipSuccess)
      return XRS_ERR_HIP;
  }
  if (bytes > x->staging_cap) {
    if (x->staging) (void)hipFree(x->staging);
    x->staging = nullptr;
    x->staging_cap = 0;
    size_t cap = std::max<size_t>(bytes, 1 << 20);
    if (hipMalloc(&x->staging, cap) != hipSuccess) return XRS_ERR_HIP;
    x->staging_cap = cap;
  }
  return XRS_OK;
}

int ensure_hstaging(const xrs_codec* x, size_t bytes) {
  if (bytes > x->hstaging_cap) {
    if (x->hstaging) (void)hipHostFree(x->hstaging);
    x->hstaging = x->hstaging_dev = nullptr;
    x->hstaging_cap = 0;
    const size_t cap = std::max<size_t>(bytes, 1 << 20);
    if (hipHostMalloc(&x->hstaging, cap, hipHostMallocMapped) != hipSuccess) return XRS_ERR_HIP;
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, x->hstaging, 0) == hipSuccess) x->hstaging_dev = static_cast<uint8_t*>(dp);
    x->hstaging_cap = cap;
  }
  return XRS_OK;
}

// Wait for everything enqueued on the sync stream.  The stream writes a fresh
// sequence number into a pinned host word after the call's work and the
// caller spins on it: a blocking stream sync sees a small call done several
// us later (a spinning hipStreamQuery sees an empty kernel done 12-16 us after
// its launch call, a host word written by the stream 7.4 us after:
// tools/qlat_probe.hip, profiles/r03_queue_latency_probe.log).  A stream that
// has not written the word after kSpinNs gets a hipStreamSynchronize, which
// also reports a failed launch.  XRS_SYNC_WAIT=block: the plain sync (A/B).
int sync(const xrs_codec* x) {
  constexpr uint64_t kSpinNs = 2000000;
  static const bool block = [] {
    const char* v = std::getenv("XRS_SYNC_WAIT");
    return v && std::strcmp(v, "block") == 0;
  }();
  if (!block && !x->done_word) {
    void* dp = nullptr;
    if (hipHostMalloc(reinterpret_cast<void**>(&x->done_word), 64, hipHostMallocMapped) == hipSuccess &&
        hipHostGetDevicePointer(&dp, x->done_word, 0) == hipSuccess) {
      *x->done_word = x->done_seq;
      x->done_word_dev = static_cast<uint32_t*>(dp);
    } else if (x->done_word) {
      (void)hipHostFree(x->done_word);
      x->done_word = nullptr;
    }
  }
  if (block || !x->done_word ||
      hipStreamWriteValue32(x->stream, x->done_word_dev, ++x->done_seq, 0) != hipSuccess)
    return hip_err(hipStreamSynchronize(x->stream));
  volatile uint32_t* w = x->done_word;
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; *w != x->done_seq; ++i) {
    _mm_pause();
    if ((i & 255) == 255 &&
        std::chrono::steady_clock::now() - t0 > std::chrono::nanoseconds(kSpinNs)) {
      const int e = hip_err(hipStreamSynchronize(x->stream));
      return e ? e : (*w == x->done_seq ? XRS_OK : XRS_ERR_HIP);
    }
  }
  std::atomic_thread_fence(std::memory_order_acquire);  // outputs after the word
  return XRS_OK;
}

size_t env_size(const char* name, size_t dflt) {
  const char* v = std::getenv(name);
  return (v && *v) ? static_cast<size_t>(std::strtoull(v, nullptr, 0)) : dflt;
}

// Concurrent per-stripe calls.  The sync calls of one codec serialize on
// x->mu, so Encode / ReconstOne / Reconst / Update / Replace called per
// stripe from many threads (a Go server's goroutines through the cgo shim)
// would run one at a time, 15-30 us each at 4 KiB.  A call of up to
// kAutoQueueMax bytes per vect that finds the codec busy goes through a
// batching queue for its vect size instead (queue.cpp; created on first use,
// batches of 4 MiB or one stripe, at most kAutoQueues sizes per codec), so
// concurrent callers share device batches (1 MiB vects: one stripe per
// batch, four in flight); a lone caller keeps the direct path.  Same arguments, same results, same
// errors (inputs are validated before the choice).  XRS_AUTO_QUEUE=0 turns
// it off.
constexpr size_t kAutoQueueMax = 1u << 20;
// A staged stripe of at most 16 MiB (12+4 at 1 MiB vects): each queue holds
// at most 6 batches x max(4 MiB, one stripe) of pinned and of device staging.
constexpr size_t kAutoQueueStripeMax = 16u << 20;
constexpr int kAutoQueues = 4;

xrs_queue* auto_queue(const xrs_codec* x, size_t size) {
  static const bool off = [] {
    const char* v = std::getenv("XRS_AUTO_QUEUE");
    return v && v[0] == '0';
  }();
  if (off || size > kAutoQueueMax || (size & 1) || size == 0) return nullptr;
  const size_t stripe = static_cast<size_t>(std::max(x->d + x->p, x->p + 2)) * size;
  if (stripe > kAutoQueueStripeMax) return nullptr;
  std::lock_guard<std::mutex> g(x->aq_mu);
  for (const auto& e : x->aq)
    if (e.first == size) return e.second;  // (nullptr: creation failed once, not retried)
  if (static_cast<int>(x->aq.size()) >= kAutoQueues) return nullptr;
  xrs_queue* q = nullptr;
  if (xrs_queue_new(x, size, std::max<size_t>(1, (4u << 20) / stripe), 50, &q) != XRS_OK) q = nullptr;
  x->aq.push_back({size, q});
  return q;
}

// Base offset that puts the b-half (vect[S/2:]) of a vect staged at a 16-B
// boundary on a 16-B boundary (xrs_batch_layout): 0 when S/2 % 16 == 0.
size_t half_align_offset(size_t size) { return (16 - (size / 2) % 16) % 16; }

// The transfers of one synchronous call (xrs_encode ... xrs_replace), laid out
// as `total` bytes of staging rows:
//  * ZeroCopy (total <= XRS_SYNC_ZC_MAX, default 4 MiB): inputs are
//    gathered by CPU memcpy into the pinned mirror and the kernel reads and
//    writes the mirror in place over PCIe: no DMA, one launch, one sync.
//  * Pinned (total <= 8 MiB): the same gather, then one H2D of the touched
//    span, the kernel, one D2H of the written span.
//  * Direct: one copy per vect straight to / from device staging.
// Outputs are scattered to the caller's buffers after the sync.
class Stage {
 public:
  enum Mode { kZeroCopy, kPinned, kDirect };

  // `vect` = the call's vect size: the staged rows start at the odd-size base
  // offset (half_align_offset), so every b-half of an odd vect size is as
  // aligned as in a batch laid out by xrs_batch_layout.
  Stage(const xrs_codec* x, size_t total, size_t vect)
      : x_(x), bo_(half_align_offset(vect)), total_(std::max<size_t>(total, 1) + bo_) {}

  int init() {
    int e = ensure_staging(x_, mode_for() == kZeroCopy ? 1 : total_);  // also creates the stream
    if (e) return e;
    mode_ = mode_for();
    if (mode_ != kDirect) {
      if ((e = ensure_hstaging(x_, total_))) return e;
      if (mode_ == kZeroCopy && !x_->hstaging_dev) {
        mode_ = kPinned;
        if ((e = ensure_staging(x_, total_))) return e;
      }
    }
    return XRS_OK;
  }
  uint8_t* base() const { return (mode_ == kZeroCopy ? x_->hstaging_dev : x_->staging) + bo_; }
  Layout layout(size_t shard_stride, size_t off = 0) const { return {base() + off, shard_stride, total_}; }

  int in(size_t off, const void* src, size_t n) {
    if (n == 0) return XRS_OK;
    if (!src) return XRS_ERR_INVALID_ARG;
    off += bo_;
    if (mode_ == kDirect)
      return hip_err(hipMemcpyAsync(x_->staging + off, src, n, hipMemcpyHostToDevice, x_->stream));
    std::memcpy(x_->hstaging + off, src, n);
    in_lo_ = std::min(in_lo_, off);
    in_hi_ = std::max(in_hi_, off + n);
    return XRS_OK;
  }
  // After the last in(), before the kernel.
  int upload() {
    if (mode_ != kPinned || in_hi_ <= in_lo_) return XRS_OK;
    return hip_err(hipMemcpyAsync(x_->staging + in_lo_, x_->hstaging + in_lo_, in_hi_ - in_lo_,
                                  hipMemcpyHostToDevice, x_->stream));
  }
  void out(void* dst, size_t off, size_t n) {
    if (n == 0) return;
    off += bo_;
    outs_.push_back({dst, off, n});
    out_lo_ = std::min(out_lo_, off);
    out_hi_ = std::max(out_hi_, off + n);
  }
  // After the kernel(s): download, sync, scatter.  Returns a transfer error.
  int finish() {
    int e = XRS_OK;
    if (mode_ == kDirect) {
      for (const Out& o : outs_)
        if (!e) e = hip_err(hipMemcpyAsync(o.dst, x_->staging + o.off, o.n, hipMemcpyDeviceToHost, x_->stream));
    } else if (mode_ == kPinned && out_hi_ > out_lo_) {
      e = hip_err(hipMemcpyAsync(x_->hstaging + out_lo_, x_->staging + out_lo_, out_hi_ - out_lo_,
                                 hipMemcpyDeviceToHost, x_->stream));
    }
    const int es = sync(x_);
    if (e || es) return e ? e : es;
    if (mode_ != kDirect)
      for (const Out& o : outs_) std::memcpy(o.dst, x_->hstaging + o.off, o.n);
    return XRS_OK;
  }

 private:
  struct Out {
    void* dst;
    size_t off, n;
  };
  Mode mode_for() const {
    if (total_ <= env_size("XRS_SYNC_ZC_MAX", 4u << 20)) return kZeroCopy;
    if (total_ <= env_size("XRS_SYNC_PINNED_MAX", 8u << 20)) return kPinned;
    return kDirect;
  }
  const xrs_codec* x_;
  size_t bo_;     // odd-size base offset of the staged rows (0..15)
  size_t total_;  // staging bytes, bo_ included
  Mode mode_ = kDirect;
  size_t in_lo_ = SIZE_MAX, in_hi_ = 0, out_lo_ = SIZE_MAX, out_hi_ = 0;
  std::vector<Out> outs_;
};

// ---------------------------------------------------- host-resident pipeline
constexpr size_t kChunkBytes = 64u << 20;  // device bytes per pipeline chunk

int ensure_pipe(const xrs_codec* x, size_t bytes, size_t bounce) {
  if (x->device < 0) return XRS_ERR_NO_DEVICE;
  for (int i = 0; i < xrs_codec::kPipe; ++i)
    if (!x->pstream[i] && hipStreamCreateWithFlags(&x->pstream[i], hipStreamNonBlocking) != hipSuccess)
      return XRS_ERR_HIP;
  if (bytes > x->slot_cap) {
    for (int i = 0; i < xrs_codec::kPipe; ++i) {
      if (x->slot[i]) (void)hipFree(x->slot[i]);
      x->slot[i] = nullptr;
    }
    x->slot_cap = 0;
    for (int i = 0; i < xrs_codec::kPipe; ++i)
      if (hipMalloc(&x->slot[i], bytes) != hipSuccess) return XRS_ERR_HIP;
    x->slot_cap = bytes;
  }
  if (bounce > x->bounce_cap) {
    for (int i = 0; i < xrs_codec::kPipe; ++i) {
      if (x->bounce[i]) (void)hipHostFree(x->bounce[i]);
      x->bounce[i] = nullptr;
    }
    x->bounce_cap = 0;
    for (int i = 0; i < xrs_codec::kPipe; ++i)
      if (hipHostMalloc(reinterpret_cast<void**>(&x->bounce[i]), bounce, hipHostMallocDefault) != hipSuccess)
        return XRS_ERR_HIP;
    x->bounce_cap = bounce;
  }
  return XRS_OK;
}

// ----------------------------------------------------- DMA-clean row copies
// The runtime's rectangular DMA copy (hipMemcpy2DAsync) needs both row bases
// 4-byte aligned and both pitches multiples of 4 (any width is fine).  A
// misaligned base is refused ("DMA buffer failed with code 4097") and the
// copy falls back to 5.6 GB/s H2D, 12-14 GB/s D2H; a pitch that is not a
// multiple of 4 runs row by row at 0.56-0.61 GB/s; aligned copies run at
// 47-49 GB/s (tools/dma_rect_probe.cpp, profiles/r06_dma_rect_probe.log).
// Odd vect sizes put rows on every residue, so the copies below keep every
// rectangle aligned for any host layout, given a device image whose rows
// have the host rows' address residues mod 4 (dev = host, dpitch = hpitch,
// mod 4; or a mirror of the host bytes, as the queue's staging is):
//  * a row set is split into k = 1, 2, 4 (or 8) pitch groups (every k-th
//    row), so every group's pitches are multiples of 4 and at least as long
//    as its widened rows;
//  * host to device, each row starts at its enclosing aligned word (at most 3
//    bytes more, read from the same word; the device image has slack there);
//  * device to host, the aligned body of each row is copied straight back,
//    and its 1-3 head bytes go through a pinned bounce buffer that the CPU
//    writes back once the stream has finished (HeadFix) -- or, into a mirror,
//    widened like host to device.
inline size_t res4(const void* p) { return reinterpret_cast<uintptr_t>(p) & 3u; }
inline size_t pitch_groups(size_t a, size_t b) {
  const size_t r = (a | b) & 3u;
  return r == 0 ? 1 : (r & 1u) ? 4 : 2;
}

// Head bytes of device-to-host rows whose host start is not 4-byte aligned:
// rows t < rows of the group at host + t * pitch get n bytes from
// words + 4 * t + m once the copies into `words` have finished.
struct HeadFix {
  uint8_t* host;
  size_t pitch, rows, m, n;
  const uint8_t* words;
};
struct HeadBounce {
  uint8_t* buf = nullptr;  // pinned
  size_t cap = 0, used = 0;
  std::vector<HeadFix> fixes;
  uint8_t* take(size_t n) {
    if (!buf || used + n > cap) return nullptr;
    uint8_t* p = buf + used;
    used += n;
    return p;
  }
  void apply() {
    for (const HeadFix& f : fixes)
      for (size_t t = 0; t < f.rows; ++t) std::memcpy(f.host + t * f.pitch, f.words + 4 * t + f.m, f.n);
    fixes.clear();
    used = 0;
  }
};

// `rows` rows of `len` bytes between host (row r at host + r * hp) and device
// (dev + r * dp).  H2D always widens; D2H widens when `mirror`, else it takes
// the head bytes through `hb`.
int copy_rows(hipMemcpyKind kind, uint8_t* dev, size_t dp, uint8_t* host, size_t hp, size_t len,
              size_t rows, hipStream_t s, bool mirror, HeadBounce* hb) {
  if (!len || !rows) return XRS_OK;
  // (a widened row may be longer than the pitch -- back-to-back rows, or a
  // whole staged stripe -- and a rectangle's width may not exceed its pitch:
  // then every 2nd or 4th row)
  size_t k = pitch_groups(hp, dp);
  const size_t slack = (((hp | dp) & 3u) || res4(host)) ? 3 : 0;  // widening, at most
  while (k < 8 && (k * hp < len + slack || k * dp < len + slack)) k *= 2;
  for (size_t g = 0; g < k && g < rows; ++g) {
    uint8_t* h = host + g * hp;
    uint8_t* d = dev + g * dp;
    const size_t n = (rows - g + k - 1) / k, m = res4(h);
    if (res4(d) != m) return XRS_ERR_INVALID_ARG;  // (the image guarantees it)
    hipError_t r = hipSuccess;
    if (kind == hipMemcpyHostToDevice || mirror) {
      const size_t w = m + len;  // (the width needs no alignment)
      r = kind == hipMemcpyHostToDevice
              ? hipMemcpy2DAsync(d - m, k * dp, h - m, k * hp, w, n, kind, s)
              : hipMemcpy2DAsync(h - m, k * hp, d - m, k * dp, w, n, kind, s);
    } else if (m == 0) {
      r = hipMemcpy2DAsync(h, k * hp, d, k * dp, len, n, kind, s);
    } else {
      const size_t head = std::min(4 - m, len);
      if (len > head) r = hipMemcpy2DAsync(h + head, k * hp, d + head, k * dp, len - head, n, kind, s);
      uint8_t* words = hb ? hb->take(4 * n) : nullptr;
      if (!words) return XRS_ERR_INVALID_ARG;
      if (r == hipSuccess) r = hipMemcpy2DAsync(words, 4, d - m, k * dp, 4, n, kind, s);
      hb->fixes.push_back({h, k * hp, n, m, head, words});
    }
    if (r != hipSuccess) return XRS_ERR_HIP;
  }
  return XRS_OK;
}

// The device image of a set of host rows that share one stripe pitch: row j
// of stripe s at host0[j] + s * hp on the host, at chunk_slot + region +
// off[j] + s * dp on the device.
//  * compact (every copy of the op is already DMA-clean in it): rows back to
//    back from the odd-size base offset, as a recommended device batch
//    (half_align_offset) -- the layout the pipeline always had;
//  * otherwise residue-matched: off[j] = host0[j] and dp = hp (mod 4), 32 B
//    of slack around every row, the b-half on the 16-byte boundary where the
//    residue allows it.
struct Image {
  std::vector<uint8_t*> host0;
  size_t hp = 0, len = 0;  // host pitch, row (vect) length
  bool compact = true;
  std::vector<size_t> off;
  size_t dp = 0, region = 0;
};
// A copy of part of row `row` of image `im`: bytes [at, at + len).
struct Piece {
  int im, row;
  size_t at, len;
};

void plan_image(Image* im, const std::vector<Piece>& pieces, int idx) {
  const size_t S = im->len, H = S / 2, m = im->host0.size(), bo = half_align_offset(S);
  bool clean = (im->hp & 3u) == 0 && ((m * S) & 3u) == 0;
  for (const Piece& p : pieces)
    if (p.im == idx)
      clean = clean && res4(im->host0[p.row] + p.at) == 0 && ((bo + p.row * S + p.at) & 3u) == 0;
  im->compact = clean;
  im->off.assign(m, 0);
  if (clean) {
    for (size_t j = 0; j < m; ++j) im->off[j] = bo + j * S;
    im->dp = m * S;
    return;
  }
  const size_t S16 = ((S + 15) & ~size_t(15)) + 32, t = (16 - H % 16) % 16;
  for (size_t j = 0; j < m; ++j) {
    const size_t o = (t + ((res4(im->host0[j]) - t) & 3u)) & 15u;  // = host0[j] (mod 4)
    im->off[j] = 16 + j * S16 + o;
  }
  im->dp = 16 + m * S16 + (im->hp & 3u);  // = hp (mod 4)
}

// The op's layout over image `im` in a chunk slot (tab: per-row bases of a
// residue-matched image, which Layout reads at launch).
Layout image_layout(const Image& im, uint8_t* slot, std::vector<uint64_t>* tab) {
  if (im.compact) return {slot + im.region + im.off[0], im.len, im.dp};
  tab->resize(im.off.size());
  for (size_t j = 0; j < im.off.size(); ++j)
    (*tab)[j] = reinterpret_cast<uint64_t>(slot + im.region + im.off[j]);
  return {nullptr, 0, im.dp, tab->data()};
}

// Chunked H2D -> kernel -> D2H over kPipe streams.  `in` / `out` list the
// pieces moved per stripe; launch(slot, n, stream) runs the op on the chunk's
// device images (image_layout).  Images and pieces as above.
template <class Launch>
int run_pipeline(const xrs_codec* x, std::vector<Image>& ims, size_t n_stripes,
                 const std::vector<Piece>& in, const std::vector<Piece>& out, Launch launch) {
  std::vector<Piece> all(in);
  all.insert(all.end(), out.begin(), out.end());
  size_t rows_bytes = 0;  // (chunks are sized by the rows, not the slack)
  for (size_t i = 0; i < ims.size(); ++i) {
    plan_image(&ims[i], all, static_cast<int>(i));
    rows_bytes += ims[i].len * ims[i].host0.size();
  }
  const size_t chunk = std::max<size_t>(1, std::min(n_stripes, kChunkBytes / rows_bytes));
  size_t bytes = 0;
  for (Image& im : ims) {  // each image's chunk region, 256-byte aligned
    im.region = bytes;
    bytes += (chunk * im.dp + 255) & ~size_t(255);
  }
  std::lock_guard<std::mutex> lk(x->pipe_mu);
  DeviceGuard g(x->device);
  int e = ensure_pipe(x, bytes, std::max<size_t>(4096, out.size() * chunk * 4));
  if (e) return e;
  HeadBounce hb[xrs_codec::kPipe];
  for (int k = 0; k < xrs_codec::kPipe; ++k) {
    hb[k].buf = x->bounce[k];
    hb[k].cap = x->bounce_cap;
  }
  size_t i = 0;
  for (size_t c0 = 0; c0 < n_stripes && !e; c0 += chunk, ++i) {
    const int si = static_cast<int>(i % xrs_codec::kPipe);
    hipStream_t st = x->pstream[si];
    if (!hb[si].fixes.empty()) {  // this slot's previous chunk: its head bytes
      if (hipStreamSynchronize(st) != hipSuccess) {
        e = XRS_ERR_HIP;
        break;
      }
      hb[si].apply();
    }
    uint8_t* slot = x->slot[si];
    const size_t nc = std::min(chunk, n_stripes - c0);
    auto dev_at = [&](const Piece& p) {
      const Image& im = ims[p.im];
      return slot + im.region + im.off[p.row] + p.at;
    };
    auto host_at = [&](const Piece& p) {
      const Image& im = ims[p.im];
      return im.host0[p.row] + c0 * im.hp + p.at;
    };
    for (const Piece& p : in)
      if (!e)
        e = copy_rows(hipMemcpyHostToDevice, dev_at(p), ims[p.im].dp, host_at(p), ims[p.im].hp,
                      p.len, nc, st, false, nullptr);
    if (!e) e = launch(slot, nc, st);
    for (const Piece& p : out)
      if (!e)
        e = copy_rows(hipMemcpyDeviceToHost, dev_at(p), ims[p.im].dp, host_at(p), ims[p.im].hp,
                      p.len, nc, st, false, &hb[si]);
  }
  int es = XRS_OK;
  for (int k = 0; k < xrs_codec::kPipe; ++k)
    if (hipStreamSynchronize(x->pstream[k]) != hipSuccess) es = XRS_ERR_HIP;
  if (!e && !es)
    for (HeadBounce& b : hb) b.apply();
  return e ? e : es;
}

// One image of a host batch's d+p shards (shard j of stripe s at base +
// s * stripe_stride + j * shard_stride), and its pieces: (shard, half) with
// half 0 = a, 1 = b, 2 = the whole vect.
Image batch_image(const xrs_codec* x, uint8_t* base, size_t size, size_t shard_stride,
                  size_t stripe_stride) {
  Image im;
  for (int j = 0; j < x->d + x->p; ++j) im.host0.push_back(base + static_cast<size_t>(j) * shard_stride);
  im.hp = stripe_stride;
  im.len = size;
  return im;
}
std::vector<Piece> halves(const std::vector<std::pair<int, int>>& hs, size_t size) {
  std::vector<Piece> v;
  for (const auto& h : hs)
    v.push_back({0, h.first, h.second == 1 ? size / 2 : 0, h.second == 2 ? size : size / 2});
  return v;
}

bool vects_ok(uint8_t* const* v, int n) {
  if (!v) return false;
  for (int i = 0; i < n; ++i)
    if (!v[i]) return false;
  return true;
}

}  // namespace

// Entry points for the other translation units of the library (queue.cpp).
namespace xrs_detail {
int encode_dev(const xrs_codec* x, uint8_t* base, size_t size, size_t shard_stride,
               size_t stripe_stride, size_t n_stripes, void* stream) {
  return encode_impl(x, {base, shard_stride, stripe_stride}, size, n_stripes,
                     static_cast<hipStream_t>(stream));
}
int reconst_one_dev(const xrs_codec* x, uint8_t* base, size_t size, size_t shard_stride,
                    size_t stripe_stride, size_t n_stripes, int k, void* stream) {
  return reconst_one_impl(x, {base, shard_stride, stripe_stride}, size, n_stripes, k,
                          static_cast<hipStream_t>(stream));
}
int need_set(const xrs_codec* x, int k, std::vector<int>* a_need, int* bi) {
  return need_vects(x, k, a_need, bi);
}
// The queue's batches of callers' own buffers: stripe s's rows through the
// table at tab + s * tab_stride bytes (two entries per staged row, a- and
// b-half; Layout::ind).  Rows are numbered as in the queue's staging: Encode,
// ReconstOne, Reconst the d+p vects; Update [0, p) parity, p old, p+1 new;
// Replace [0, p) parity, [p, p+n) data.
int encode_table(const xrs_codec* x, const uint64_t* tab, size_t tab_stride, size_t size,
                 size_t n, void* stream) {
  return encode_impl(x, {nullptr, 0, 0, nullptr, tab, tab_stride}, size, n,
                     static_cast<hipStream_t>(stream));
}
int reconst_one_table(const xrs_codec* x, const uint64_t* tab, size_t tab_stride, size_t size,
                      size_t n, int k, void* stream) {
  return reconst_one_impl(x, {nullptr, 0, 0, nullptr, tab, tab_stride}, size, n, k,
                          static_cast<hipStream_t>(stream));
}
int reconst_table(const xrs_codec* x, const uint64_t* tab, size_t tab_stride, size_t size, size_t n,
                  const int* dp_has, int n_has, const int* need, int n_need, void* stream) {
  Written w;
  return reconst_impl(x, {nullptr, 0, 0, nullptr, tab, tab_stride}, size, n, dp_has, n_has, need,
                      n_need, static_cast<hipStream_t>(stream), &w);
}
int update_rows_table(const xrs_codec* x, const uint64_t* tab, size_t tab_stride, size_t size,
                      const int32_t* rows, size_t n, void* stream) {
  const Layout L{nullptr, 0, 0, nullptr, tab, tab_stride};
  return update_rows_impl(x, L.row(x->p, 0), L.row(x->p + 1, 0), size, rows, 0, L, n,
                          static_cast<hipStream_t>(stream));
}
int replace_table(const xrs_codec* x, const uint64_t* tab, size_t tab_stride, const int* rows,
                  int n_rows, size_t size, size_t n, void* stream) {
  const Layout P{nullptr, 0, 0, nullptr, tab, tab_stride};
  const Layout D{nullptr, 0, 0, nullptr, tab + 2 * x->p, tab_stride};
  return replace_impl(x, D, rows, n_rows, size, P, n, static_cast<hipStream_t>(stream));
}
// The queue's staging copies (its pinned staging and device batch are
// mirrors: same offsets, same pitch): DMA-clean for any vect size.
int copy_rows_mirror(bool to_device, uint8_t* dev, uint8_t* host, size_t pitch, size_t len,
                     size_t rows, void* stream) {
  return copy_rows(to_device ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost, dev, pitch, host,
                   pitch, len, rows, static_cast<hipStream_t>(stream), true, nullptr);
}
int codec_device(const xrs_codec* x) { return x->device; }
int codec_d(const xrs_codec* x) { return x->d; }
int codec_p(const xrs_codec* x) { return x->p; }
}  // namespace xrs_detail

// ====================================================================== C ABI
extern "C" {

const char* xrs_strerror(int code) {
  switch (code) {
    case XRS_OK: return "ok";
    case XRS_ERR_ILLEGAL_PARITY: return "illegal parity";
    case XRS_ERR_SIZE_NOT_EVEN: return "vect size not even";
    case XRS_ERR_ILLEGAL_DATA_INDEX: return "illegal data index";
    case XRS_ERR_ILLEGAL_VECTS: return "illegal vects";
    case XRS_ERR_TOO_FEW_SURVIVORS: return "too few survivors";
    case XRS_ERR_ILLEGAL_INDEX: return "illegal index";
    case XRS_ERR_SINGULAR: return "singular matrix";
    case XRS_ERR_HIP: return "hip runtime error";
    case XRS_ERR_INVALID_ARG: return "invalid argument";
    case XRS_ERR_NO_DEVICE: return "no gpu device";
    case XRS_ERR_BUSY: return "queue busy";
    default: return "unknown error";
  }
}

int xrs_format_error(int code, long long arg, char* buf, size_t buflen) {
  if (!buf || buflen == 0) return 0;
  int n;
  if (code == XRS_ERR_SIZE_NOT_EVEN)
    n = std::snprintf(buf, buflen, "vect size not even: %lld", arg);  // xrs.go:133
  else if (code == XRS_ERR_ILLEGAL_DATA_INDEX)
    n = std::snprintf(buf, buflen, "illegal data index: %lld", arg);  // xrs.go:149
  else
    n = std::snprintf(buf, buflen, "%s", xrs_strerror(code));
  return n < 0 ? 0 : n;
}

int xrs_trace_kernels(int on) {
  xrs::trace_kernels(on != 0);
  return XRS_OK;
}

size_t xrs_traced_kernels(char* buf, size_t cap) { return xrs::traced_kernels(buf, cap); }

// xrs.go:55-68 New + makeXORSet :77-100
int xrs_new(int data_num, int parity_num, xrs_codec** out) {
  if (!out) return XRS_ERR_INVALID_ARG;
  *out = nullptr;
  if (parity_num == 1) return XRS_ERR_ILLEGAL_PARITY;  // xrs.go:56-59
  if (data_num <= 0 || parity_num <= 0 || data_num + parity_num > 256) return XRS_ERR_ILLEGAL_VECTS;
  const GF& gf = GF::get();
  auto* x = new xrs_codec();
  const int d = data_num, p = parity_num, n = d + p;
  x->d = d;
  x->p = p;
  x->gen.assign(static_cast<size_t>(n) * d, 0);
  for (int i = 0; i < d; ++i) x->gen[static_cast<size_t>(i) * d + i] = 1;
  for (int i = d; i < n; ++i)
    for (int j = 0; j < d; ++j) x->gen[static_cast<size_t>(i) * d + j] = gf.inv(static_cast<uint8_t>(i ^ j));
  x->xs.assign(n, {});
  x->bi_of.assign(d, 0);
  int j = d + 1;
  for (int i = 0; i < d; ++i) {
    if (j > d + p - 1) j = d + 1;
    x->xs[j].push_back(i);
    x->bi_of[i] = j;
    ++j;
  }
  x->r1_bk.assign(d, {});  // ReconstOne plans: built on first use of each k
  x->r1_brs.assign(d, {});
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  int count = 0;
  if (dev >= 0 && (hipGetDeviceCount(&count) != hipSuccess || count <= 0)) dev = -1;
  x->device = dev;
  // Encode padding rows and the persistent kernel's tile counters of the
  // codec's device, made here so a launch on it never allocates (a launch on
  // another device's stream makes that device's on first use)
  if (dev >= 0) {
    (void)xrs::zero_rows(dev);
    (void)xrs::tile_counters(dev);
  }
  *out = x;
  return XRS_OK;
}

void xrs_free(xrs_codec* x) {
  if (!x) return;
  for (const auto& e : x->aq) xrs_queue_free(e.second);
  if (x->device >= 0) {
    DeviceGuard g(x->device);
    if (x->stream) (void)hipStreamDestroy(x->stream);
    if (x->staging) (void)hipFree(x->staging);
    if (x->hstaging) (void)hipHostFree(x->hstaging);
    if (x->done_word) (void)hipHostFree(x->done_word);
    for (int i = 0; i < xrs_codec::kPipe; ++i) {
      if (x->pstream[i]) (void)hipStreamDestroy(x->pstream[i]);
      if (x->slot[i]) (void)hipFree(x->slot[i]);
      if (x->bounce[i]) (void)hipHostFree(x->bounce[i]);
    }
  }
  delete x;
}

int xrs_data_num(const xrs_codec* x) { return x ? x->d : XRS_ERR_INVALID_ARG; }
int xrs_parity_num(const xrs_codec* x) { return x ? x->p : XRS_ERR_INVALID_ARG; }

int xrs_gen_matrix(const xrs_codec* x, uint8_t* out, size_t cap) {
  if (!x || !out || cap < x->gen.size()) return XRS_ERR_INVALID_ARG;
  std::memcpy(out, x->gen.data(), x->gen.size());
  return XRS_OK;
}

int xrs_xorset(const xrs_codec* x, int parity_index, int* data_idx, int cap, int* len) {
  if (!x || !len) return XRS_ERR_INVALID_ARG;
  *len = 0;
  if (parity_index < 0 || parity_index >= x->d + x->p) return XRS_OK;
  const auto& v = x->xs[parity_index];
  if (static_cast<int>(v.size()) > cap || (!data_idx && !v.empty())) return XRS_ERR_INVALID_ARG;
  for (size_t i = 0; i < v.size(); ++i) data_idx[i] = v[i];
  *len = static_cast<int>(v.size());
  return XRS_OK;
}

// xrs.go:146-171
int xrs_get_need_vects(const xrs_codec* x, int k, int* a_need, int* a_len, int b_need[2]) {
  if (!x || !a_len || !b_need) return XRS_ERR_INVALID_ARG;
  std::vector<int> an;
  int bi = 0;
  const int e = need_vects(x, k, &an, &bi);
  if (e) return e;
  if (!a_need && !an.empty()) return XRS_ERR_INVALID_ARG;
  for (size_t i = 0; i < an.size(); ++i) a_need[i] = an[i];
  *a_len = static_cast<int>(an.size());
  b_need[0] = x->d;
  b_need[1] = bi;
  return XRS_OK;
}

// ---------------------------------------------------------------- batched
int xrs_batch_strides(size_t size, int n_shards, size_t* shard_stride, size_t* stripe_stride) {
  if (!shard_stride || !stripe_stride || n_shards < 1) return XRS_ERR_INVALID_ARG;
  // With the XCD-aware block order (kernels.hip) back-to-back shards stream
  // as fast as padded ones below 4 MiB; 8 MiB Encode still gains ~3% from a
  // 4 KiB + 256 B pad (profiles/r01_order_ab.log).  A vect size that is not a
  // multiple of 16 stays back to back below 32 KiB (the kernels take any
  // alignment) and is rounded up to 16 from there: the rate follows the
  // stride through the HBM address mapping, and a 16-rounded stride of
  // 4,100-B vects (4,112) ran Encode / ReconstOne 17% / 8% slower than the
  // back-to-back 4,100, while at 64 KiB + 2 and 1 MiB + 2 the rounded
  // stride is 4-5% faster (tools/stride_probe.py, profiles/r02_stride_probe.log).
  // The stripe stride is rounded up to a power of two when that costs at most
  // 1/7 of the packed stripe: a power-of-two stripe streams ReconstOne at
  // 4-16 KiB vects 6-16% faster (12+3 @ 4 KiB 0.657 -> 0.752 of 8 TB/s, 10+4
  // +10%, 13+2 +16%) and Encode 0-5%; from 64 KiB up it moves both by
  // -1.3..+3.7% (tools/layout_ab.py, profiles/r02_layout_*.log).
  // Callers size a batch as n_stripes * stripe_stride (which may exceed
  // n_shards * shard_stride by up to 1/7).  Sizes whose strides would not fit
  // in size_t are refused.
  const size_t pad = size >= (4u << 20) ? 4096 + 256 : 0;
  if (size > SIZE_MAX / 2 / static_cast<size_t>(n_shards)) return XRS_ERR_INVALID_ARG;
  const size_t s = (size % 16 && size < (32u << 10)) ? size : (size + 15) / 16 * 16 + pad;
  const size_t packed = s * static_cast<size_t>(n_shards);
  size_t p2 = 1;
  while (p2 < packed && p2 <= SIZE_MAX / 2) p2 <<= 1;
  if (p2 < packed) p2 = packed;  // no power of two above packed fits: keep it packed
  *shard_stride = s;
  *stripe_stride = (p2 - packed) <= packed / 7 ? p2 : packed;
  return XRS_OK;
}

int xrs_batch_layout(size_t size, int n_shards, size_t* shard_stride, size_t* stripe_stride,
                     size_t* base_offset) {
  if (!base_offset) return XRS_ERR_INVALID_ARG;
  const int e = xrs_batch_strides(size, n_shards, shard_stride, stripe_stride);
  if (e) return e;
  // An odd half (a vect size that is not a multiple of 32) leaves every
  // b-half (vect[S/2:]) off 16-B alignment when the a-halves are aligned.
  // ReconstOne reads 13 b-halves and 3 a-halves of 12+4, so the batch is
  // shifted to put shard 0's b-half on a 16-B boundary: with the recommended
  // strides every b-half is then 4-B (4,100, 4,098 B) or 16-B (1 MiB + 2)
  // aligned.  Measured on MI355X (tools/layout_ab.py,
  // profiles/r03_layout_odd.log, fraction of 8 TB/s): ReconstOne 4,100 B
  // 0.602 -> 0.684, 4,098 B 0.594 -> 0.663, 1 MiB + 2 0.643 -> 0.716;
  // 2-lost Reconst +2..+8%; Encode unchanged (reads a- and b-halves alike).
  *base_offset = half_align_offset(size);
  return XRS_OK;
}

int xrs_encode_batched(const xrs_codec* x, uint8_t* base, size_t size, size_t shard_stride,
                       size_t stripe_stride, size_t n_stripes, void* stream) {
  if (!x) return XRS_ERR_INVALID_ARG;
  int e = check_size(size);
  if (e) return e;
  if (n_stripes == 0 || size == 0) return XRS_OK;
  if (!base) return XRS_ERR_INVALID_ARG;
  if (x->device < 0) return XRS_ERR_NO_DEVICE;
  return encode_impl(x, {base, shard_stride, stripe_stride}, size, n_stripes,
                     static_cast<hipStream_t>(stream));
}

int xrs_reconst_one_batched(const xrs_codec* x, uint8_t* base, size_t size, size_t shard_stride,
                            size_t stripe_stride, size_t n_stripes, int k, void* stream) {
  if (!x) return XRS_ERR_INVALID_ARG;
  int e = check_size(size);
  if (e) return e;
  if (k < 0 || k >= x->d) return XRS_ERR_ILLEGAL_DATA_INDEX;
  if (n_stripes == 0 || size == 0) return XRS_OK;
  if (!base) return XRS_ERR_INVALID_ARG;
  if (x->device < 0) return XRS_ERR_NO_DEVICE;
  return reconst_one_impl(x, {base, shard_stride, stripe_stride}, size, n_stripes, k,
                          static_cast<hipStream_t>(stream));
}

int xrs_reconst_batched(const xrs_codec* x, uint8_t* base, size_t size, size_t shard_stride,
                        size_t stripe_stride, size_t n_stripes, const int* dp_has, int n_has,
                        const int* need, int n_need, void* stream) {
  if (!x || n_has < 0 || n_need < 0 || (n_has && !dp_has) || (n_need && !need))
    return XRS_ERR_INVALID_ARG;
  if (n_need == 1 && need[0] < x->d)  // xrs.go:238-240
    return xrs_reconst_one_batched(x, base, size, shard_stride, stripe_stride, n_stripes, need[0],
                                   stream);
  int e = check_size(size);
  if (e) return e;
  if (x->device < 0) return XRS_ERR_NO_DEVICE;
  Written w;
  const size_t ns = (size == 0 || !base) ? 0 : n_stripes;
  return reconst_impl(x, {base, shard_stride, stripe_stride}, size, ns, dp_has, n_has, need,
                      n_need, static_cast<hipStream_t>(stream), &w);
}

int xrs_update_batched(const xrs_codec* x, const uint8_t* old_base, size_t old_stripe_stride,
                       const uint8_t* new_base, size_t new_stripe_stride, size_t size, int row,
                       uint8_t* parity_base, size_t parity_shard_stride,
                       size_t parity_stripe_stride, size_t n_stripes, void* stream) {
  if (!x) return XRS_ERR_INVALID_ARG;
  int e = check_size(size);
  if (e) return e;
  if (row < 0 || row >= x->d) return XRS_ERR_ILLEGAL_DATA_INDEX;
  if (n_stripes == 0 || size == 0) return XRS_OK;
  if (!old_base || !new_base || !parity_base) return XRS_ERR_INVALID_ARG;
  if (x->device < 0) return XRS_ERR_NO_DEVICE;
  const RowRef o{reinterpret_cast<uint64_t>(old_base), old_stripe_stride};
  const RowRef nw{reinterpret_cast<uint64_t>(new_base), new_stripe_stride};
  return update_impl(x, o, nw, size, row, {parity_base, parity_shard_stride, parity_stripe_stride},
                     n_stripes, static_cast<hipStream_t>(stream));
}

int xrs_update_rows_batched(const xrs_codec* x, const uint8_t* old_base,
                            size_t old_stripe_stride, const uint8_t* new_base,
                            size_t new_stripe_stride, size_t size, const int32_t* rows,
                            uint8_t* parity_base, size_t parity_shard_stride,
                            size_t parity_stripe_stride, size_t n_stripes, void* stream) {
  if (!x) return XRS_ERR_INVALID_ARG;
  int e = check_size(size);
  if (e) return e;
  if (n_stripes == 0 || size == 0) return XRS_OK;
  if (!old_base || !new_base || !parity_base || !rows) return XRS_ERR_INVALID_ARG;
  if (x->device < 0) return XRS_ERR_NO_DEVICE;
  const RowRef o{reinterpret_cast<uint64_t>(old_base), old_stripe_stride};
  const RowRef nw{reinterpret_cast<uint64_t>(new_base), new_stripe_stride};
  return update_rows_impl(x, o, nw, size, rows, 0,
                          {parity_base, parity_shard_stride, parity_stripe_stride}, n_stripes,
                          static_cast<hipStream_t>(stream));
}

int xrs_replace_batched(const xrs_codec* x, const uint8_t* data_base, size_t data_shard_stride,
                        size_t data_stripe_stride, const int* rows, int n, size_t size,
                        uint8_t* parity_base, size_t parity_shard_stride,
                        size_t parity_stripe_stride, size_t n_stripes, void* stream) {
  if (!x) return XRS_ERR_INVALID_ARG;
  int e = check_replace(x, rows, n, size);
  if (e) return e;
  if (n_stripes == 0 || size == 0) return XRS_OK;
  if (!data_base || !parity_base) return XRS_ERR_INVALID_ARG;
  if (x->device < 0) return XRS_ERR_NO_DEVICE;
  return replace_impl(x, {const_cast<uint8_t*>(data_base), data_shard_stride, data_stripe_stride},
                      rows, n, size, {parity_base, parity_shard_stride, parity_stripe_stride},
                      n_stripes, static_cast<hipStream_t>(stream));
}

// ------------------------------------------------------ per-shard pointer tables
static bool table_ok(uint8_t* const* shards, int n) {
  if (!shards) return false;
  for (int i = 0; i < n; ++i)
    if (!shards[i]) return false;
  return true;
}

int xrs_encode_shards(const xrs_codec* x, uint8_t* const* shards, size_t stripe_stride,
                      size_t size, size_t n_stripes, void* stream) {
  if (!x) return XRS_ERR_INVALID_ARG;
  int e = check_size(size);
  if (e) return e;
  if (n_stripes == 0 || size == 0) return XRS_OK;
  if (!table_ok(shards, x->d + x->p)) return XRS_ERR_INVALID_ARG;
  if (x->device < 0) return XRS_ERR_NO_DEVICE;
  std::vector<uint64_t> t(x->d + x->p);
  for (int i = 0; i < x->d + x->p; ++i) t[i] = reinterpret_cast<uint64_t>(shards[i]);
  return encode_impl(x, {nullptr, 0, stripe_stride, t.data()}, size, n_stripes,
                     static_cast<hipStream_t>(stream));
}

int xrs_reconst_one_shards(const xrs_codec* x, uint8_t* const* shards, size_t stripe_stride,
                           size_t size, size_t n_stripes, int k, void* stream) {
  if (!x) return XRS_ERR_INVALID_ARG;
  int e = check_size(size);
  if (e) return e;
  if (k < 0 || k >= x->d) return XRS_ERR_ILLEGAL_DATA_INDEX;
  if (n_stripes == 0 || size == 0) return XRS_OK;
  if (!shards) return XRS_ERR_INVALID_ARG;
  std::vector<int> a_need;
  int bi = 0;
  need_vects(x, k, &a_need, &bi);
  // Only the GetNeedVects set and vect k must be valid pointers.
  std::vector<uint64_t> t(x->d + x->p, 0);
  std::vector<int> used = {k, x->d, bi};
  for (int m = 0; m < x->d; ++m) used.push_back(m);
  for (int a : a_need) used.push_back(a);
  for (int i : used) {
    if (!shards[i]) return XRS_ERR_INVALID_ARG;
    t[i] = reinterpret_cast<uint64_t>(shards[i]);
  }
  if (x->device < 0) return XRS_ERR_NO_DEVICE;
  return reconst_one_impl(x, {nullptr, 0, stripe_stride, t.data()}, size, n_stripes, k,
                          static_cast<hipStream_t>(stream));
}

int xrs_reconst_shards(const xrs_codec* x, uint8_t* const* shards, size_t stripe_stride,
                       size_t size, size_t n_stripes, const int* dp_has, int n_has,
                       const int* need, int n_need, void* stream) {
  if (!x || n_has < 0 || n_need < 0 || (n_has && !dp_has) || (n_need && !need))
    return XRS_ERR_INVALID_ARG;
  if (n_need == 1 && need[0] < x->d)
    return xrs_reconst_one_shards(x, shards, stripe_stride, size, n_stripes, need[0], stream);
  int e = check_size(size);
  if (e) return e;
  if (!table_ok(shards, x->d + x->p)) return XRS_ERR_INVALID_ARG;
  if (x->device < 0) return XRS_ERR_NO_DEVICE;
  std::vector<uint64_t> t(x->d + x->p);
  for (int i = 0; i < x->d + x->p; ++i) t[i] = reinterpret_cast<uint64_t>(shards[i]);
  Written w;
  return reconst_impl(x, {nullptr, 0, stripe_stride, t.data()}, size, size ? n_stripes : 0,
                      dp_has, n_has, need, n_need, static_cast<hipStream_t>(stream), &w);
}

int xrs_enable_peer_access(int device, int peer) {
  int prev = -1, can = 0;
  if (hipDeviceCanAccessPeer(&can, device, peer) != hipSuccess || !can) return XRS_ERR_INVALID_ARG;
  (void)hipGetDevice(&prev);
  if (hipSetDevice(device) != hipSuccess) return XRS_ERR_HIP;
  hipError_t r = hipDeviceEnablePeerAccess(peer, 0);
  if (prev >= 0) (void)hipSetDevice(prev);
  if (r == hipErrorPeerAccessAlreadyEnabled) {
    (void)hipGetLastError();
    return XRS_OK;
  }
  return hip_err(r);
}

// ------------------------------------------------------ host-resident batches
}  // extern "C"

namespace {

// Host-resident batch in pinned, device-mapped memory that lies inside one
// allocation: the device address of host_base, else nullptr.  The kernels then
// run on it in place over PCIe (no DMA; measured 15-28% faster than the copy
// pipeline, profiles/r01_bench_host.log).  XRS_HOST_ZC=0 disables.
uint8_t* host_zero_copy(uint8_t* host_base, size_t extent) {
  const char* v = std::getenv("XRS_HOST_ZC");
  if (v && v[0] == '0') return nullptr;
  // A failed probe (pageable memory) leaves the runtime's last-error set;
  // clear it, or the next launch's hipGetLastError() reports it.
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, host_base, 0) != hipSuccess || !d) {
    (void)hipGetLastError();
    return nullptr;
  }
  hipDeviceptr_t base = nullptr;
  size_t len = 0;
  if (hipMemGetAddressRange(&base, &len, static_cast<hipDeviceptr_t>(d)) != hipSuccess || !base) {
    (void)hipGetLastError();
    return nullptr;
  }
  const uintptr_t lo = reinterpret_cast<uintptr_t>(base), p0 = reinterpret_cast<uintptr_t>(d);
  if (p0 < lo || p0 + extent > lo + len) return nullptr;
  return static_cast<uint8_t*>(d);
}

size_t batch_extent(const xrs_codec* x, size_t size, size_t shard_stride, size_t stripe_stride,
                    size_t n_stripes) {
  return (n_stripes - 1) * stripe_stride + static_cast<size_t>(x->d + x->p - 1) * shard_stride + size;
}

// Run one batched op on the sync stream and wait.
template <class F>
int run_in_place(const xrs_codec* x, F&& fn) {
  std::lock_guard<std::mutex> lk(x->mu);
  DeviceGuard g(x->device);
  int e = ensure_staging(x, 1);  // creates the stream
  if (!e) e = fn(x->stream);
  const int es = sync(x);
  return e ? e : es;
}

}  // namespace

namespace {
// Per-stripe calls on caller-registered memory (hostreg.h): when every vect
// a call touches lies in a range pinned and mapped by xrs_host_alloc /
// xrs_host_register, the call runs in place -- the kernels read and write the
// caller's buffers over PCIe through a per-vect pointer table (Layout::table),
// with no CPU gather into pinned staging and no scatter back.  dev[i] is vect
// i's device address for the listed vects (0 for the others).
// XRS_SYNC_REG=0 turns it off (A/B).
bool reg_vects(uint8_t* const* v, int n, const std::vector<int>& use, size_t size,
               std::vector<uint64_t>* dev) {
  static const bool off = [] {
    const char* e = std::getenv("XRS_SYNC_REG");
    return e && e[0] == '0';
  }();
  if (off) return false;
  dev->assign(n, 0);
  const xrs_detail::HostRangesView ranges;
  for (int i : use) {
    if (i < 0 || i >= n || !v[i]) return false;
    const uint64_t a = ranges.device(v[i], size);
    if (!a) return false;
    (*dev)[i] = a;
  }
  xrs::trace_event("host:sync_in_place");
  return true;
}

std::vector<int> iota_vects(int n) {
  std::vector<int> u(n);
  for (int i = 0; i < n; ++i) u[i] = i;
  return u;
}

// may_queue: a busy codec hands the call to its auto queue (the queue's own
// fallback for calls it cannot batch comes back here with false).
int reconst_sync(const xrs_codec* x, uint8_t* const* vects, int n, size_t size, const int* dp_has,
                 int n_has, const int* need, int n_need, bool may_queue) {
  if (!x || n_has < 0 || n_need < 0 || (n_has && !dp_has) || (n_need && !need))
    return XRS_ERR_INVALID_ARG;
  if (n_need == 1 && need[0] < x->d) return xrs_reconst_one(x, vects, n, size, need[0]);
  int e = check_size(size);
  if (e) return e;
  if (n != x->d + x->p) return XRS_ERR_ILLEGAL_VECTS;
  if (!vects_ok(vects, n)) return XRS_ERR_INVALID_ARG;
  std::unique_lock<std::mutex> lk(x->mu, std::try_to_lock);
  if (!lk.owns_lock()) {  // busy: concurrent callers share a queue's batches
    if (xrs_queue* q = may_queue && size ? auto_queue(x, size) : nullptr)
      return xrs_queue_reconst(q, vects, n, dp_has, n_has, need, n_need);
    lk.lock();
  }
  DeviceGuard g(x->device);
  std::vector<uint64_t> dv;
  if (size && reg_vects(vects, n, iota_vects(n), size, &dv)) {  // in place, registered memory
    if ((e = ensure_staging(x, 1))) return e;
    Written w;
    e = reconst_impl(x, {nullptr, 0, 0, dv.data()}, size, 1, dp_has, n_has, need, n_need, x->stream, &w);
    const int es = sync(x);
    return e ? e : es;
  }
  Stage st(x, static_cast<size_t>(n) * size, size);
  if ((e = st.init())) return e;
  for (int i = 0; i < n && !e; ++i) e = st.in(static_cast<size_t>(i) * size, vects[i], size);
  if (!e) e = st.upload();
  if (e) {
    (void)sync(x);
    return e;
  }
  Written w;
  const int er = reconst_impl(x, st.layout(size), size, size ? 1 : 0, dp_has, n_has, need, n_need,
                              x->stream, &w);
  // Copy back every half the device wrote, also when a later step failed
  // (the reference's Reconst is not atomic either).
  const size_t half = size / 2;
  for (auto& h : w.halves)
    st.out(vects[h.first] + h.second * half, static_cast<size_t>(h.first) * size + h.second * half,
           half);
  e = st.finish();
  return er ? er : e;
}
}  // namespace

namespace xrs_detail {
int reconst_direct(const xrs_codec* x, uint8_t* const* vects, int n, size_t size,
                   const int* dp_has, int n_has, const int* need, int n_need) {
  return reconst_sync(x, vects, n, size, dp_has, n_has, need, n_need, false);
}
}  // namespace xrs_detail

extern "C" {

int xrs_encode_host(const xrs_codec* x, uint8_t* host_base, size_t size, size_t shard_stride,
                    size_t stripe_stride, size_t n_stripes) {
  if (!x) return XRS_ERR_INVALID_ARG;
  int e = check_size(size);
  if (e) return e;
  if (n_stripes == 0 || size == 0) return XRS_OK;
  if (!host_base) return XRS_ERR_INVALID_ARG;
  if (x->device < 0) return XRS_ERR_NO_DEVICE;
  const int d = x->d, p = x->p;
  std::vector<std::pair<int, int>> in, out;
  for (int j = 0; j < d; ++j) in.push_back({j, 2});
  for (int r = 0; r < p; ++r) out.push_back({d + r, 2});
  if (uint8_t* zb = host_zero_copy(host_base, batch_extent(x, size, shard_stride, stripe_stride, n_stripes)))
    return run_in_place(x, [&](hipStream_t s) {
      return encode_impl(x, {zb, shard_stride, stripe_stride}, size, n_stripes, s);
    });
  std::vector<Image> ims = {batch_image(x, host_base, size, shard_stride, stripe_stride)};
  std::vector<uint64_t> tab;
  return run_pipeline(x, ims, n_stripes, halves(in, size), halves(out, size),
                      [&](uint8_t* slot, size_t n, hipStream_t s) {
    return encode_impl(x, image_layout(ims[0], slot, &tab), size, n, s);
  });
}

int xrs_reconst_one_host(const xrs_codec* x, uint8_t* host_base, size_t size, size_t shard_stride,
                         size_t stripe_stride, size_t n_stripes, int k) {
  if (!x) return XRS_ERR_INVALID_ARG;
  int e = check_size(size);
  if (e) return e;
  std::vector<int> a_need;
  int bi = 0;
  if ((e = need_vects(x, k, &a_need, &bi))) return e;
  if (n_stripes == 0 || size == 0) return XRS_OK;
  if (!host_base) return XRS_ERR_INVALID_ARG;
  if (x->device < 0) return XRS_ERR_NO_DEVICE;
  const int d = x->d;
  // Only the GetNeedVects set crosses PCIe (xrs.go:146-171).
  std::vector<std::pair<int, int>> in, out = {{k, 2}};
  for (int m = 0; m < d; ++m) in.push_back({m == k ? d : m, 1});
  in.push_back({bi, 1});
  for (int i : a_need) in.push_back({i, 0});
  if (uint8_t* zb = host_zero_copy(host_base, batch_extent(x, size, shard_stride, stripe_stride, n_stripes)))
    return run_in_place(x, [&](hipStream_t s) {
      return reconst_one_impl(x, {zb, shard_stride, stripe_stride}, size, n_stripes, k, s);
    });
  std::vector<Image> ims = {batch_image(x, host_base, size, shard_stride, stripe_stride)};
  std::vector<uint64_t> tab;
  return run_pipeline(x, ims, n_stripes, halves(in, size), halves(out, size),
                      [&](uint8_t* slot, size_t n, hipStream_t s) {
    return reconst_one_impl(x, image_layout(ims[0], slot, &tab), size, n, k, s);
  });
}

// xrs.go:236 Reconst(dpHas, need) of every stripe of a host-resident batch.
// For a clean call (indexes valid and distinct, need disjoint from dpHas)
// only the survivors go up and only the halves the reference writes come
// back (lost a-halves, retrieveRS b-halves of surviving piggybacked parity,
// needed b-halves); otherwise whole stripes go both ways, so the reference's
// toggling on repeated indexes is kept.  On an error part-way through a
// pageable batch, earlier chunks keep their results (the reference's Reconst
// is not atomic either).
int xrs_reconst_host(const xrs_codec* x, uint8_t* host_base, size_t size, size_t shard_stride,
                     size_t stripe_stride, size_t n_stripes, const int* dp_has, int n_has,
                     const int* need, int n_need) {
  if (!x || n_has < 0 || n_need < 0 || (n_has && !dp_has) || (n_need && !need))
    return XRS_ERR_INVALID_ARG;
  if (n_need == 1 && need[0] < x->d)  // xrs.go:238-240 (a negative k is rejected there)
    return xrs_reconst_one_host(x, host_base, size, shard_stride, stripe_stride, n_stripes,
                                need[0]);
  int e = check_size(size);
  if (e) return e;
  if (n_stripes == 0 || size == 0) return XRS_OK;
  if (!host_base) return XRS_ERR_INVALID_ARG;
  if (x->device < 0) return XRS_ERR_NO_DEVICE;
  const int d = x->d, m = x->d + x->p;
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
  std::vector<std::pair<int, int>> in, out;
  for (int i = 0; i < m; ++i) {
    if (!clean) {
      in.push_back({i, 2});
      out.push_back({i, 2});
    } else if (in_has[i]) {
      in.push_back({i, 2});
      if (i > d && !x->xs[i].empty()) out.push_back({i, 1});  // retrieveRS (xrs.go:305-320)
    } else {
      out.push_back({i, in_need[i] ? 2 : 0});
    }
  }
  Written w;
  if (uint8_t* zb = host_zero_copy(host_base, batch_extent(x, size, shard_stride, stripe_stride, n_stripes)))
    return run_in_place(x, [&](hipStream_t s) {
      return reconst_impl(x, {zb, shard_stride, stripe_stride}, size, n_stripes, dp_has, n_has,
                          need, n_need, s, &w);
    });
  std::vector<Image> ims = {batch_image(x, host_base, size, shard_stride, stripe_stride)};
  std::vector<uint64_t> tab;
  return run_pipeline(x, ims, n_stripes, halves(in, size), halves(out, size),
                      [&](uint8_t* slot, size_t n, hipStream_t s) {
    return reconst_impl(x, image_layout(ims[0], slot, &tab), size, n, dp_has, n_has, need, n_need,
                        s, &w);
  });
}

// xrs.go:324 Update(old, new, row, parity) of every stripe of a host batch:
// old/new rows at old_base / new_base + s * stride, parity shard r of stripe s
// at parity_base + s * parity_stripe_stride + r * parity_shard_stride.
int xrs_update_host(const xrs_codec* x, const uint8_t* old_base, size_t old_stripe_stride,
                    const uint8_t* new_base, size_t new_stripe_stride, size_t size, int row,
                    uint8_t* parity_base, size_t parity_shard_stride,
                    size_t parity_stripe_stride, size_t n_stripes) {
  if (!x) return XRS_ERR_INVALID_ARG;
  int e = check_size(size);
  if (e) return e;
  if (row < 0 || row >= x->d) return XRS_ERR_ILLEGAL_DATA_INDEX;
  if (n_stripes == 0 || size == 0) return XRS_OK;
  if (!old_base || !new_base || !parity_base) return XRS_ERR_INVALID_ARG;
  if (x->device < 0) return XRS_ERR_NO_DEVICE;
  const int p = x->p;
  const size_t last = n_stripes - 1;
  uint8_t* zo = host_zero_copy(const_cast<uint8_t*>(old_base), last * old_stripe_stride + size);
  uint8_t* zn = host_zero_copy(const_cast<uint8_t*>(new_base), last * new_stripe_stride + size);
  uint8_t* zp = host_zero_copy(parity_base, last * parity_stripe_stride +
                                                static_cast<size_t>(p - 1) * parity_shard_stride + size);
  if (zo && zn && zp)
    return run_in_place(x, [&](hipStream_t s) {
      return update_impl(x, {reinterpret_cast<uint64_t>(zo), old_stripe_stride},
                         {reinterpret_cast<uint64_t>(zn), new_stripe_stride}, size, row,
                         {zp, parity_shard_stride, parity_stripe_stride}, n_stripes, s);
    });
  // device images: the p parity rows, old, new (each its own host pitch)
  std::vector<Image> ims(3);
  for (int r = 0; r < p; ++r) ims[0].host0.push_back(parity_base + r * parity_shard_stride);
  ims[0].hp = parity_stripe_stride;
  ims[1].host0 = {const_cast<uint8_t*>(old_base)};
  ims[1].hp = old_stripe_stride;
  ims[2].host0 = {const_cast<uint8_t*>(new_base)};
  ims[2].hp = new_stripe_stride;
  for (Image& im : ims) im.len = size;
  std::vector<Piece> in, out;
  for (int r = 0; r < p; ++r) {
    in.push_back({0, r, 0, size});
    out.push_back({0, r, 0, size});
  }
  in.push_back({1, 0, 0, size});
  in.push_back({2, 0, 0, size});
  std::vector<uint64_t> tp, to, tn;
  return run_pipeline(x, ims, n_stripes, in, out, [&](uint8_t* slot, size_t n, hipStream_t s) {
    const Layout o = image_layout(ims[1], slot, &to), nw = image_layout(ims[2], slot, &tn);
    return update_impl(x, o.row(0, 0), nw.row(0, 0), size, row, image_layout(ims[0], slot, &tp), n, s);
  });
}

// xrs.go:363 Replace(data, rows, parity) of every stripe of a host batch:
// data i of stripe s at data_base + s * data_stripe_stride + i * data_shard_stride.
int xrs_replace_host(const xrs_codec* x, const uint8_t* data_base, size_t data_shard_stride,
                     size_t data_stripe_stride, const int* rows, int n, size_t size,
                     uint8_t* parity_base, size_t parity_shard_stride,
                     size_t parity_stripe_stride, size_t n_stripes) {
  if (!x) return XRS_ERR_INVALID_ARG;
  int e = check_replace(x, rows, n, size);
  if (e) return e;
  if (n_stripes == 0 || size == 0) return XRS_OK;
  if (!data_base || !parity_base) return XRS_ERR_INVALID_ARG;
  if (x->device < 0) return XRS_ERR_NO_DEVICE;
  const int p = x->p;
  const size_t last = n_stripes - 1;
  uint8_t* zd = host_zero_copy(const_cast<uint8_t*>(data_base),
                               last * data_stripe_stride + static_cast<size_t>(n - 1) * data_shard_stride + size);
  uint8_t* zp = host_zero_copy(parity_base, last * parity_stripe_stride +
                                                static_cast<size_t>(p - 1) * parity_shard_stride + size);
  if (zd && zp)
    return run_in_place(x, [&](hipStream_t s) {
      return replace_impl(x, {zd, data_shard_stride, data_stripe_stride}, rows, n, size,
                          {zp, parity_shard_stride, parity_stripe_stride}, n_stripes, s);
    });
  // device images: the p parity rows, the n data rows
  std::vector<Image> ims(2);
  for (int r = 0; r < p; ++r) ims[0].host0.push_back(parity_base + r * parity_shard_stride);
  ims[0].hp = parity_stripe_stride;
  for (int i = 0; i < n; ++i)
    ims[1].host0.push_back(const_cast<uint8_t*>(data_base) + i * data_shard_stride);
  ims[1].hp = data_stripe_stride;
  for (Image& im : ims) im.len = size;
  std::vector<Piece> in, out;
  for (int r = 0; r < p; ++r) {
    in.push_back({0, r, 0, size});
    out.push_back({0, r, 0, size});
  }
  for (int i = 0; i < n; ++i) in.push_back({1, i, 0, size});
  std::vector<uint64_t> tp, td;
  return run_pipeline(x, ims, n_stripes, in, out, [&](uint8_t* slot, size_t ns, hipStream_t s) {
    return replace_impl(x, image_layout(ims[1], slot, &td), rows, n, size,
                        image_layout(ims[0], slot, &tp), ns, s);
  });
}

void* xrs_host_alloc(size_t bytes) {
  void* p = nullptr;
  // Portable: pinned and mapped for every GPU, so one allocation can feed a
  // group of devices (group.cpp).
  if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocMapped | hipHostMallocPortable) != hipSuccess)
    return nullptr;
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, p, 0) == hipSuccess) xrs_detail::host_ranges_add(p, bytes ? bytes : 1, d);
  else (void)hipGetLastError();
  return p;
}
void* xrs_host_device_pointer(void* host) {
  void* d = nullptr;
  if (!host) return nullptr;
  if (hipHostGetDevicePointer(&d, host, 0) != hipSuccess) {
    (void)hipGetLastError();  // not mapped: do not leave the error for the next launch
    return nullptr;
  }
  return d;
}
void xrs_host_free(void* p) {
  if (!p) return;
  xrs_detail::host_ranges_remove(p);
  (void)hipHostFree(p);
}
int xrs_host_register(void* p, size_t bytes) {
  if (!p || !bytes) return XRS_ERR_INVALID_ARG;
  const int e = hip_err(hipHostRegister(p, bytes, hipHostRegisterMapped | hipHostRegisterPortable));
  if (e) return e;
  // the per-stripe calls find the range here without a HIP call (hostreg.h)
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, p, 0) == hipSuccess) xrs_detail::host_ranges_add(p, bytes, d);
  else (void)hipGetLastError();
  return XRS_OK;
}
int xrs_host_unregister(void* p) {
  if (!p) return XRS_ERR_INVALID_ARG;
  xrs_detail::host_ranges_remove(p);
  return hip_err(hipHostUnregister(p));
}

// ------------------------------------------------------------------- sync
// xrs.go:103-128
int xrs_encode(const xrs_codec* x, uint8_t* const* vects, int n, size_t size) {
  if (!x) return XRS_ERR_INVALID_ARG;
  if (n < 1) return XRS_ERR_ILLEGAL_VECTS;
  int e = check_size(size);
  if (e) return e;
  if (n != x->d + x->p) return XRS_ERR_ILLEGAL_VECTS;
  if (!vects_ok(vects, n)) return XRS_ERR_INVALID_ARG;
  if (size == 0) return XRS_OK;
  std::unique_lock<std::mutex> lk(x->mu, std::try_to_lock);
  if (!lk.owns_lock()) {  // busy: concurrent callers share a queue's batches
    if (xrs_queue* q = auto_queue(x, size)) return xrs_queue_encode(q, vects, n);
    lk.lock();
  }
  DeviceGuard g(x->device);
  std::vector<uint64_t> dv;
  if (reg_vects(vects, n, iota_vects(n), size, &dv)) {  // in place, registered memory
    if ((e = ensure_staging(x, 1))) return e;
    e = encode_impl(x, {nullptr, 0, 0, dv.data()}, size, 1, x->stream);
    const int es = sync(x);
    return e ? e : es;
  }
  Stage st(x, static_cast<size_t>(n) * size, size);
  if ((e = st.init())) return e;
  for (int j = 0; j < x->d && !e; ++j) e = st.in(static_cast<size_t>(j) * size, vects[j], size);
  if (!e) e = st.upload();
  if (!e) e = encode_impl(x, st.layout(size), size, 1, x->stream);
  if (!e)
    for (int r = 0; r < x->p; ++r)
      st.out(vects[x->d + r], static_cast<size_t>(x->d + r) * size, size);
  const int es = st.finish();
  return e ? e : es;
}

// xrs.go:175-221: only the GetNeedVects set travels to the device.
int xrs_reconst_one(const xrs_codec* x, uint8_t* const* vects, int n, size_t size, int k) {
  if (!x) return XRS_ERR_INVALID_ARG;
  int e = check_size(size);
  if (e) return e;
  std::vector<int> a_need;
  int bi = 0;
  if ((e = need_vects(x, k, &a_need, &bi))) return e;
  if (n != x->d + x->p) return XRS_ERR_ILLEGAL_VECTS;
  if (!vects) return XRS_ERR_INVALID_ARG;
  if (size == 0) return XRS_OK;
  const int d = x->d;
  const size_t half = size / 2;
  std::vector<std::pair<int, int>> reads;  // (shard, half)
  for (int m = 0; m < d; ++m) reads.push_back({m == k ? d : m, 1});
  reads.push_back({bi, 1});
  for (int i : a_need) reads.push_back({i, 0});
  for (auto& r : reads)
    if (!vects[r.first]) return XRS_ERR_INVALID_ARG;
  if (!vects[k]) return XRS_ERR_INVALID_ARG;
  std::unique_lock<std::mutex> lk(x->mu, std::try_to_lock);
  if (!lk.owns_lock()) {  // busy: concurrent callers share a queue's batches
    // (the queue takes every vect; vects outside the need set may be null here)
    xrs_queue* q = vects_ok(vects, n) ? auto_queue(x, size) : nullptr;
    if (q) return xrs_queue_reconst_one(q, vects, n, k);
    lk.lock();
  }
  DeviceGuard g(x->device);
  std::vector<int> use = {k};
  for (auto& r : reads) use.push_back(r.first);
  std::vector<uint64_t> dv;
  if (reg_vects(vects, n, use, size, &dv)) {  // in place, registered memory
    if ((e = ensure_staging(x, 1))) return e;
    e = reconst_one_impl(x, {nullptr, 0, 0, dv.data()}, size, 1, k, x->stream);
    const int es = sync(x);
    return e ? e : es;
  }
  Stage st(x, static_cast<size_t>(n) * size, size);
  if ((e = st.init())) return e;
  for (size_t i = 0; i < reads.size() && !e; ++i) {
    const size_t off = static_cast<size_t>(reads[i].first) * size + reads[i].second * half;
    e = st.in(off, vects[reads[i].first] + reads[i].second * half, half);
  }
  if (!e) e = st.upload();
  if (!e) e = reconst_one_impl(x, st.layout(size), size, 1, k, x->stream);
  if (!e) st.out(vects[k], static_cast<size_t>(k) * size, size);
  const int es = st.finish();
  return e ? e : es;
}

// xrs.go:236-301
int xrs_reconst(const xrs_codec* x, uint8_t* const* vects, int n, size_t size, const int* dp_has,
                int n_has, const int* need, int n_need) {
  return reconst_sync(x, vects, n, size, dp_has, n_has, need, n_need, true);
}

// xrs.go:324-346
int xrs_update(const xrs_codec* x, const uint8_t* old_data, const uint8_t* new_data, size_t size,
               int row, uint8_t* const* parity, int n_parity) {
  if (!x) return XRS_ERR_INVALID_ARG;
  int e = check_size(size);
  if (e) return e;
  if (row < 0 || row >= x->d) return XRS_ERR_ILLEGAL_DATA_INDEX;
  if (n_parity != x->p) return XRS_ERR_ILLEGAL_VECTS;
  if (!old_data || !new_data || !vects_ok(parity, n_parity)) return XRS_ERR_INVALID_ARG;
  if (size == 0) return XRS_OK;
  const int p = x->p;
  std::unique_lock<std::mutex> lk(x->mu, std::try_to_lock);
  if (!lk.owns_lock()) {  // busy: concurrent callers share a queue's batches
    if (xrs_queue* q = auto_queue(x, size))
      return xrs_queue_update(q, old_data, new_data, row, parity, n_parity);
    lk.lock();
  }
  DeviceGuard g(x->device);
  {  // in place, registered memory: rows [0, p) parity, p old, p+1 new
    std::vector<uint8_t*> v(parity, parity + p);
    v.push_back(const_cast<uint8_t*>(old_data));
    v.push_back(const_cast<uint8_t*>(new_data));
    std::vector<uint64_t> dv;
    if (reg_vects(v.data(), p + 2, iota_vects(p + 2), size, &dv)) {
      if ((e = ensure_staging(x, 1))) return e;
      e = update_impl(x, {dv[p], 0}, {dv[p + 1], 0}, size, row, {nullptr, 0, 0, dv.data()}, 1,
                      x->stream);
      const int es = sync(x);
      return e ? e : es;
    }
  }
  // staging rows: [0, p) parity, p old, p+1 new
  const size_t stride = static_cast<size_t>(p + 2) * size;
  Stage st(x, stride, size);
  if ((e = st.init())) return e;
  for (int r = 0; r < p && !e; ++r) e = st.in(static_cast<size_t>(r) * size, parity[r], size);
  if (!e) e = st.in(static_cast<size_t>(p) * size, old_data, size);
  if (!e) e = st.in(static_cast<size_t>(p + 1) * size, new_data, size);
  if (!e) e = st.upload();
  const Layout P = st.layout(size);
  if (!e) e = update_impl(x, P.row(p, 0), P.row(p + 1, 0), size, row, P, 1, x->stream);
  if (!e)
    for (int r = 0; r < p; ++r) st.out(parity[r], static_cast<size_t>(r) * size, size);
  const int es = st.finish();
  return e ? e : es;
}

// xrs.go:363-387
int xrs_replace(const xrs_codec* x, uint8_t* const* data, const int* rows, int n, size_t size,
                uint8_t* const* parity, int n_parity) {
  if (!x) return XRS_ERR_INVALID_ARG;
  int e = check_replace(x, rows, n, size);
  if (e) return e;
  if (n_parity != x->p) return XRS_ERR_ILLEGAL_VECTS;
  if (!vects_ok(data, n) || !vects_ok(parity, n_parity)) return XRS_ERR_INVALID_ARG;
  if (size == 0) return XRS_OK;
  const int p = x->p;
  std::unique_lock<std::mutex> lk(x->mu, std::try_to_lock);
  if (!lk.owns_lock()) {  // busy: concurrent callers share a queue's batches
    if (xrs_queue* q = auto_queue(x, size))
      return xrs_queue_replace(q, data, rows, n, parity, n_parity);
    lk.lock();
  }
  DeviceGuard g(x->device);
  {  // in place, registered memory: rows [0, p) parity, [p, p+n) data
    std::vector<uint8_t*> v(parity, parity + p);
    v.insert(v.end(), data, data + n);
    std::vector<uint64_t> dv;
    if (reg_vects(v.data(), p + n, iota_vects(p + n), size, &dv)) {
      if ((e = ensure_staging(x, 1))) return e;
      e = replace_impl(x, {nullptr, 0, 0, dv.data() + p}, rows, n, size, {nullptr, 0, 0, dv.data()}, 1,
                       x->stream);
      const int es = sync(x);
      return e ? e : es;
    }
  }
  // staging rows: [0, p) parity, [p, p+n) data
  const size_t stride = static_cast<size_t>(p + n) * size;
  Stage st(x, stride, size);
  if ((e = st.init())) return e;
  for (int r = 0; r < p && !e; ++r) e = st.in(static_cast<size_t>(r) * size, parity[r], size);
  for (int i = 0; i < n && !e; ++i) e = st.in(static_cast<size_t>(p + i) * size, data[i], size);
  if (!e) e = st.upload();
  const Layout P = st.layout(size);
  const Layout D = st.layout(size, static_cast<size_t>(p) * size);
  if (!e) e = replace_impl(x, D, rows, n, size, P, 1, x->stream);
  if (!e)
    for (int r = 0; r < p; ++r) st.out(parity[r], static_cast<size_t>(r) * size, size);
  const int es = st.finish();
  return e ? e : es;
}

}  // extern "C"
