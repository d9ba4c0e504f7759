// xrs_plan.h -- launch plans shared by the host planner (codec.cpp) and the
// gfx950 kernels (kernels.hip).  Internal; not part of the C ABI.
//
// Four kernel shapes cover the whole xrs.go API surface: "pair" and "rows"
// below, the one-pass general Reconst ("staged", StagedPlan) and Update
// ("update_rows", UpdRowsPlan).
//
//  * "pair" kernel  (Encode xrs.go:103, Replace :363):
//      for every byte offset o of the a-half (H = size/2):
//        dst_r[o]   (^)= sum_c coef[c][r] * src_c[o]
//        dst_r[H+o] (^)= sum_c coef[c][r] * src_c[H+o]  ^  XOR_{c: pb[c]==r} src_c[o]
//    i.e. the RS matrix on both halves plus the piggyback XOR (xrs.go:118-126)
//    in ONE pass over HBM (the reference makes two).
//
//  * "rows" kernel  (ReconstOne xrs.go:175, the 4 steps of Reconst :236,
//    retrieveRS :305):
//      dst_r[o] (^)= sum_{m<NM} coef[m][r] * msrc_m[o]  ^  XOR_{x: xmask[x]>>r&1} xsrc_x[o]
//    over arbitrary half-rows (a row = one half of one shard).
//
// A row is addressed as ptr + stripe * stripe_stride (+ o); ptr is a device
// address.  GF(2^8) multiply by a constant c is done with three v_perm_b32
// byte lookups (see GfTab) so every coefficient is a 20-byte table.
#pragma once
#include <stdint.h>

namespace xrs {

// Per-coefficient byte-permute tables.  For x = b7..b0:
//   c*x = T0[x & 7] ^ T1[(x >> 3) & 7] ^ T2[x >> 6]
// T0/T1 have 8 one-byte entries (two dwords: lo = entries 0..3, hi = 4..7),
// T2 has 4 (one dword).  v_perm_b32 looks up 4 bytes at once.
struct GfTab {
  uint32_t lo0, hi0, lo1, hi1, top;
};

struct RowRef {
  uint64_t ptr;            // device address of this row in stripe 0
  uint64_t stripe_stride;  // bytes between consecutive stripes
};
// An indirect row (stripe_stride has this bit): ptr is the device-readable
// address of stripe 0's entry in a table of row addresses, and stripe s's row
// starts at the address stored at ptr + s * (stripe_stride & ~kRowInd).  The
// batching queue addresses its callers' own (registered) buffers this way.
constexpr uint64_t kRowInd = uint64_t(1) << 63;

constexpr int kMaxOut = 4;   // outputs per launch (parity rows / rebuilt rows)
constexpr int kMaxSrc = 24;  // GF sources per launch (more: chained ACC launches)
constexpr int kMaxXor = 24;  // XOR-only sources per launch (rows kernel)

struct PairPlan {
  int P;             // outputs (<= kMaxOut)
  int C;             // sources (<= kMaxSrc)
  bool acc;          // true: XOR into existing dst (Replace/Update, chained chunks)
  GfTab tab[kMaxSrc][kMaxOut];
  RowRef src[kMaxSrc];
  RowRef dst[kMaxOut];
  int8_t pb[kMaxSrc];  // piggyback target output of source c's a-half, or -1
  bool encode_xs;      // whole Encode in one launch: source c = data c, and c's
                       // a-half rides on output 1 + c % (P-1) (the XORSet)
  uint64_t half;       // H = size/2 bytes
  uint64_t n_stripes;
  uint64_t off0, end;  // byte range [off0, end) of each half (set by launch_pair)
  bool overlap;        // set by launch_pair: ragged end as one overlapping 16-B chunk
};

struct RowsPlan {
  int R;   // outputs (<= kMaxOut)
  int NM;  // GF sources (<= kMaxSrc)
  int NX;  // XOR sources (<= kMaxXor)
  bool acc;
  GfTab tab[kMaxSrc][kMaxOut];
  RowRef msrc[kMaxSrc];
  RowRef xsrc[kMaxXor];
  uint32_t xmask[kMaxXor];  // bit r set: XOR xsrc into output r
  RowRef dst[kMaxOut];
  uint64_t len;  // bytes per row
  uint64_t n_stripes;
  uint64_t off0, end;  // byte range [off0, end) of each row (set by launch_rows)
  bool overlap;        // set by launch_rows: ragged end as one overlapping 16-B chunk
};

// "staged" kernel: the general Reconst (xrs.go:236-301) in one pass, each of
// the reference's four steps kept as a stage in registers:
//   1. al_q = sum_{m<nd} acoef[m][q] * a(asrc_m)          -> adst_q   (lost a-halves)
//   2. b(bsrc_m) ^= abar(bret[m]), stored if bstore bit m  (retrieveRS)
//   3. out_u = sum_{m<nd} bcoef[m][u] * b(bsrc_m)  ^  abar(nmask[u]) -> bdst_u
// where abar(mask) XORs a-rows (bit m < kStSrc: a(asrc_m)) and rebuilt lost
// a-halves (bit kStSrc + q: al_q).  asrc/bsrc[0..nd) are the d survivors used
// by the RS inverse; entries past nd are extra survivors read only for XORs.
constexpr int kStSrc = 16;
constexpr int kStOut = 4;
// b-rows: the d survivors plus surviving piggybacked parity past dpHas[:d]
// (16+4: up to 19).  More than kStSrc only on the wave-specialised kernel
// (launch_staged declines otherwise and the caller runs the step plan).
constexpr int kStB = 20;

struct StagedPlan {
  int nd;      // GF sources (d)
  int na, nb;  // a-/b-half rows read (nd + extras), <= kStSrc / kStB
  int nl, nn;  // lost a-halves / needed b-halves written, <= kStOut
  RowRef asrc[kStSrc], bsrc[kStB];
  RowRef adst[kStOut], bdst[kStOut];
  uint8_t acoef[kStSrc][kStOut], bcoef[kStSrc][kStOut];
  uint32_t bret[kStB];     // abar mask XORed into b row m (0: none)
  uint32_t bstore;         // bit m: write b row m back
  uint32_t nmask[kStOut];  // abar mask XORed into output u
  uint64_t half;
  uint64_t n_stripes;
  uint64_t off0, end;  // byte range [off0, end) of each half (set by launch_staged)
  bool overlap;        // unused (in-place writes: the ragged end is its own launch)
};

// "update_rows" kernel: Update (xrs.go:324) where every stripe names its own
// data row (a batch of small writes to different shards):
//   r = rows[s] - row0 (stripes with r outside [0, nrows) are skipped),
//   delta = old ^ new,
//   dst_q[o]   ^= tab[r][q] * delta[o]
//   dst_q[H+o] ^= tab[r][q] * delta[H+o]  ^  (pbq[r] == q ? delta[o] : 0)
struct UpdRowsPlan {
  int P;      // outputs (<= kMaxOut)
  int nrows;  // data rows covered by this launch (<= kMaxSrc), starting at row0
  int row0;
  GfTab tab[kMaxSrc][kMaxOut];
  int8_t pbq[kMaxSrc];  // output whose b-half takes row r's delta a-half, or -1
  RowRef old_row, new_row;
  RowRef dst[kMaxOut];
  uint64_t rows;  // device-readable address of n_stripes int32 data rows;
                  // 0: every stripe uses row0 (nrows == 1)
  uint64_t half;
  uint64_t n_stripes;
  uint64_t off0, end;  // byte range [off0, end) of each half (set by launch_update_rows)
  bool overlap;        // unused (accumulates: the ragged end is its own launch)
};

// Kernel launchers (kernels.hip).  Return a hipError_t value as int.
int launch_pair(const PairPlan& plan, void* stream);
int launch_rows(const RowsPlan& plan, void* stream);
// kStagedDecline: the plan has more than kStSrc b-rows and cannot run as one
// 16-byte wave-specialised launch (a ragged end, more than kStOut retrieveRS
// rows); nothing was launched.
constexpr int kStagedDecline = -1;
int launch_staged(const StagedPlan& plan, void* stream);
int launch_update_rows(const UpdRowsPlan& plan, void* stream);
// Launch trace (diagnostics): record every kernel instantiation launched from
// here on (on: clears the record); traced_kernels writes "name count" lines.
void trace_kernels(bool on);
size_t traced_kernels(char* buf, size_t cap);
// Records a host-path event under `name` (e.g. "host:sync_in_place") in the
// same trace, when tracing is on.
void trace_event(const char* name);
// Device address of the zero rows that pad an Encode to a compile-time
// source count on device `dev` (allocated and zeroed on first call for that
// device, never freed: a launch in flight may read it), or 0.  xrs_new calls
// it for the codec's device, so a launch there never allocates; a launch on
// another device's stream makes that device's rows on first use.
uint64_t zero_rows(int dev);
// Makes device `dev`'s ring of tile-counter slots for the persistent staged
// kernel (kernels.hip ctr_ring: on first call for that device, never freed);
// false if it cannot be made (the one-shot kernels run instead).  xrs_new
// calls it for the codec's device; a launch on another device's stream makes
// that device's ring on first use.
bool tile_counters(int dev);

}  // namespace xrs
