// kbody_rows.h -- the rows kernel's body (kernels.hip), included inside the
// kernel functions: XRS_IND 0 with XRS_ROW(row, stripe, off) naming the row
// addressing (rows_kernel), XRS_IND 1 for table rows (rows_ind_kernel, runtime
// counts, always grouped).  Not a header.
  constexpr int W = VEC ? 4 : 1;
  const uint64_t gid = logical_block(a.order) * BS + threadIdx.x;
  if (gid >= a.total) return;
  const uint64_t stripe = gid / a.chunks;
  uint64_t off = a.off0 + (gid - stripe * a.chunks) * (4 * W);
  if (VEC && off > a.last) off = a.last;  // ragged end: overlapping last chunk
  const int nb = VEC ? 16 : static_cast<int>(a.len - off < 4 ? a.len - off : 4);

#if XRS_IND
  // Table rows: every base address read up front, in one round trip (see
  // kbody_pair.h).
  uint64_t db[R], mb[kMaxSrc], xb[kMaxXor];
#pragma unroll
  for (int r = 0; r < R; ++r) db[r] = row_base_ind(a.dst[r], stripe);
#pragma unroll
  for (int m = 0; m < kMaxSrc; ++m)
    if (m < a.nm) mb[m] = row_base_ind(a.msrc[m], stripe);
#pragma unroll
  for (int x = 0; x < kMaxXor; ++x)
    if (x < a.nx) xb[x] = row_base_ind(a.xsrc[x], stripe);
#define XRS_DST(r) (db[r] + off)
#define XRS_MSRC(m) (mb[m] + off)
#define XRS_XSRC(x) (xb[x] + off)
#else
#define XRS_DST(r) XRS_ROW(a.dst[r], stripe, off)
#define XRS_MSRC(m) XRS_ROW(a.msrc[m], stripe, off)
#define XRS_XSRC(x) XRS_ROW(a.xsrc[x], stripe, off)
#endif
  uint32_t acc[R][W];
  if constexpr (ACC) {
#pragma unroll
    for (int r = 0; r < R; ++r) ld<VEC>(acc[r], XRS_DST(r), nb);
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int w = 0; w < W; ++w) acc[r][w] = 0u;
  }

  if constexpr (NM != kDyn && NX != kDyn) {
    uint32_t xm[NM > 0 ? NM : 1][W], xx[NX > 0 ? NX : 1][W];
    // Raised priority while this wave issues its loads, so fresh waves get
    // their requests out ahead of waves that are computing (measured +1.7%
    // on ReconstOne 1 MiB; tools/kbench.hip "rw prio").
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int m = 0; m < NM; ++m) ld<VEC>(xm[m], XRS_MSRC(m), nb);
#pragma unroll
    for (int x = 0; x < NX; ++x) ld<VEC>(xx[x], XRS_XSRC(x), nb);
    __builtin_amdgcn_s_setprio(0);
#pragma unroll
    for (int m = 0; m + 1 < NM; m += 2) rows_mac2<R, W>(acc, a.tab[m], a.tab[m + 1], xm[m], xm[m + 1]);
    if constexpr (NM & 1) rows_mac1<R, W>(acc, a.tab[NM - 1], xm[NM - 1]);
#pragma unroll
    for (int x = 0; x < NX; ++x) rows_xor<R, W>(acc, a.xmask[x], xx[x]);
  } else if (XRS_IND || a.grouped) {
    // Runtime counts, small grid (latency-bound): groups of kGrp rows, each
    // group's loads issued together, so a launch pays ceil(rows / kGrp)
    // memory round trips instead of one per row.
    constexpr int kGrp = 8;
#if XRS_IND
#pragma unroll
    for (int m0 = 0; m0 < kMaxSrc; m0 += kGrp) {  // unrolled: mb[] indexes static
      if (m0 >= a.nm) break;
#else
    for (int m0 = 0; m0 < a.nm; m0 += kGrp) {
#endif
      uint32_t v[kGrp][W];
#pragma unroll
      for (int g = 0; g < kGrp; ++g)
        if (m0 + g < a.nm) ld<VEC>(v[g], XRS_MSRC(m0 + g), nb);
#pragma unroll
      for (int g = 0; g < kGrp; ++g)
        if (m0 + g < a.nm) rows_mac1<R, W>(acc, a.tab[m0 + g], v[g]);
    }
#if XRS_IND
#pragma unroll
    for (int x0 = 0; x0 < kMaxXor; x0 += kGrp) {
      if (x0 >= a.nx) break;
#else
    for (int x0 = 0; x0 < a.nx; x0 += kGrp) {
#endif
      uint32_t v[kGrp][W];
#pragma unroll
      for (int g = 0; g < kGrp; ++g)
        if (x0 + g < a.nx) ld<VEC>(v[g], XRS_XSRC(x0 + g), nb);
#pragma unroll
      for (int g = 0; g < kGrp; ++g)
        if (x0 + g < a.nx) rows_xor<R, W>(acc, a.xmask[x0 + g], v[g]);
    }
  } else {
#if !XRS_IND
    // Runtime counts, large grid: one row at a time (measured: grouping 8
    // loads per wave cost 0-2% at 4 KiB and 2-7% at 1 MiB over seven (d, p)
    // in the XCD order; profiles/r01_others_rows_grouped{0,1}.log).
    for (int m = 0; m < a.nm; ++m) {
      uint32_t v[W];
      ld<VEC>(v, XRS_MSRC(m), nb);
      rows_mac1<R, W>(acc, a.tab[m], v);
    }
    for (int x = 0; x < a.nx; ++x) {
      uint32_t v[W];
      ld<VEC>(v, XRS_XSRC(x), nb);
      rows_xor<R, W>(acc, a.xmask[x], v);
    }
#endif
  }

#pragma unroll
  for (int r = 0; r < R; ++r) st<VEC>(acc[r], XRS_DST(r), nb);
#undef XRS_DST
#undef XRS_MSRC
#undef XRS_XSRC
