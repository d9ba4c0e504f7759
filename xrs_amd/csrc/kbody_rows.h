// kbody_rows.h -- the rows kernel's body (kernels.hip), included inside the
// kernel functions with XRS_ROW(row, stripe, off) naming the row addressing:
// row_addr for rows_kernel, row_addr_ind for rows_ind_kernel.  Not a header.
  constexpr int W = VEC ? 4 : 1;
  const uint64_t gid = logical_block(a.order) * BS + threadIdx.x;
  if (gid >= a.total) return;
  const uint64_t stripe = gid / a.chunks;
  uint64_t off = a.off0 + (gid - stripe * a.chunks) * (4 * W);
  if (VEC && off > a.last) off = a.last;  // ragged end: overlapping last chunk
  const int nb = VEC ? 16 : static_cast<int>(a.len - off < 4 ? a.len - off : 4);

  uint32_t acc[R][W];
  if constexpr (ACC) {
#pragma unroll
    for (int r = 0; r < R; ++r) ld<VEC>(acc[r], XRS_ROW(a.dst[r], stripe, off), nb);
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
    for (int m = 0; m < NM; ++m) ld<VEC>(xm[m], XRS_ROW(a.msrc[m], stripe, off), nb);
#pragma unroll
    for (int x = 0; x < NX; ++x) ld<VEC>(xx[x], XRS_ROW(a.xsrc[x], stripe, off), nb);
    __builtin_amdgcn_s_setprio(0);
#pragma unroll
    for (int m = 0; m + 1 < NM; m += 2) rows_mac2<R, W>(acc, a.tab[m], a.tab[m + 1], xm[m], xm[m + 1]);
    if constexpr (NM & 1) rows_mac1<R, W>(acc, a.tab[NM - 1], xm[NM - 1]);
#pragma unroll
    for (int x = 0; x < NX; ++x) rows_xor<R, W>(acc, a.xmask[x], xx[x]);
  } else if (a.grouped) {
    // Runtime counts, small grid (latency-bound): groups of kGrp rows, each
    // group's loads issued together, so a launch pays ceil(rows / kGrp)
    // memory round trips instead of one per row.
    constexpr int kGrp = 8;
    for (int m0 = 0; m0 < a.nm; m0 += kGrp) {
      uint32_t v[kGrp][W];
#pragma unroll
      for (int g = 0; g < kGrp; ++g)
        if (m0 + g < a.nm) ld<VEC>(v[g], XRS_ROW(a.msrc[m0 + g], stripe, off), nb);
#pragma unroll
      for (int g = 0; g < kGrp; ++g)
        if (m0 + g < a.nm) rows_mac1<R, W>(acc, a.tab[m0 + g], v[g]);
    }
    for (int x0 = 0; x0 < a.nx; x0 += kGrp) {
      uint32_t v[kGrp][W];
#pragma unroll
      for (int g = 0; g < kGrp; ++g)
        if (x0 + g < a.nx) ld<VEC>(v[g], XRS_ROW(a.xsrc[x0 + g], stripe, off), nb);
#pragma unroll
      for (int g = 0; g < kGrp; ++g)
        if (x0 + g < a.nx) rows_xor<R, W>(acc, a.xmask[x0 + g], v[g]);
    }
  } else {
    // Runtime counts, large grid: one row at a time (measured: grouping 8
    // loads per wave cost 0-2% at 4 KiB and 2-7% at 1 MiB over seven (d, p)
    // in the XCD order; profiles/r01_others_rows_grouped{0,1}.log).
    for (int m = 0; m < a.nm; ++m) {
      uint32_t v[W];
      ld<VEC>(v, XRS_ROW(a.msrc[m], stripe, off), nb);
      rows_mac1<R, W>(acc, a.tab[m], v);
    }
    for (int x = 0; x < a.nx; ++x) {
      uint32_t v[W];
      ld<VEC>(v, XRS_ROW(a.xsrc[x], stripe, off), nb);
      rows_xor<R, W>(acc, a.xmask[x], v);
    }
  }

#pragma unroll
  for (int r = 0; r < R; ++r) st<VEC>(acc[r], XRS_ROW(a.dst[r], stripe, off), nb);
