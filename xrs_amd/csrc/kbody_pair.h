// kbody_pair.h -- the pair kernel's body (kernels.hip), included inside the
// kernel functions: XRS_IND 0 with XRS_ROW(row, stripe, off) naming the row
// addressing (pair_kernel), XRS_IND 1 for table rows (pair_ind_kernel, runtime
// source count only).  Not a header.
  constexpr int W = VEC ? 4 : 1;
  const uint64_t gid = (PLAIN ? uint64_t(blockIdx.x) : logical_block(a.order)) * BS + threadIdx.x;
  if (gid >= a.total) return;
  const uint64_t stripe = gid / a.chunks;
  uint64_t off = a.off0 + (gid - stripe * a.chunks) * (4 * W);
  if (VEC && off > a.last) off = a.last;  // ragged end: overlapping last chunk
  const int nb = VEC ? 16 : static_cast<int>(a.half - off < 4 ? a.half - off : 4);

#if XRS_IND
  // Table rows: every row's base address read up front, in one round trip.
  // vmcnt retires in order, so a table read issued after a row's data loads
  // would also wait for them: one round trip per row (measured 2x per batch).
  uint64_t db[P], sb[kMaxSrc];
#pragma unroll
  for (int r = 0; r < P; ++r) db[r] = row_base_ind(a.dst[r], stripe);
#pragma unroll
  for (int c = 0; c < kMaxSrc; ++c)
    if (c < a.n_src) sb[c] = row_base_ind(a.src[c], stripe);
#define XRS_DST(r) (db[r] + off)
#define XRS_SRC(c) (sb[c] + off)
#else
#define XRS_DST(r) XRS_ROW(a.dst[r], stripe, off)
#define XRS_SRC(c) XRS_ROW(a.src[c], stripe, off)
#endif
  uint32_t acc_a[P][W], acc_b[P][W];
  if constexpr (ACC) {
#pragma unroll
    for (int r = 0; r < P; ++r) {
      const uint64_t d = XRS_DST(r);
      ld<VEC>(acc_a[r], d, nb);
      ld<VEC>(acc_b[r], d + a.half, nb);
    }
  } else {
#pragma unroll
    for (int r = 0; r < P; ++r)
#pragma unroll
      for (int w = 0; w < W; ++w) acc_a[r][w] = acc_b[r][w] = 0u;
  }

  if constexpr (C != kDyn) {
    // Compile-time source count: every load issued up front.
    uint32_t xa[C][W], xb[C][W];
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const uint64_t s = XRS_SRC(c);
      ld<VEC>(xa[c], s, nb);
      ld<VEC>(xb[c], s + a.half, nb);
    }
#pragma unroll
    for (int c = 0; c + 1 < C; c += 2)
      pair_mac2<P, W>(acc_a, acc_b, a.tab[c], a.tab[c + 1], xa[c], xb[c], xa[c + 1], xb[c + 1]);
    if constexpr (C & 1) pair_mac1<P, W>(acc_a, acc_b, a.tab[C - 1], xa[C - 1], xb[C - 1]);
    if constexpr (!ACC) {
      // Piggyback, compile-time XORSet of a (C+P) codec (xrs.go:77-100): data
      // c rides on parity 1 + c % (P-1).  Compile-time source counts are only
      // launched for a whole Encode (PairPlan::encode_xs).
#pragma unroll
      for (int c = 0; c < C; ++c)
#pragma unroll
        for (int w = 0; w < W; ++w) acc_b[1 + c % (P - 1)][w] ^= xa[c][w];
    } else {
#pragma unroll
      for (int c = 0; c < C; ++c) piggyback<P, W>(acc_b, a.pbmask, c, xa[c]);
    }
  } else {
    // Runtime source count: groups of kGrp sources, each group's loads issued
    // together (wave-uniform guards keep the register indexes static).
    constexpr int kGrp = 6;
#if XRS_IND
#pragma unroll
    for (int c0 = 0; c0 < kMaxSrc; c0 += kGrp) {  // unrolled: sb[] indexes static
      if (c0 >= a.n_src) break;
#else
    for (int c0 = 0; c0 < a.n_src; c0 += kGrp) {
#endif
      uint32_t xa[kGrp][W], xb[kGrp][W];
#pragma unroll
      for (int g = 0; g < kGrp; ++g)
        if (c0 + g < a.n_src) {
          const uint64_t s = XRS_SRC(c0 + g);
          ld<VEC>(xa[g], s, nb);
          ld<VEC>(xb[g], s + a.half, nb);
        }
#pragma unroll
      for (int g = 0; g < kGrp; ++g)
        if (c0 + g < a.n_src) {
          pair_mac1<P, W>(acc_a, acc_b, a.tab[c0 + g], xa[g], xb[g]);
          piggyback<P, W>(acc_b, a.pbmask, c0 + g, xa[g]);
        }
    }
  }

#pragma unroll
  for (int r = 0; r < P; ++r) {
    const uint64_t d = XRS_DST(r);
    st<VEC>(acc_a[r], d, nb);
    st<VEC>(acc_b[r], d + a.half, nb);
  }
#undef XRS_DST
#undef XRS_SRC
