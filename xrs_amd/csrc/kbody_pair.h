// kbody_pair.h -- the pair kernel's body (kernels.hip), included inside the
// kernel functions with XRS_ROW(row, stripe, off) naming the row addressing:
// row_addr for pair_kernel, row_addr_ind for pair_ind_kernel.  Not a header.
  constexpr int W = VEC ? 4 : 1;
  const uint64_t gid = (PLAIN ? uint64_t(blockIdx.x) : logical_block(a.order)) * BS + threadIdx.x;
  if (gid >= a.total) return;
  const uint64_t stripe = gid / a.chunks;
  uint64_t off = a.off0 + (gid - stripe * a.chunks) * (4 * W);
  if (VEC && off > a.last) off = a.last;  // ragged end: overlapping last chunk
  const int nb = VEC ? 16 : static_cast<int>(a.half - off < 4 ? a.half - off : 4);

  uint32_t acc_a[P][W], acc_b[P][W];
  if constexpr (ACC) {
#pragma unroll
    for (int r = 0; r < P; ++r) {
      const uint64_t d = XRS_ROW(a.dst[r], stripe, off);
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
      const uint64_t s = XRS_ROW(a.src[c], stripe, off);
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
    for (int c0 = 0; c0 < a.n_src; c0 += kGrp) {
      uint32_t xa[kGrp][W], xb[kGrp][W];
#pragma unroll
      for (int g = 0; g < kGrp; ++g)
        if (c0 + g < a.n_src) {
          const uint64_t s = XRS_ROW(a.src[c0 + g], stripe, off);
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
    const uint64_t d = XRS_ROW(a.dst[r], stripe, off);
    st<VEC>(acc_a[r], d, nb);
    st<VEC>(acc_b[r], d + a.half, nb);
  }
