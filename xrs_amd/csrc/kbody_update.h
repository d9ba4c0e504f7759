// kbody_update.h -- the update_rows kernel's body (kernels.hip), included
// inside the kernel functions: XRS_IND 0 with XRS_ROW(row, stripe, off)
// naming the row addressing (update_rows_kernel), XRS_IND 1 for table rows
// (update_rows_ind_kernel).  Not a header.
  constexpr int W = VEC ? 4 : 1;
  const uint64_t gid = logical_block(a.order) * kBlock + threadIdx.x;
  if (gid >= a.total) return;
  const uint64_t stripe = gid / a.chunks;
  const uint64_t off = a.off0 + (gid - stripe * a.chunks) * (4 * W);
  const int nb = VEC ? 16 : static_cast<int>(a.half - off < 4 ? a.half - off : 4);
  // rows == nullptr: one row for the whole batch (plain Update), table 0.
  const int r = a.rows ? a.rows[stripe] - a.row0 : 0;
  if (r < 0 || r >= a.nrows) return;  // another launch's row, or not a data row

#if XRS_IND
  // Table rows: every base address read up front, in one round trip (see
  // kbody_pair.h).
  uint64_t dqb[P];
  const uint64_t o = row_base_ind(a.old_row, stripe) + off, n = row_base_ind(a.new_row, stripe) + off;
#pragma unroll
  for (int q = 0; q < P; ++q) dqb[q] = row_base_ind(a.dst[q], stripe) + off;
#define XRS_DST(q) dqb[q]
#else
  const uint64_t o = XRS_ROW(a.old_row, stripe, off), n = XRS_ROW(a.new_row, stripe, off);
#define XRS_DST(q) XRS_ROW(a.dst[q], stripe, off)
#endif
  uint32_t oa[W], ob[W], na[W], nw[W], pa[P][W], pb[P][W];
  ld<VEC>(oa, o, nb);
  ld<VEC>(ob, o + a.half, nb);
  ld<VEC>(na, n, nb);
  ld<VEC>(nw, n + a.half, nb);
#pragma unroll
  for (int q = 0; q < P; ++q) {
    const uint64_t dq = XRS_DST(q);
    ld<VEC>(pa[q], dq, nb);
    ld<VEC>(pb[q], dq + a.half, nb);
  }
  const int pbq = a.pbq[r];
#pragma unroll
  for (int w = 0; w < W; ++w) {
    const uint32_t da = oa[w] ^ na[w], db = ob[w] ^ nw[w];
    const Sel sa = sel_of(da), sb = sel_of(db);
#pragma unroll
    for (int q = 0; q < P; ++q) {
      const GfTab t = a.tab[r][q];
      pa[q][w] ^= gmul(t, sa);
      pb[q][w] = xor_masked(pb[q][w] ^ gmul(t, sb), da, pbq == q ? ~0u : 0u);
    }
  }
#pragma unroll
  for (int q = 0; q < P; ++q) {
    const uint64_t dq = XRS_DST(q);
    st<VEC>(pa[q], dq, nb);
    st<VEC>(pb[q], dq + a.half, nb);
  }
#undef XRS_DST
