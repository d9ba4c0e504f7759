// gf256.cpp -- host GF(2^8)/0x11d tables, v_perm lookup tables, matrix inverse.
#include "gf256.h"

#include <utility>

namespace xrs {

const GF& GF::get() {
  static const GF g;
  return g;
}

GF::GF() {
  unsigned v = 1;
  for (int i = 0; i < 255; ++i) {
    exp_[i] = static_cast<uint8_t>(v);
    log_[v] = static_cast<uint8_t>(i);
    v <<= 1;
    if (v & 0x100) v ^= 0x11d;
  }
  for (int i = 255; i < 512; ++i) exp_[i] = exp_[i - 255];
  log_[0] = 0;
  auto pack = [&](uint8_t c, int e0, int e1, int e2, int e3) -> uint32_t {
    return static_cast<uint32_t>(mul(c, static_cast<uint8_t>(e0))) |
           static_cast<uint32_t>(mul(c, static_cast<uint8_t>(e1))) << 8 |
           static_cast<uint32_t>(mul(c, static_cast<uint8_t>(e2))) << 16 |
           static_cast<uint32_t>(mul(c, static_cast<uint8_t>(e3))) << 24;
  };
  for (int c = 0; c < 256; ++c) {
    const uint8_t cc = static_cast<uint8_t>(c);
    GfTab& t = tabs_[c];
    t.lo0 = pack(cc, 0, 1, 2, 3);            // bits 0-2, entries 0..3
    t.hi0 = pack(cc, 4, 5, 6, 7);            //           entries 4..7
    t.lo1 = pack(cc, 0, 8, 16, 24);          // bits 3-5, entries 0..3
    t.hi1 = pack(cc, 32, 40, 48, 56);        //           entries 4..7
    t.top = pack(cc, 0, 64, 128, 192);       // bits 6-7
  }
}

bool GF::invert(std::vector<uint8_t>& m, int n) const {
  std::vector<uint8_t> r(static_cast<size_t>(n) * n, 0);
  for (int i = 0; i < n; ++i) r[static_cast<size_t>(i) * n + i] = 1;
  auto at = [n](std::vector<uint8_t>& a, int i, int j) -> uint8_t& {
    return a[static_cast<size_t>(i) * n + j];
  };
  for (int c = 0; c < n; ++c) {
    int piv = -1;
    for (int i = c; i < n; ++i)
      if (at(m, i, c)) {
        piv = i;
        break;
      }
    if (piv < 0) return false;
    if (piv != c)
      for (int j = 0; j < n; ++j) {
        std::swap(at(m, c, j), at(m, piv, j));
        std::swap(at(r, c, j), at(r, piv, j));
      }
    const uint8_t f = inv(at(m, c, c));
    for (int j = 0; j < n; ++j) {
      at(m, c, j) = mul(at(m, c, j), f);
      at(r, c, j) = mul(at(r, c, j), f);
    }
    for (int i = 0; i < n; ++i) {
      const uint8_t g = at(m, i, c);
      if (i == c || g == 0) continue;
      for (int j = 0; j < n; ++j) {
        at(m, i, j) ^= mul(g, at(m, c, j));
        at(r, i, j) ^= mul(g, at(r, c, j));
      }
    }
  }
  m.swap(r);
  return true;
}

}  // namespace xrs
