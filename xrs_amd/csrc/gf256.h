// gf256.h -- host-side GF(2^8) arithmetic for the codec planner.
//
// Field: GF(2^8) with the primitive polynomial 0x11d (x^8+x^4+x^3+x^2+1),
// generator 2 -- the field of github.com/templexxx/reedsolomon v1.1.3
// (go.mod:6), pinned by the reference KAT xrs_test.go:108-115.
#pragma once
#include <stdint.h>

#include <vector>

#include "xrs_plan.h"

namespace xrs {

class GF {
 public:
  static const GF& get();
  uint8_t mul(uint8_t a, uint8_t b) const {
    return (a == 0 || b == 0) ? 0 : exp_[log_[a] + log_[b]];
  }
  uint8_t inv(uint8_t a) const { return a == 0 ? 0 : exp_[255 - log_[a]]; }
  // v_perm_b32 lookup tables for "multiply by c" (see GfTab).
  GfTab tab(uint8_t c) const { return tabs_[c]; }

  // In-place inverse of an n x n row-major matrix; false if singular.
  bool invert(std::vector<uint8_t>& m, int n) const;

 private:
  GF();
  uint8_t exp_[512];
  uint8_t log_[256];
  GfTab tabs_[256];
};

}  // namespace xrs
