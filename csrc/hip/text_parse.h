// text_parse.h — decimal parsing shared by the text kernels (text.hip) and
// the fused CSV fold (generic.hip), so both parse a field identically.
#pragma once
#include <hip/hip_runtime.h>
#include "mr_common.h"

namespace mr {
namespace tx {

static __device__ __constant__ double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                             1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

// Decimal number of text[s, s + len): [spaces] [+-] digits [. digits] [eE [+-] digits] [spaces].
// Exact (correctly rounded) when the significant digits fit 2^53 and the
// decimal exponent is within +-22 (one IEEE multiply or divide by an exact
// power of ten); otherwise within a few ulp.  Malformed spans: NaN, and bit 0 of *err.
__device__ __forceinline__ double parse_f64(const u8* p, int len, bool& bad) {
  int j = 0;
  while (j < len && is_ws(p[j])) ++j;
  bool neg = false;
  if (j < len && (p[j] == '+' || p[j] == '-')) neg = p[j++] == '-';
  u64 mant = 0;
  int digits = 0, exp10 = 0, nd = 0;
  bool dot = false;
  for (; j < len; ++j) {
    const u32 ch = p[j];
    if (ch >= '0' && ch <= '9') {
      ++nd;
      if (mant == 0 && ch == '0') {
        if (dot) --exp10;
        continue;
      }
      if (digits < 19) {
        mant = mant * 10 + (ch - '0');
        ++digits;
        if (dot) --exp10;
      } else if (!dot) {
        ++exp10;
      }
    } else if (ch == '.' && !dot) {
      dot = true;
    } else {
      break;
    }
  }
  if (nd == 0) {
    bad = true;
    return __longlong_as_double(0x7FF8000000000000ll);
  }
  if (j < len && (p[j] == 'e' || p[j] == 'E')) {
    ++j;
    bool eneg = false;
    if (j < len && (p[j] == '+' || p[j] == '-')) eneg = p[j++] == '-';
    int e = 0, ne = 0;
    for (; j < len && p[j] >= '0' && p[j] <= '9'; ++j, ++ne) e = e < 100000 ? e * 10 + (p[j] - '0') : e;
    if (ne == 0) bad = true;
    exp10 += eneg ? -e : e;
  }
  while (j < len && is_ws(p[j])) ++j;
  if (j != len) bad = true;
  double v;
  if (mant == 0) {
    v = 0.0;
  } else if (mant < (1ull << 53) && exp10 >= -22 && exp10 <= 22) {
    v = (double)mant;
    v = exp10 >= 0 ? v * kPow10[exp10] : v / kPow10[-exp10];
  } else {
    v = (double)mant * pow(10.0, (double)exp10);
  }
  return neg ? -v : v;
}

}  // namespace tx
}  // namespace mr
