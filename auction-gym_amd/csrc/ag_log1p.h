// ag_log1p.h -- log1p for the DR bidder's softplus, bit-identical on host and device.
//
// The fdlibm algorithm (public domain): 1 + x = 2^k (1 + f) with 1 + f in [sqrt(2)/2,
// sqrt(2)), s = f / (2 + f), log(1 + f) = f - (hfsq - s (hfsq + R(s^2))), R an odd
// minimax polynomial, plus a correction term c for the rounding of 1 + x. Only IEEE
// double operations (no FMA: compile with -ffp-contract=off), so every compiler / target
// gives the same bits -- unlike libm vs ocml log1p, which differ in the last ulp on ~0.1 %
// of inputs. Accuracy: < 1 ulp (tests/test_exp_restatement.py checks the oracle's copy
// of the same algorithm against libm).
#pragma once
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define AG_L1P_HD __host__ __device__ __forceinline__
#define AG_L1P_MEMBER __host__ __device__ __forceinline__
#else
#define AG_L1P_HD static inline
#define AG_L1P_MEMBER inline
#endif

namespace aglog1p {

AG_L1P_HD uint64_t bits(double x) {
  uint64_t u;
  memcpy(&u, &x, 8);
  return u;
}
AG_L1P_HD double from_bits(uint64_t u) {
  double x;
  memcpy(&x, &u, 8);
  return x;
}

AG_L1P_HD double log1p(double x) {
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  const double Lp1 = 6.666666666666735130e-01, Lp2 = 3.999999999940941908e-01,
               Lp3 = 2.857142874366239149e-01, Lp4 = 2.222219843214978396e-01,
               Lp5 = 1.818357216161805012e-01, Lp6 = 1.531383769920937332e-01,
               Lp7 = 1.479819860511658591e-01;
  const int32_t hx = (int32_t)(bits(x) >> 32), ax = hx & 0x7fffffff;
  int32_t hu = 0, k = 1;
  double f = 0.0, c = 0.0;
  if (hx < 0x3FDA827A) {
    if (ax >= 0x3ff00000) return x == -1.0 ? -__builtin_inf() : __builtin_nan("");
    if (ax < 0x3e200000) {
      if (ax < 0x3c900000) return x;
      return x - x * x * 0.5;
    }
    if (hx > 0 || hx <= (int32_t)0xbfd2bec4) {
      k = 0;
      f = x;
      hu = 1;
    }
  }
  if (hx >= 0x7ff00000) return x + x;
  if (k != 0) {
    double u;
    if (hx < 0x43400000) {
      u = 1.0 + x;
      hu = (int32_t)(bits(u) >> 32);
      k = (hu >> 20) - 1023;
      c = (k > 0) ? 1.0 - (u - x) : x - (u - 1.0);
      c /= u;
    } else {
      u = x;
      hu = (int32_t)(bits(u) >> 32);
      k = (hu >> 20) - 1023;
      c = 0;
    }
    hu &= 0x000fffff;
    const uint64_t lo = bits(u) & 0xffffffffull;
    if (hu < 0x6a09e) {
      u = from_bits(((uint64_t)(uint32_t)(hu | 0x3ff00000) << 32) | lo);
    } else {
      k += 1;
      u = from_bits(((uint64_t)(uint32_t)(hu | 0x3fe00000) << 32) | lo);
      hu = (0x00100000 - hu) >> 2;
    }
    f = u - 1.0;
  }
  const double hfsq = 0.5 * f * f;
  if (hu == 0) {
    if (f == 0.0) {
      if (k == 0) return 0.0;
      c += k * ln2_lo;
      return k * ln2_hi + c;
    }
    const double R = hfsq * (1.0 - 0.66666666666666666 * f);
    if (k == 0) return f - R;
    return k * ln2_hi - ((R - (k * ln2_lo + c)) - f);
  }
  const double s = f / (2.0 + f), z = s * s;
  const double R = z * (Lp1 + z * (Lp2 + z * (Lp3 + z * (Lp4 + z * (Lp5 + z * (Lp6 + z * Lp7))))));
  if (k == 0) return f - (hfsq - s * (hfsq + R));
  return k * ln2_hi - ((hfsq - (s * (hfsq + R) + (k * ln2_lo + c))) - f);
}

// log1p(x) for 2^-29 <= x < 2^53 without branches: both of log1p's paths for a positive x
// (f = x, k = 0 below sqrt(2) - 1; 1 + x = 2^k (1 + f) with the rounding correction c
// above) computed and selected, then the shared tail -- for k = 0 the general tail
// k ln2_hi - ((hfsq - (s (hfsq + R) + (k ln2_lo + c))) - f) equals f - (hfsq - s (hfsq + R))
// bit for bit (IEEE subtraction is antisymmetric, adding +0 is exact). ok = false outside
// that range and on log1p's hu == 0 special case (f on a power-of-two boundary): the caller
// then takes log1p(x).
// D: the two divisions, c / u (u = 1 + x) and f / (2 + f), as D::cu(c, u) and D::fs(f, d) --
// IeeeDiv the plain operator; a device caller may pass its own (ag_dr.hip: a reciprocal of
// 1 + x shared with its own division by 1 + x), which must give the same bits
struct IeeeDiv {
  AG_L1P_MEMBER double cu(double c, double u) const { return c / u; }
  AG_L1P_MEMBER double fs(double f, double d) const { return f / d; }
};
template <class D>
AG_L1P_HD double log1p_main_t(double x, bool &ok, const D &div) {
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  const double Lp1 = 6.666666666666735130e-01, Lp2 = 3.999999999940941908e-01,
               Lp3 = 2.857142874366239149e-01, Lp4 = 2.222219843214978396e-01,
               Lp5 = 1.818357216161805012e-01, Lp6 = 1.531383769920937332e-01,
               Lp7 = 1.479819860511658591e-01;
  const int32_t hx = (int32_t)(bits(x) >> 32);
  const bool small = hx < 0x3FDA827A;  // k = 0: f = x
  double u = 1.0 + x;
  int32_t hu = (int32_t)(bits(u) >> 32);
  int32_t k = (hu >> 20) - 1023;
  double c = (k > 0) ? 1.0 - (u - x) : x - (u - 1.0);
  c = div.cu(c, u);
  hu &= 0x000fffff;
  const uint64_t lo = bits(u) & 0xffffffffull;
  const bool low = hu < 0x6a09e;
  u = from_bits(((uint64_t)(uint32_t)(hu | (low ? 0x3ff00000 : 0x3fe00000)) << 32) | lo);
  k += low ? 0 : 1;
  hu = low ? hu : (0x00100000 - hu) >> 2;
  double f = u - 1.0;
  f = small ? x : f;
  k = small ? 0 : k;
  c = small ? 0.0 : c;
  hu = small ? 1 : hu;
  ok = hx >= 0x3e200000 && hx < 0x43400000 && hu != 0;
  const double hfsq = 0.5 * f * f;
  const double s = div.fs(f, 2.0 + f), z = s * s;
  const double R = z * (Lp1 + z * (Lp2 + z * (Lp3 + z * (Lp4 + z * (Lp5 + z * (Lp6 + z * Lp7))))));
  return k * ln2_hi - ((hfsq - (s * (hfsq + R) + (k * ln2_lo + c))) - f);
}
AG_L1P_HD double log1p_main(double x, bool &ok) { return log1p_main_t(x, ok, IeeeDiv()); }

}  // namespace aglog1p
