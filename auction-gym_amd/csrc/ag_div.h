// ag_div.h -- IEEE double division as its parts, so that divisions by one denominator share
// the reciprocal (the learners' BCE rows: p = n / (1 + e) and log1p's c / u divide by the same
// u = 1 + e).
//
// The compiler lowers an IEEE f64 `a / b` on gfx950 to
//   v_div_scale(b, b, a); v_rcp; four FMAs refining the reciprocal r; v_div_scale(a, b, a);
//   q = a' r; rem = fma(-b', q, a'); v_div_fmas(rem, r, q); v_div_fixup(., b, a)
// v_div_scale leaves its operand unchanged (and clears VCC, so v_div_fmas is a plain FMA) unless
// a or b is zero, denormal or near the ends of the exponent range, and v_div_fixup only acts on
// zeros, infinities, NaNs and over/underflow. recip() + div_core() below are that sequence with
// the scaling and the fixup left out: for operands inside div_safe()'s range they give the bits
// of `a / b` (ag_div_selftest compares them over random operands on the device).
#pragma once

namespace agdiv {

// the refined reciprocal of b: the sequence's r (depends on b alone)
__device__ __forceinline__ double recip(double b) {
  const double r0 = __builtin_amdgcn_rcp(b);
  const double e0 = __builtin_fma(-b, r0, 1.0);
  const double r1 = __builtin_fma(r0, e0, r0);
  const double e1 = __builtin_fma(-b, r1, 1.0);
  return __builtin_fma(r1, e1, r1);
}

// a / b given r = recip(b)
__device__ __forceinline__ double div_core(double a, double b, double r) {
  const double q = a * r;
  const double rem = __builtin_fma(-b, q, a);
  return __builtin_fma(rem, r, q);
}

// operands the sequence does not scale and whose quotient the fixup leaves alone: a zero (a
// positive zero: -0 / b would come out +0) or 2^-900 <= |a| <= 2^600, 2^-60 <= |b| <= 2^60
// (v_div_scale scales for a below 2^-969, an exponent difference of 768 or more, a denormal
// b, 1/b or quotient)
__device__ __forceinline__ bool div_safe(double a, double b) {
  const double fa = __builtin_fabs(a), fb = __builtin_fabs(b);
  const bool a_ok = (fa >= 0x1p-900 && fa <= 0x1p600) || (a == 0.0 && !__builtin_signbit(a));
  return a_ok && fb >= 0x1p-60 && fb <= 0x1p60;
}

}  // namespace agdiv
