// ag_exp.h -- FP64 exp with bit-identical results to the glibc 2.35 x86-64 FMA build of
// exp(), and the reference sigmoid built on it.
//
// Why: the reference's bids are `value * sigmoid(items @ ctx)` (src/Models.py:10-12,
// src/Bidder.py:34-35) and second-price charges ARE bids, so bit-exact charges need an
// exp whose every result equals the one the reference used. The pinned numba 0.55.1
// (requirements.txt:7) lowers np.exp in the jitted sigmoid to the libm call, i.e. glibc.
//
// Algorithm (glibc's table-driven exp; restated, not copied): x = k*ln2/128 + r,
// exp(x) = 2^(k/128) * exp(r), 2^(k/128) from a 128-entry table (ag_exp_table.h, built by
// tools/gen_exp_table.py), exp(r) - 1 by a degree-5 polynomial, with the FMAs placed
// where the FMA build of glibc contracts them. The host test
// (tests/test_exp_restatement.py) compares this exact source, compiled for the CPU,
// against the host libm on 4e7 inputs over the full double range; the GPU test compares
// the device build against the same libm.
//
// Compile with -ffp-contract=off: every FMA below is explicit.
#pragma once
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define AG_HD __host__ __device__ __forceinline__
#else
#define AG_HD static inline
#include <math.h>
#endif

namespace agexp {

constexpr double kInvLn2N = 0x1.71547652b82fep0 * 128.0;
constexpr double kNegLn2HiN = -0x1.62e42fefa0000p-8;
constexpr double kNegLn2LoN = -0x1.cf79abc9e3b3ap-47;
constexpr double kShift = 0x1.8p52;
constexpr double kC2 = 0x1.ffffffffffdbdp-2;
constexpr double kC3 = 0x1.555555555543cp-3;
constexpr double kC4 = 0x1.55555cf172b91p-5;
constexpr double kC5 = 0x1.1111167a4d017p-7;

AG_HD uint64_t asu64(double x) {
  uint64_t u;
  memcpy(&u, &x, 8);
  return u;
}
AG_HD double asf64(uint64_t u) {
  double x;
  memcpy(&x, &u, 8);
  return x;
}

// |x| >= 512 (or the rare k range where the table scale would over/underflow).
AG_HD double exp_special(double tmp, uint64_t sbits, uint64_t ki) {
  if ((ki & 0x80000000ull) == 0) {
    sbits -= 1009ull << 52;  // k > 0: scale down, multiply back
    double scale = asf64(sbits);
    return 0x1p1009 * fma(scale, tmp, scale);
  }
  sbits += 1022ull << 52;  // k < 0: careful rounding into the subnormal range
  double scale = asf64(sbits);
  double y = scale + scale * tmp;
  if (y < 1.0) {
    double lo = (scale - y) + scale * tmp;  // not contracted in the glibc build
    double hi = 1.0 + y;
    lo = 1.0 - hi + y + lo;
    y = (hi + lo) - 1.0;
    if (y == 0.0) y = 0.0;
  }
  return 0x1p-1022 * y;
}

// `tab` points at the 256-entry table (LDS copy on the device, ag_exp_tab on the host).
AG_HD double exp(double x, const uint64_t *tab) {
  uint64_t ux = asu64(x);
  uint32_t abstop = (uint32_t)(ux >> 52) & 0x7ff;
  if (abstop - 0x3c9u >= 0x408u - 0x3c9u) {           // |x| < 2^-54 or |x| >= 512
    if (abstop - 0x3c9u >= 0x80000000u) return 1.0 + x; // tiny
    if (abstop >= 0x409u) {                            // |x| >= 1024, inf, nan
      if (ux == 0xfff0000000000000ull) return 0.0;
      if (abstop >= 0x7ffu) return 1.0 + x;
      return (ux >> 63) ? 0.0 : asf64(0x7ff0000000000000ull);
    }
    abstop = 0;  // large |x|: exp_special below
  }
  double z = kInvLn2N * x;
  double kd = z + kShift;
  uint64_t ki = asu64(kd);
  kd -= kShift;
  double r = fma(kd, kNegLn2LoN, fma(kd, kNegLn2HiN, x));
  uint64_t idx = 2 * (ki & 127);
  uint64_t top = ki << 45;
  double tail = asf64(tab[idx]);
  uint64_t sbits = tab[idx + 1] + top;
  double r2 = r * r;
  double tmp = fma(r2 * r2, fma(r, kC5, kC4), fma(r2, fma(r, kC3, kC2), tail + r));
  if (abstop == 0) return exp_special(tmp, sbits, ki);
  double scale = asf64(sbits);
  return fma(scale, tmp, scale);
}

// The main path of exp above alone, without its range checks: equal to exp(x) whenever
// exp_in_main(x) (2^-54 <= |x| < 512, where exp takes exactly this path). Branch-free, so
// independent calls interleave; callers patch the rare other inputs with exp().
AG_HD bool exp_in_main(double x) {
  const uint32_t abstop = (uint32_t)(asu64(x) >> 52) & 0x7ff;
  return abstop - 0x3c9u < 0x408u - 0x3c9u;
}
AG_HD double exp_main(double x, const uint64_t *tab) {
  double z = kInvLn2N * x;
  double kd = z + kShift;
  uint64_t ki = asu64(kd);
  kd -= kShift;
  double r = fma(kd, kNegLn2LoN, fma(kd, kNegLn2HiN, x));
  uint64_t idx = 2 * (ki & 127);
  uint64_t top = ki << 45;
  double tail = asf64(tab[idx]);
  uint64_t sbits = tab[idx + 1] + top;
  double r2 = r * r;
  double tmp = fma(r2 * r2, fma(r, kC5, kC4), fma(r2, fma(r, kC3, kC2), tail + r));
  double scale = asf64(sbits);
  return fma(scale, tmp, scale);
}

// exp(x) through the branch-free main path, the inputs outside it patched with exp(): the
// same bits as exp(), cheaper in divergent code (AG_EXP_FAST=0: plain exp, for A/B).
#ifndef AG_EXP_FAST
#define AG_EXP_FAST 1
#endif
AG_HD double exp_fast(double x, const uint64_t *tab) {
#if AG_EXP_FAST
  double e = exp_main(x, tab);
  if (__builtin_expect(!exp_in_main(x), 0)) e = exp(x, tab);
  return e;
#else
  return exp(x, tab);
#endif
}

// glibc 2.35's float expf (the algorithm of sysdeps/ieee754/flt-32/e_expf.c, restated):
// x 32/ln2 = k + r (k rounded to nearest through the 1.5 2^52 shift, both steps fused as
// the x86-64 FMA build does), 2^(k/32) from a 32-entry table, 2^(r/32) by a degree-3
// polynomial in double, one rounding to float. What torch.sigmoid's scalar path calls
// (std::exp on a float); equal to the host libm expf for every float
// (tests/test_exp_restatement.py, exhaustive).
// tab32[j] = bits(2^(j/32)) - (j << 47) = ag_exp_tab[8 j + 1] (every 4th 2^(j/128) entry,
// the same correctly rounded values); kept as its own contiguous 256-B table in LDS
// (kExpTabLds layout below), where 32 random lanes hit 32 distinct bank pairs.
constexpr int kExpTabLds = 256 + 32;  // LDS copy: ag_exp_tab, then tab32
AG_HD uint64_t expf_tab_entry(const uint64_t *exp_tab, int j) { return exp_tab[8 * j + 1]; }
constexpr double kInvLn2F = 0x1.71547652b82fep0 * 32.0;
constexpr double kF0 = 0x1.c6af84b912394p-5 / 32768.0;
constexpr double kF1 = 0x1.ebfce50fac4f3p-3 / 1024.0;
constexpr double kF2 = 0x1.62e42ff0c52d6p-1 / 32.0;
AG_HD float expf_glibc(float x, const uint64_t *tab32) {
  // glibc branches out for |x| >= 88 or nan and otherwise falls through to the main path
  // below; here the main path always runs and the out-of-range results are selected
  // (branch-free, for unrolled divergent code)
  const double xd = (double)x;
  double kd = fma(kInvLn2F, xd, kShift);
  const uint64_t ki = asu64(kd);
  kd -= kShift;
  const double r = fma(kInvLn2F, xd, -kd);
  const double s = asf64(tab32[ki & 31] + (ki << 47));
  const double z = fma(kF0, r, kF1);
  const double r2 = r * r;
  double y = fma(kF2, r, 1.0);
  y = fma(z, r2, y);
  float e = (float)(y * s);
  e = x > 0x1.62e42ep6f ? __builtin_inff() : e;  // overflow (+inf included)
  e = x < -0x1.9fe368p6f ? 0.0f : e;             // underflow (-inf included)
  return x != x ? x + x : e;
}

// src/Models.py:10-12  sigmoid(x) = 1.0 / (1.0 + np.exp(-x))  (IEEE division).
AG_HD double sigmoid(double z, const uint64_t *tab) { return 1.0 / (1.0 + exp(-z, tab)); }
AG_HD double sigmoid_fast(double z, const uint64_t *tab) { return 1.0 / (1.0 + exp_fast(-z, tab)); }

}  // namespace agexp
