// ag_philox.h -- Philox4x32-10 (Salmon et al., SC'11), the counter-based generator of the
// synthetic inputs (ag_generate*) and of the learning bidders' synthetic fit noise.
// oracle/ag_oracle.c ora_philox4x32_10 is the same function on the host.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

__device__ __forceinline__ void philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                       uint32_t k1, uint32_t (&o)[4]) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    const uint32_t n1 = (uint32_t)p1;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    const uint32_t n3 = (uint32_t)p0;
    c0 = n0;
    c1 = n1;
    c2 = n2;
    c3 = n3;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  o[0] = c0;
  o[1] = c1;
  o[2] = c2;
  o[3] = c3;
}

// One synthetic auction (ag_generate; fused into k_oracle's generate mode): Philox4x32-10
// keyed by seed, counter = (global auction index, block, stream). Stream 0, block 0: u ~ U[0,1)
// with 53 bits from words 0-1, the first two participants (Floyd's algorithm, slot order =
// insertion order) from words 2-3; later picks from stream 1, four per call. The context
// (stream 2, two Box-Muller pairs per call): normals z ~ N(0, 1) from 32-bit uniforms in
// float32 -- the hardware log2 / sqrt / sin / cos (v_sin_f32(t) = sin(2 pi t)), |z| <= 6.7 --,
// ctx = scale * z (numpy normal(0, scale) in distribution; tests check it). Round 5: 3
// Philox calls per SP_Oracle auction instead of 5 and no FP64 log / sincos (the generate mode
// was VALU-bound on them). oracle/ag_oracle.c ora_gen_* restate u and the participants bit
// for bit. part holds P <= MAXP entries, x E.
__device__ __forceinline__ float gen_normal_r(uint32_t a) {  // sqrt(-2 ln u1), u1 = (a + 1) / 2^32 in (0, 1]
  const float u1 = (float)(((double)a + 1.0) * 0x1p-32);
  return __builtin_sqrtf(-2.0f * 0.693147180559945309f * __builtin_amdgcn_logf(u1));
}
template <int MAXP, int MAXE>
__device__ __forceinline__ void gen_auction(uint32_t k0, uint32_t k1, uint64_t idx, int N, int P, int E,
                                            double scale, double (&x)[MAXE], int (&part)[MAXP], double &u) {
  const uint32_t c0 = (uint32_t)idx, c1 = (uint32_t)(idx >> 32);
  uint32_t w[4], v[4];
  philox(c0, c1, 0, 0, k0, k1, w);
  u = (double)((((uint64_t)w[0] << 32) | w[1]) >> 11) * 0x1p-53;
  for (int j = N - P; j < N; ++j) {
    const int step = j - (N - P);
    uint32_t word;
    if (step < 2) {
      word = w[2 + step];
    } else {
      if (((step - 2) & 3) == 0) philox(c0, c1, (uint32_t)((step - 2) >> 2), 1, k0, k1, v);
      word = v[(step - 2) & 3];
    }
    int pick = (int)(((uint64_t)word * (uint64_t)(j + 1)) >> 32);
    for (int q = 0; q < step; ++q)
      if (part[q] == pick) {
        pick = j;
        break;
      }
    part[step] = pick;
  }
  for (int m = 0; 2 * m < E; ++m) {
    if ((m & 1) == 0) philox(c0, c1, (uint32_t)(m >> 1), 2, k0, k1, v);
    const float r = gen_normal_r(v[2 * (m & 1)]);
    const float t = (float)v[2 * (m & 1) + 1] * 0x1p-32f;  // [0, 1]
    x[2 * m] = 0.0 + scale * (double)(r * __builtin_amdgcn_cosf(t));
    if (2 * m + 1 < E) x[2 * m + 1] = 0.0 + scale * (double)(r * __builtin_amdgcn_sinf(t));
  }
}

// Synthetic per-participant draws (ag_generate_noise writes them; the general kernel's generate
// mode draws the same bits in place). Same key and counter scheme, stream by kind and slot s:
//  - LR-TS Thompson noise (torch.normal(0, 1/sqrt(q)), src/Models.py:31): coefficient c of slot
//    s from block c / 4 of stream 4 + s, four float32 normals per Philox call (two Box-Muller
//    pairs from 32-bit uniforms, the hardware transcendentals, as the contexts above; round 6:
//    before, one FP64 pair per call -- 30 calls and 30 FP64 log / sincos per slot), times
//    1 / sqrtf(q) of the coefficient;
//  - a fitted policy's rsample draw: the first normal of block 0 of stream 16 + s;
//  - shading draws N(prev_gamma, sigma) (numpy normal(loc, scale), src/Bidder.py:51, :177):
//    prev_gamma + sigma * the first normal of block s of stream 3 (round 6: float32 Box-Muller;
//    before, an FP64 pair -- its log / sincospi held ~100 VGPRs in the generate-mode kernel).
__device__ __forceinline__ void gen_normals4(uint32_t c0, uint32_t c1, uint32_t blk, uint32_t stream, uint32_t k0,
                                             uint32_t k1, float (&z)[4]) {
  uint32_t w[4];
  philox(c0, c1, blk, stream, k0, k1, w);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const float r = gen_normal_r(w[2 * h]);
    const float t = (float)w[2 * h + 1] * 0x1p-32f;
    z[2 * h] = r * __builtin_amdgcn_cosf(t);
    z[2 * h + 1] = r * __builtin_amdgcn_sinf(t);
  }
}
__device__ __forceinline__ float gen_normal1(uint32_t c0, uint32_t c1, uint32_t blk, uint32_t stream, uint32_t k0,
                                             uint32_t k1) {
  uint32_t w[4];
  philox(c0, c1, blk, stream, k0, k1, w);
  return gen_normal_r(w[0]) * __builtin_amdgcn_cosf((float)w[1] * 0x1p-32f);
}
__device__ __forceinline__ double gen_shading_raw(uint32_t c0, uint32_t c1, int s, uint32_t k0, uint32_t k1,
                                                  double prev_gamma, double sigma) {
  return prev_gamma + sigma * (double)gen_normal1(c0, c1, (uint32_t)s, 3, k0, k1);
}
