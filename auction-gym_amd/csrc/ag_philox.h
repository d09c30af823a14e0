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
// keyed by seed, counter = (global auction index, sub-stream). u ~ U[0,1) with 53 bits
// (stream 0); the participants by Floyd's algorithm, slot order = insertion order (stream
// 1); the context as Box-Muller pairs (stream 2), ctx = 0 + scale * z (numpy normal(0,
// scale)). oracle/ag_oracle.c ora_gen_* restate it. part holds P <= MAXP entries, x E.
template <int MAXP, int MAXE>
__device__ __forceinline__ void gen_auction(uint32_t k0, uint32_t k1, uint64_t idx, int N, int P, int E,
                                            double scale, double (&x)[MAXE], int (&part)[MAXP], double &u) {
  const uint32_t c0 = (uint32_t)idx, c1 = (uint32_t)(idx >> 32);
  uint32_t w[4];
  philox(c0, c1, 0, 0, k0, k1, w);
  u = (double)((((uint64_t)w[0] << 32) | w[1]) >> 11) * 0x1p-53;
  for (int j = N - P; j < N; ++j) {
    const int step = j - (N - P);
    if ((step & 3) == 0) philox(c0, c1, (uint32_t)(step >> 2), 1, k0, k1, w);
    int pick = (int)(((uint64_t)w[step & 3] * (uint64_t)(j + 1)) >> 32);
    for (int q = 0; q < step; ++q)
      if (part[q] == pick) {
        pick = j;
        break;
      }
    part[step] = pick;
  }
  for (int m = 0; 2 * m < E; ++m) {
    philox(c0, c1, (uint32_t)m, 2, k0, k1, w);
    const double u1 = (double)(((((uint64_t)w[0] << 32) | w[1]) >> 11) + 1) * 0x1p-53;
    const double u2 = (double)((((uint64_t)w[2] << 32) | w[3]) >> 11) * 0x1p-53;
    const double r = sqrt(-2.0 * log(u1));
    double sn, cs;
    sincospi(2.0 * u2, &sn, &cs);
    x[2 * m] = 0.0 + scale * (r * cs);
    if (2 * m + 1 < E) x[2 * m + 1] = 0.0 + scale * (r * sn);
  }
}
