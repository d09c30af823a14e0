// ag_replay.cpp -- replay-mode draws on the host, in C: the reference's per-round numpy
// draws (src/Auction.py:30-42, :65; the shading bidders' src/Bidder.py:51, 177, 354, 461)
// for a whole batch of rounds in one call, instead of one Python round trip per round.
//
// The generator is numpy's Generator(PCG64) (src/main.py:29 np.random.default_rng(seed)):
//  - PCG64 (PCG-XSL-RR 128/64: 128-bit LCG step, then the xor-shift-low / random-rotation
//    output of the new state) restated here, with numpy's 32-bit half buffer (has_uint32,
//    uinteger) -- the caller passes bit_generator.state in and gets it back advanced, so the
//    Python generator continues exactly where the reference's would;
//  - the distributions are numpy's own C implementations from libnpyrandom (numpy's
//    documented C API, numpy/random/lib/libnpyrandom.a): random_normal (ziggurat),
//    random_bounded_uint64(_fill) (Lemire's bounded integers);
//  - Generator.choice(N, P, replace=False) restated from numpy's Generator.choice (Floyd's
//    sampling with a linear-probing hash set, then a Fisher-Yates shuffle of the sample; a
//    tail shuffle of arange(N) when N > 10000 and P > N // 50).
// Validated against numpy itself round by round and state by state
// (tests/test_host.py::test_replay_draws_match_numpy).
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <sched.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "auctiongym.h"
#include "ag_host.h"

extern "C" {
// numpy/_core/include/numpy/random/bitgen.h
typedef struct bitgen {
  void *state;
  uint64_t (*next_uint64)(void *st);
  uint32_t (*next_uint32)(void *st);
  double (*next_double)(void *st);
  uint64_t (*next_raw)(void *st);
} bitgen_t;
// numpy/_core/include/numpy/random/distributions.h (libnpyrandom)
double random_normal(bitgen_t *bitgen_state, double loc, double scale);
double random_uniform(bitgen_t *bitgen_state, double lower, double range);
uint64_t random_bounded_uint64(bitgen_t *bitgen_state, uint64_t off, uint64_t rng, uint64_t mask, bool use_masked);
void random_bounded_uint64_fill(bitgen_t *bitgen_state, uint64_t off, uint64_t rng, intptr_t cnt, bool use_masked,
                                uint64_t *out);
}

namespace {

struct Pcg64 {
  unsigned __int128 state, inc;
  int has_uint32;
  uint32_t uinteger;
};

constexpr unsigned __int128 kPcgMult = ((unsigned __int128)2549297995355413924ULL << 64) | 4865540595714422341ULL;

uint64_t pcg_next64(void *st) {
  Pcg64 *p = static_cast<Pcg64 *>(st);
  p->state = p->state * kPcgMult + p->inc;
  const uint64_t hi = (uint64_t)(p->state >> 64), lo = (uint64_t)p->state;
  const unsigned rot = (unsigned)(p->state >> 122);
  const uint64_t x = hi ^ lo;
  return (x >> rot) | (x << ((64 - rot) & 63));
}

uint32_t pcg_next32(void *st) {
  Pcg64 *p = static_cast<Pcg64 *>(st);
  if (p->has_uint32) {
    p->has_uint32 = 0;
    return p->uinteger;
  }
  const uint64_t n = pcg_next64(st);
  p->has_uint32 = 1;
  p->uinteger = (uint32_t)(n >> 32);
  return (uint32_t)(n & 0xffffffffu);
}

double pcg_next_double(void *st) { return (double)(pcg_next64(st) >> 11) * (1.0 / 9007199254740992.0); }

uint64_t gen_mask(uint64_t m) {
  m |= m >> 1;
  m |= m >> 2;
  m |= m >> 4;
  m |= m >> 8;
  m |= m >> 16;
  m |= m >> 32;
  return m;
}

void shuffle_int(bitgen_t *bg, int64_t n, int64_t first, int64_t *data) {
  for (int64_t i = n - 1; i >= first; --i) {
    const int64_t j = (int64_t)random_bounded_uint64(bg, 0, (uint64_t)i, 0, false);
    const int64_t t = data[j];
    data[j] = data[i];
    data[i] = t;
  }
}

// Generator.choice(pop, size, replace=False) -> out[size]
void choice_no_replace(bitgen_t *bg, int64_t pop, int64_t size, int64_t *out, std::vector<int64_t> &arange,
                       std::vector<uint64_t> &hash_set) {
  if (pop > 10000 && size > pop / 50) {  // tail shuffle
    arange.resize((size_t)pop);
    for (int64_t i = 0; i < pop; ++i) arange[(size_t)i] = i;
    shuffle_int(bg, pop, pop - size > 1 ? pop - size : 1, arange.data());
    memcpy(out, arange.data() + (pop - size), (size_t)size * sizeof(int64_t));
    return;
  }
  const uint64_t mask = gen_mask((uint64_t)(1.2 * (double)size));
  hash_set.assign((size_t)(mask + 1), ~0ull);
  for (int64_t j = pop - size; j < pop; ++j) {
    const uint64_t val = random_bounded_uint64(bg, 0, (uint64_t)j, 0, false);
    uint64_t loc = val & mask;
    while (hash_set[loc] != ~0ull && hash_set[loc] != val) loc = (loc + 1) & mask;
    if (hash_set[loc] == ~0ull) {
      hash_set[loc] = val;
      out[j - pop + size] = (int64_t)val;
    } else {
      loc = (uint64_t)j & mask;
      while (hash_set[loc] != ~0ull) loc = (loc + 1) & mask;
      hash_set[loc] = (uint64_t)j;
      out[j - pop + size] = j;
    }
  }
  shuffle_int(bg, size, 1, out);
}

// ---- torch's CPU generator (at::CPUGeneratorImpl), restated: the mt19937 engine
// (ATen/core/MT19937RNGEngine.h), random() = one 32-bit output, random64() = (first << 32) |
// second, and the distributions the reference's draws reach (ATen/core/DistributionsHelper.h,
// ATen/native/cpu/DistributionTemplates.h). The state travels as the blob of
// torch.get_rng_state() (CPUGeneratorImplState, layout in include/auctiongym.h).
constexpr int kMtN = 624, kMtM = 397;
constexpr int64_t kTorchStateBytes = 5056;

struct TorchRng {
  uint64_t seed;
  int32_t left, seeded;
  uint32_t next;
  uint32_t state[kMtN];
  double normal_y;  // the cached second value of normal_distribution<double>
  int32_t normal_valid;
};

void torch_load(TorchRng &t, const uint8_t *b) {
  uint64_t next, w;
  memcpy(&t.seed, b, 8);
  memcpy(&t.left, b + 8, 4);
  memcpy(&t.seeded, b + 12, 4);
  memcpy(&next, b + 16, 8);
  t.next = (uint32_t)next;
  for (int i = 0; i < kMtN; ++i) {
    memcpy(&w, b + 24 + 8 * i, 8);
    t.state[i] = (uint32_t)w;
  }
  memcpy(&t.normal_y, b + 5024, 8);
  memcpy(&t.normal_valid, b + 5040, 4);
}

void torch_store(const TorchRng &t, uint8_t *b) {
  const uint64_t next = t.next;
  memcpy(b + 8, &t.left, 4);
  memcpy(b + 16, &next, 8);
  for (int i = 0; i < kMtN; ++i) {
    const uint64_t w = t.state[i];
    memcpy(b + 24 + 8 * i, &w, 8);
  }
  // torch's get_state() fills normal_y only while the cached value is valid (0 otherwise)
  const double y = t.normal_valid ? t.normal_y : 0.0;
  memcpy(b + 5024, &y, 8);
  memcpy(b + 5040, &t.normal_valid, 4);
}

uint32_t mt_twist(uint32_t u, uint32_t v) {
  return (((u & 0x80000000u) | (v & 0x7fffffffu)) >> 1) ^ ((v & 1u) ? 0x9908b0dfu : 0u);
}

uint32_t torch_random(TorchRng &t) {
  if (--t.left == 0) {  // next_state: the whole vector regenerated
    t.left = kMtN;
    t.next = 0;
    for (int i = 0; i < kMtN - kMtM; ++i) t.state[i] = t.state[i + kMtM] ^ mt_twist(t.state[i], t.state[i + 1]);
    for (int i = kMtN - kMtM; i < kMtN - 1; ++i)
      t.state[i] = t.state[i + kMtM - kMtN] ^ mt_twist(t.state[i], t.state[i + 1]);
    t.state[kMtN - 1] = t.state[kMtM - 1] ^ mt_twist(t.state[kMtN - 1], t.state[0]);
  }
  uint32_t y = t.state[t.next++];
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

// uniform_real_distribution<double>(0, 1): 53 bits of random64()
double torch_uniform_double(TorchRng &t) {
  const uint64_t hi = torch_random(t), lo = torch_random(t);
  return (double)(((hi << 32) | lo) & ((1ull << 53) - 1)) * 0x1p-53;
}

// normal_distribution<double>(0, 1)() (Box-Muller, the second value cached in the generator):
// what torch.empty(1).normal_() returns (cast to float) -- Normal.rsample of one value
double torch_normal_double(TorchRng &t) {
  if (t.normal_valid) {
    t.normal_valid = 0;
    return t.normal_y;
  }
  const double u1 = torch_uniform_double(t), u2 = torch_uniform_double(t);
  const double r = sqrt(-2.0 * log1p(-u2));
  const double theta = 2.0 * 3.14159265358979323846 * u1;
  t.normal_y = r * sin(theta);
  t.normal_valid = 1;
  return r * cos(theta);
}

// torch.normal's CPU kernel for float tensors of >= 16 elements is normal_fill_AVX2
// (ATen/native/cpu/DistributionTemplates.h; the AVX2 code serves the AVX512 capability too):
// Box-Muller over blocks of 16 with the Cephes single-precision log / sincos of avx_mathfun.h
// (Julien Pommier's SSE/AVX port of Cephes logf, sinf, cosf). Restated per lane below, with
// the multiply-adds the x86-64 build fuses (GCC contracts the intrinsic mul + add pairs)
// written as fmaf; checked against torch on every 24-bit uniform it can feed them
// (tests/test_host.py::test_torch_normal_fill_restatement, tools/torch_normal_probe.sh).
inline uint32_t f2u(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}
inline float u2f(uint32_t u) {
  float f;
  memcpy(&f, &u, 4);
  return f;
}

// log256_ps for x in (0, 1] (the Box-Muller radius argument 1 - u, u in [0, 1))
float cephes_logf(float x) {
  if (x < u2f(0x00800000u)) x = u2f(0x00800000u);  // cut off denormals (max with min_norm_pos)
  int32_t ex = (int32_t)(f2u(x) >> 23) - 0x7f;
  x = u2f((f2u(x) & ~0x7f800000u) | f2u(0.5f));
  float e = (float)ex + 1.0f;
  const bool lt = x < 0.707106781186547524f;
  const float tmp = lt ? x : 0.0f;
  x = x - 1.0f;
  e = e - (lt ? 1.0f : 0.0f);
  x = x + tmp;
  const float z = x * x;
  float y = 7.0376836292E-2f;
  y = fmaf(y, x, -1.1514610310E-1f);
  y = fmaf(y, x, 1.1676998740E-1f);
  y = fmaf(y, x, -1.2420140846E-1f);
  y = fmaf(y, x, 1.4249322787E-1f);
  y = fmaf(y, x, -1.6668057665E-1f);
  y = fmaf(y, x, 2.0000714765E-1f);
  y = fmaf(y, x, -2.4999993993E-1f);
  y = fmaf(y, x, 3.3333331174E-1f);
  y = y * x;
  y = fmaf(y, z, e * -2.12194440e-4f);
  y = fmaf(-z, 0.5f, y);
  x = x + y;
  return fmaf(e, 0.693359375f, x);
}

// sincos256_ps for x >= 0 (theta = 2 pi u)
void cephes_sincosf(float x, float *s, float *c) {
  const uint32_t sign_sin0 = f2u(x) & 0x80000000u;
  x = u2f(f2u(x) & 0x7fffffffu);
  int32_t j = (int32_t)(x * 1.27323954473516f);  // cvttps: truncation
  j = (j + 1) & ~1;
  const float y = (float)j;
  const uint32_t swap_sin = (uint32_t)(j & 4) << 29;
  const bool poly = (j & 2) == 0;
  x = fmaf(y, -0.78515625f, x);
  x = fmaf(y, -2.4187564849853515625e-4f, x);
  x = fmaf(y, -3.77489497744594108e-8f, x);
  const uint32_t sign_cos = (uint32_t)(~(j - 2) & 4) << 29;
  const uint32_t sign_sin = sign_sin0 ^ swap_sin;
  const float z = x * x;
  float yc = 2.443315711809948E-005f;
  yc = fmaf(yc, z, -1.388731625493765E-003f);
  yc = fmaf(yc, z, 4.166664568298827E-002f);
  yc = yc * z;
  yc = fmaf(yc, z, -(z * 0.5f));
  yc = yc + 1.0f;
  float ys = -1.9515295891E-4f;
  ys = fmaf(ys, z, 8.3321608736E-3f);
  ys = fmaf(ys, z, -1.6666654611E-1f);
  ys = ys * z;
  ys = fmaf(ys, x, x);
  // the polynomial selection as the vector code does it (and / andnot, subtract, add)
  const float ysin2 = poly ? ys : 0.0f, ysin1 = poly ? 0.0f : yc;
  const float s_ = ysin1 + ysin2, c_ = (yc - ysin1) + (ys - ysin2);
  *s = u2f(f2u(s_) ^ sign_sin);
  *c = u2f(f2u(c_) ^ sign_cos);
}

// normal_fill_16_AVX2 with mean 0, std 1 (u1 = 1 - x[j], u2 = x[j + 8])
void normal_block16(float *d) {
  const float two_pi = (float)(2.0 * 3.14159265358979323846);
  for (int j = 0; j < 8; ++j) {
    const float u1 = 1.0f - d[j], u2 = d[j + 8];
    const float radius = sqrtf(-2.0f * cephes_logf(u1));
    float sn, cs;
    cephes_sincosf(two_pi * u2, &sn, &cs);
    d[j] = fmaf(radius * cs, 1.0f, 0.0f);
    d[j + 8] = fmaf(radius * sn, 1.0f, 0.0f);
  }
}

// normal_fill_AVX2 of n >= 16 contiguous floats, split in two: the generator's part (n 24-bit
// uniforms, then 16 fresh ones for the recomputed last block when n % 16 != 0: u[n + 16]) runs
// in draw order; the transform (the blocks of 16, then the last block from the fresh
// uniforms) depends on nothing else, so a batch's transforms run in parallel afterwards.
int normal_fill_uniforms(int n) { return n + (n % 16 ? 16 : 0); }
void torch_normal_fill_uniforms(TorchRng &t, float *u, int n) {
  for (int i = 0; i < normal_fill_uniforms(n); ++i) u[i] = (float)((double)(torch_random(t) & 0xffffffu) * 0x1p-24);
}
void torch_normal_fill_transform(float *x, const float *u, int n) {
  for (int i = 0; i < n; ++i) x[i] = u[i];
  for (int i = 0; i + 16 <= n; i += 16) normal_block16(x + i);
  if (n % 16) {
    float *d = x + n - 16;
    for (int i = 0; i < 16; ++i) d[i] = u[n + i];
    normal_block16(d);
  }
}

// host threads for the parallel transforms: AG_HOST_THREADS, else the CPUs this process may
// run on, capped by the cgroup's CPU quota (a GPU box shows every core of the machine but
// grants a share) and by 16
int host_threads() {
  if (const char *e = getenv("AG_HOST_THREADS")) {
    const int n = atoi(e);
    if (n > 0) return n;
  }
  cpu_set_t set;
  int n = 1;
  if (sched_getaffinity(0, sizeof set, &set) == 0) n = CPU_COUNT(&set);
  if (FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char q[32] = {0};
    long long per = 0;
    if (fscanf(f, "%31s %lld", q, &per) == 2 && strcmp(q, "max") != 0 && per > 0) {
      const long long lim = (atoll(q) + per - 1) / per;
      if (lim >= 1 && lim < n) n = (int)lim;
    }
    fclose(f);
  }
  return n < 1 ? 1 : (n > 16 ? 16 : n);
}

template <typename F>
void parallel_for(int64_t n, F fn) {
  const int T = (int)std::min<int64_t>(host_threads(), std::max<int64_t>(1, n / 1024));
  if (T <= 1) {
    fn(0, n);
    return;
  }
  std::vector<std::thread> th;
  for (int k = 0; k < T; ++k) th.emplace_back([&, k] { fn(n * k / T, n * (k + 1) / T); });
  for (auto &t : th) t.join();
}

}  // namespace

extern "C" int ag_replay_draw(ag_pcg64_state *rng, int64_t B, int32_t N, int32_t P, int32_t E, double embedding_var,
                              int32_t max_slots, const uint8_t *shading, const double *prev_gamma,
                              const double *gamma_sigma, double *ctx, int32_t *part, double *gamma_raw, double *u) {
  if (!rng || !ctx || !part || !u) return ag_set_error(AG_ERR_INVALID, "ag_replay_draw: null argument");
  if (int rc = ag_check_struct(rng, "ag_replay_draw", "ag_pcg64_state")) return rc;
  if (B < 0 || N < 1 || P < 1 || E < 0 || max_slots < 1)
    return ag_set_error(AG_ERR_INVALID, "ag_replay_draw: bad sizes");
  if (P > N) return ag_set_error(AG_ERR_INVALID, "Cannot take a larger sample than population when replace is False");
  if (shading && (!prev_gamma || !gamma_sigma || !gamma_raw))
    return ag_set_error(AG_ERR_INVALID, "ag_replay_draw: shading needs prev_gamma, gamma_sigma and gamma_raw");
  Pcg64 st;
  st.state = ((unsigned __int128)rng->state_hi << 64) | rng->state_lo;
  st.inc = ((unsigned __int128)rng->inc_hi << 64) | rng->inc_lo;
  st.has_uint32 = rng->has_uint32 ? 1 : 0;
  st.uinteger = rng->uinteger;
  bitgen_t bg{&st, pcg_next64, pcg_next32, pcg_next_double, pcg_next64};
  std::vector<int64_t> sample((size_t)P), arange;
  std::vector<uint64_t> hash_set;
  for (int64_t r = 0; r < B; ++r) {
    if (max_slots > 1) {  // rng.integers(1, max_slots + 1) (src/Auction.py:30); nothing drawn for 1 slot
      uint64_t slots;
      random_bounded_uint64_fill(&bg, 1, (uint64_t)(max_slots - 1), 1, false, &slots);
    }
    for (int e = 0; e < E; ++e) ctx[(int64_t)e * B + r] = random_normal(&bg, 0.0, embedding_var);  // :33
    choice_no_replace(&bg, N, P, sample.data(), arange, hash_set);                                  // :42
    for (int s = 0; s < P; ++s) {
      const int64_t a = sample[(size_t)s];
      part[(int64_t)s * B + r] = (int32_t)a;
      if (gamma_raw) {  // the shading bidders' rng.normal(prev_gamma, gamma_sigma), slot order
        gamma_raw[(int64_t)s * B + r] =
            (shading && shading[a]) ? random_normal(&bg, prev_gamma[a], gamma_sigma[a]) : (double)NAN;
      }
    }
    u[r] = pcg_next_double(&st);  // rng.binomial(1, p) consumes one next_double (:65)
  }
  rng->state_hi = (uint64_t)(st.state >> 64);
  rng->state_lo = (uint64_t)st.state;
  rng->inc_hi = (uint64_t)(st.inc >> 64);
  rng->inc_lo = (uint64_t)st.inc;
  rng->has_uint32 = st.has_uint32;
  rng->uinteger = st.uinteger;
  return AG_OK;
}

// the Box-Muller block of torch's float normal kernel (host checks only: tests/test_host.py)
extern "C" void ag_torch_normal_block16(float *d) { normal_block16(d); }

extern "C" int ag_replay_draw_population(ag_pcg64_state *rng, uint8_t *torch_state, int64_t torch_state_bytes,
                                         int64_t B, int32_t N, int32_t P, int32_t E, double embedding_var,
                                         int32_t max_slots, const uint8_t *shading, const double *prev_gamma,
                                         const double *gamma_sigma, const uint8_t *ts, const float *ts_std,
                                         int32_t KDo, const int32_t *ts_kdo, const uint8_t *policy,
                                         const uint8_t *search, double *ctx,
                                         int32_t *part, double *gamma_raw, double *u, float *ts_noise,
                                         float *policy_eps, double *gamma_grid) {
  const char *who = "ag_replay_draw_population";
  if (!rng || !ctx || !part || !u) return ag_set_error(AG_ERR_INVALID, "%s: null argument", who);
  if (int rc = ag_check_struct(rng, who, "ag_pcg64_state")) return rc;
  if (B < 0 || B >= (int64_t)1 << 31 || N < 1 || P < 1 || E < 0 || max_slots < 1)
    return ag_set_error(AG_ERR_INVALID, "%s: bad sizes", who);
  if (P > N) return ag_set_error(AG_ERR_INVALID, "Cannot take a larger sample than population when replace is False");
  if (shading && (!prev_gamma || !gamma_sigma || !gamma_raw))
    return ag_set_error(AG_ERR_INVALID, "%s: shading needs prev_gamma, gamma_sigma and gamma_raw", who);
  const bool torch_draws = ts || policy;
  if (torch_draws && (!torch_state || torch_state_bytes != kTorchStateBytes))
    return ag_set_error(AG_ERR_INVALID, "%s: torch draws need the %lld-byte torch.get_rng_state() blob", who,
                        (long long)kTorchStateBytes);
  if (ts && (!ts_std || !ts_noise || KDo < 16 || KDo > 4096))
    return ag_set_error(AG_ERR_INVALID, "%s: Thompson draws need ts_std, ts_noise and 16 <= K*Do <= 4096 "
                        "(torch's >= 16-element normal kernel)", who);
  for (int a = 0; ts && ts_kdo && a < N; ++a)
    if (ts[a] && (ts_kdo[a] < 16 || ts_kdo[a] > KDo))
      return ag_set_error(AG_ERR_INVALID, "%s: agent %d's K*Do = %d not in [16, %d]", who, a, ts_kdo[a], KDo);
  if (policy && !policy_eps) return ag_set_error(AG_ERR_INVALID, "%s: policy draws need policy_eps", who);
  if (search && !gamma_grid) return ag_set_error(AG_ERR_INVALID, "%s: search draws need gamma_grid", who);
  Pcg64 st;
  st.state = ((unsigned __int128)rng->state_hi << 64) | rng->state_lo;
  st.inc = ((unsigned __int128)rng->inc_hi << 64) | rng->inc_lo;
  st.has_uint32 = rng->has_uint32 ? 1 : 0;
  st.uinteger = rng->uinteger;
  bitgen_t bg{&st, pcg_next64, pcg_next32, pcg_next_double, pcg_next64};
  TorchRng tr;
  if (torch_draws) torch_load(tr, torch_state);
  const int64_t T = (B + 63) / 64;
  if (ts) memset(ts_noise, 0, sizeof(float) * (size_t)P * (size_t)T * (size_t)KDo * 64);
  std::vector<int64_t> sample((size_t)P), arange;
  std::vector<uint64_t> hash_set;
  const int NU = ts ? KDo + 16 : 0;  // >= normal_fill_uniforms(n) for every n <= KDo
  std::vector<float> tsu(ts ? (size_t)B * P * NU : 0);  // the Thompson draws' uniforms, [B][P][NU]
  double grid[128];
  for (int64_t r = 0; r < B; ++r) {
    if (max_slots > 1) {  // rng.integers(1, max_slots + 1) (src/Auction.py:30)
      uint64_t slots;
      random_bounded_uint64_fill(&bg, 1, (uint64_t)(max_slots - 1), 1, false, &slots);
    }
    for (int e = 0; e < E; ++e) ctx[(int64_t)e * B + r] = random_normal(&bg, 0.0, embedding_var);  // :33
    choice_no_replace(&bg, N, P, sample.data(), arange, hash_set);                                  // :42
    for (int s = 0; s < P; ++s) {
      const int64_t a = sample[(size_t)s];
      part[(int64_t)s * B + r] = (int32_t)a;
      if (gamma_raw) gamma_raw[(int64_t)s * B + r] = (double)NAN;
      if (policy) policy_eps[(int64_t)s * B + r] = 0.0f;
      if (search)
        for (int i = 0; i < 128; ++i) gamma_grid[((int64_t)s * 128 + i) * B + r] = 0.0;
      if (ts && ts[a])  // Agent.select_item: the allocator's Thompson draw (src/Models.py:31)
        torch_normal_fill_uniforms(tr, tsu.data() + ((size_t)r * P + s) * NU, ts_kdo ? ts_kdo[a] : KDo);
      if (policy && policy[a]) {  // the bidder's rsample (src/Models.py:87-88, :160-161)
        policy_eps[(int64_t)s * B + r] = (float)torch_normal_double(tr);
        continue;
      }
      if (search && search[a]) {  // src/Bidder.py:184-186
        for (int i = 0; i < 128; ++i) grid[i] = random_uniform(&bg, 0.1, 1.0 - 0.1);
        std::sort(grid, grid + 128);
        for (int i = 0; i < 128; ++i) gamma_grid[((int64_t)s * 128 + i) * B + r] = grid[i];
        continue;
      }
      if (shading && shading[a])  // an uninitialised shading bidder's Gaussian gamma
        gamma_raw[(int64_t)s * B + r] = random_normal(&bg, prev_gamma[a], gamma_sigma[a]);
    }
    u[r] = pcg_next_double(&st);  // rng.binomial(1, p) consumes one next_double (:65)
  }
  if (ts)  // the Box-Muller transforms of the Thompson draws, rounds in parallel
    parallel_for(B, [&](int64_t r0, int64_t r1) {
      std::vector<float> z((size_t)KDo);
      for (int64_t r = r0; r < r1; ++r)
        for (int s = 0; s < P; ++s) {
          const int64_t a = part[(int64_t)s * B + r];
          if (!ts[a]) continue;
          const int n = ts_kdo ? ts_kdo[a] : KDo;  // the agent's own K*Do (its rows first)
          torch_normal_fill_transform(z.data(), tsu.data() + ((size_t)r * P + s) * NU, n);
          const float *sd = ts_std + a * KDo;
          float *dst = ts_noise + (((int64_t)s * T + r / 64) * KDo) * 64 + (r % 64);
          for (int i = 0; i < n; ++i) dst[(int64_t)i * 64] = z[(size_t)i] * sd[i] + 0.0f;  // .mul_(std).add_(0.0)
        }
    });
  rng->state_hi = (uint64_t)(st.state >> 64);
  rng->state_lo = (uint64_t)st.state;
  rng->inc_hi = (uint64_t)(st.inc >> 64);
  rng->inc_lo = (uint64_t)st.inc;
  rng->has_uint32 = st.has_uint32;
  rng->uinteger = st.uinteger;
  if (torch_draws) torch_store(tr, torch_state);
  return AG_OK;
}

// `epochs` x torch.empty(n).normal_() from torch's CPU generator (the rsample draws of the
// learning bidders' policy fits, Normal.rsample -> _standard_normal, src/Models.py:160, :87),
// one epoch per row of out [epochs][n]; the generator (the torch.get_rng_state() blob) is
// advanced in place. n >= 16: normal_fill_AVX2 (n uniforms, + 16 for the recomputed last block);
// n < 16: the scalar kernel, (float) normal_distribution<double> per element with its cached
// second value. The generator pass runs in draw order, the transforms in parallel.
extern "C" int ag_torch_normal_epochs(uint8_t *torch_state, int64_t torch_state_bytes, int64_t n, int32_t epochs,
                                      float *out) {
  if (!torch_state || torch_state_bytes != kTorchStateBytes || (!out && epochs > 0))
    return ag_set_error(AG_ERR_INVALID, "ag_torch_normal_epochs: needs the %lld-byte torch.get_rng_state() blob "
                        "and out", (long long)kTorchStateBytes);
  if (n < 1 || epochs < 0 || n > (int64_t)1 << 31)
    return ag_set_error(AG_ERR_INVALID, "ag_torch_normal_epochs: bad sizes");
  TorchRng tr;
  torch_load(tr, torch_state);
  if (n < 16) {
    for (int64_t e = 0; e < epochs; ++e)
      for (int64_t i = 0; i < n; ++i) out[e * n + i] = (float)torch_normal_double(tr);
  } else {
    const int64_t U = normal_fill_uniforms((int)n);
    std::vector<float> u((size_t)U * (size_t)epochs);
    for (int64_t e = 0; e < epochs; ++e) torch_normal_fill_uniforms(tr, u.data() + (size_t)e * U, (int)n);
    // epochs split over the host threads (the per-epoch work is n floats: split by epochs * n)
    const int T = (int)std::max<int64_t>(1, std::min<int64_t>(std::min<int64_t>(host_threads(), epochs),
                                                              (int64_t)epochs * n / 4096));
    auto run = [&](int64_t e0, int64_t e1) {
      for (int64_t e = e0; e < e1; ++e) torch_normal_fill_transform(out + e * n, u.data() + (size_t)e * U, (int)n);
    };
    if (T <= 1) {
      run(0, epochs);
    } else {
      std::vector<std::thread> th;
      for (int k = 0; k < T; ++k) th.emplace_back([&, k] { run((int64_t)epochs * k / T, (int64_t)epochs * (k + 1) / T); });
      for (auto &t : th) t.join();
    }
  }
  torch_store(tr, torch_state);
  return AG_OK;
}
