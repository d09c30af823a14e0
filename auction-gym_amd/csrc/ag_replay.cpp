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
