/*
 * ag_oracle.c -- TEST INFRASTRUCTURE ONLY: CPU restatement of the reference hot path.
 *
 * This is the checker the HIP kernels are compared against (tests/, smoke(), and the
 * cpu_baseline leg of bench.py). It is pinned against the golden vectors captured
 * from the reference itself (tests/golden/, tests/test_oracle_golden.py).
 *
 * Compiled with -ffp-contract=off: every fused multiply-add below is an explicit fma()
 * because the reference's BLAS fuses exactly there (SURVEY §8 a5').
 */
#include "ag_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* src/Models.py:10-12: 1.0 / (1.0 + np.exp(-x)); exp is libm's (pinned numba 0.55.1
 * lowers np.exp to the libm call; requirements.txt:7). */
double ora_sigmoid(double z) { return 1.0 / (1.0 + exp(-z)); }

/* src/BidderAllocation.py:81-82 `self.item_embeddings @ context` and
 * src/Auction.py:52 `true_context @ items.T`: numpy -> OpenBLAS dgemv_t. Its kernel
 * takes the rows in blocks of four, one FMA accumulator per lane, then reduces the
 * lanes as (l0 + l2) + (l1 + l3); the 1-3 leftover rows are added by scalar C code
 * that the compiler contracted into FMAs. Verified bit-exact against numpy here for
 * D <= 7 at any K >= 2 and for every D when K % 4 == 0 (the shipped D = 6, K = 12
 * included); other shapes: parity unpinned (different OpenBLAS column kernels). */
double ora_dot(const double *a, const double *x, int32_t D) {
  int32_t m3 = D & 3, m1 = D - m3;
  double y = 0.0;
  if (m1 > 0) {
    double l0 = 0.0, l1 = 0.0, l2 = 0.0, l3 = 0.0;
    for (int32_t i = 0; i < m1; i += 4) {
      l0 = fma(a[i + 0], x[i + 0], l0);
      l1 = fma(a[i + 1], x[i + 1], l1);
      l2 = fma(a[i + 2], x[i + 2], l2);
      l3 = fma(a[i + 3], x[i + 3], l3);
    }
    y = (l0 + l2) + (l1 + l3);
  }
  const double *at = a + m1, *xt = x + m1;
  if (m3 == 1)
    y = fma(at[0], xt[0], y);
  else if (m3 == 2)
    y = y + fma(at[0], xt[0], at[1] * xt[1]);
  else if (m3 == 3)
    y = y + fma(at[2], xt[2], fma(at[0], xt[0], at[1] * xt[1]));
  return y;
}

/* src/Auction.py:65 rng.binomial(1, p) with numpy's inversion sampler for n = 1:
 * p <= 0.5: X = [U > exp(log(1 - p))];  p > 0.5: X = 1 - [U > exp(log(p))]
 * (numpy random_binomial / random_binomial_inversion; p == 0 draws nothing). */
int32_t ora_bernoulli(double p, double u) {
  if (p == 0.0) return 0;
  if (p <= 0.5) {
    double qn = exp(log(1.0 - p));
    return u > qn ? 1 : 0;
  }
  double q = 1.0 - p;
  double qn = exp(log(1.0 - q));
  return u > qn ? 0 : 1;
}

/* src/AuctionAllocation.py:19-23 (FirstPrice) and :32-34 (SecondPrice) for num_slots = 1:
 * winner = argsort(-bids)[0]; sorted = -sort(-bids); FP: price = sorted[0],
 * second = sorted[1]; SP: price = second = sorted[1]. Ties: lowest slot (numpy <= 1.22
 * insertion sort; SURVEY §8 a13'). Absent prices (P == 1) are NaN. */
static void top2(const double *b, int32_t P, int32_t *w, double *v1, double *v2) {
  int32_t wi = 0;
  double m1 = b[0], m2 = -INFINITY;
  for (int32_t s = 1; s < P; ++s) {
    double x = b[s];
    if (x > m1) {
      m2 = m1;
      m1 = x;
      wi = s;
    } else if (x > m2) {
      m2 = x;
    }
  }
  *w = wi;
  *v1 = m1;
  *v2 = m2;
}

void ora_allocate(int32_t mech, const double *bids, int64_t B, int32_t P, int32_t *winner,
                  double *price, double *second_price) {
  for (int64_t r = 0; r < B; ++r) {
    int32_t w;
    double m1, m2;
    top2(bids + r * P, P, &w, &m1, &m2);
    winner[r] = w;
    if (P < 2) {
      price[r] = (mech == ORA_FIRST_PRICE) ? m1 : NAN;
      second_price[r] = NAN;
    } else {
      price[r] = (mech == ORA_FIRST_PRICE) ? m1 : m2;
      second_price[r] = m2;
    }
  }
}

/* Per-record term -> fixed point: round(x * 2^36) to nearest-even (include/auctiongym.h
 * AG_FX_*); terms with |x| >= 2^26 (or non-finite) are dropped, as on the device. */
int64_t ora_to_fx(double x) {
  if (!(fabs(x) < 0x1p26)) return 0;
  return (int64_t)nearbyint(x * 0x1p36);
}

static void add_limbs(int64_t *L, __int128 v) {
  /* multiplications, not shifts: the top limb of a negative sum is negative (a left shift of
   * a negative value is undefined; found by the UBSan build, tools/sanitize_oracle.sh) */
  __int128 t = (__int128)L[2] * ((__int128)1 << 84) + (__int128)L[1] * ((__int128)1 << 42) + (__int128)L[0] + v;
  const int64_t mask = ((int64_t)1 << 42) - 1;
  L[0] = (int64_t)(t & mask);
  t >>= 42;
  L[1] = (int64_t)(t & mask);
  t >>= 42;
  L[2] = (int64_t)t;
}

/* Agent.select_item (src/Agent.py:29-42) for an OracleAllocator agent: CTR for every
 * item, first argmax of CTR * value. The same loop gives the true CTRs of
 * src/Auction.py:52-53 (true context): *ctr_best = sigmoid of the argmax, *best_ev = max. */
static int32_t oracle_select(const double *items, const double *vals, int32_t K, int32_t D,
                             const double *x, double *ctr_best, double *best_ev) {
  int32_t best = 0;
  double best_s = 0.0, best_c = 0.0;
  for (int32_t k = 0; k < K; ++k) {
    double c = ora_sigmoid(ora_dot(items + (int64_t)k * D, x, D));
    double s = c * vals[k];
    if (k == 0 || s > best_s) {
      best = k;
      best_s = s;
      best_c = c;
    }
  }
  *ctr_best = best_c;
  *best_ev = best_s;
  return best;
}

/* PyTorchLogisticRegression.forward (src/Models.py:28-33) as torch runs it on the CPU for
 * one context (src/BidderAllocation.py:67-68): F.linear(x[Do], W[K][Do]) with a 1-D input
 * is one BLAS sgemv (MKL), then torch.sigmoid over the K logits.
 *  - logit of item k: products rounded separately; for Do = 5 (obs_embedding_size 4 plus
 *    the intercept, every shipped config) summed as the sgemv kernel does -- rows in whole
 *    blocks of 4 as (fma(w1, x1, w0 x0) + w3 x3) + (w4 x4 + w2 x2), the K % 4 remainder
 *    rows as w0 x0 + ((w4 x4 + w2 x2) + (w3 x3 + w1 x1)) (all of 10800 summation trees
 *    over the 5 terms searched against torch, these two equal it on every row; test:
 *    tests/test_oracle_golden.py::test_ts_forward_matches_torch). Other Do: summed in
 *    order (parity by tolerance there).
 *  - sigmoid: elements in whole 32-lane chunks take torch's vectorised path (SLEEF expf_u10,
 *    ora_torch_sigmoidf), the rest its scalar 1 / (1 + expf(-z)) with glibc's expf
 *    (K = 12 < 32: all scalar). */
float ora_ts_logit(const float *w, const float *x, int32_t Do, int32_t k, int32_t K) {
  if (Do == 5) {
    const float p0 = w[0] * x[0], p2 = w[2] * x[2], p3 = w[3] * x[3], p4 = w[4] * x[4];
    if (k < (K & ~3)) return (fmaf(w[1], x[1], p0) + p3) + (p4 + p2);
    const float p1 = w[1] * x[1];
    return p0 + ((p4 + p2) + (p3 + p1));
  }
  float z = w[0] * x[0];
  for (int32_t d = 1; d < Do; ++d) z = z + w[d] * x[d];
  return z;
}

float ora_ts_sigmoid(float z, int32_t k, int32_t K) {
  if (k < (K & ~31)) return ora_torch_sigmoidf(z);
  return 1.0f / (1.0f + expf(-z));
}

float ora_ts_ctr(const float *w, const float *x, int32_t Do, int32_t k, int32_t K) {
  return ora_ts_sigmoid(ora_ts_logit(w, x, Do, k, K), k, K);
}

/* Gaussian shading factor of an uninitialised shading bidder (src/Bidder.py:47-58,
 * :174-179, :351-356, :458-463): gamma = rng.normal(prev_gamma, sigma) (given raw);
 * EmpiricalShadedBidder clips it to [0, 1]; the others keep it and log the Gaussian
 * density as the propensity. */
static double shading_gamma(int32_t kind, double raw) {
  if (kind == ORA_BIDDER_EMPIRICAL) {
    double g = raw;
    if (g < 0.0) g = 0.0;
    if (g > 1.0) g = 1.0;
    return g;
  }
  return raw;
}

double ora_propensity(double prev_gamma, double sigma, double g) {
  double t = (prev_gamma - g) / sigma;
  return exp(-(t * t) / 2.0) / (sigma * sqrt(2.0 * 3.141592653589793));
}

static void simulate_range(const ora_pop *pp, const double *items, const double *values,
                           int64_t r0, int64_t r1, const ora_in *in, const ora_out *out,
                           double *cnt, __int128 *fx) {
  const int32_t P = pp->P, K = pp->K, E = pp->E, D = E + 1, OE = pp->OE, Do = OE + 1;
  double x[64];
  float xo[64];
  double bids[256];
  for (int64_t r = r0; r < r1; ++r) {
    /* src/Auction.py:33-36 true context = [draws, 1.0]; observed = [first OE, 1.0] */
    for (int32_t e = 0; e < E; ++e) x[e] = in->ctx[r * E + e];
    x[E] = 1.0;
    for (int32_t e = 0; e < OE; ++e) xo[e] = (float)x[e];
    xo[OE] = 1.0f;
    /* src/Auction.py:44-54 per participant, in slot order */
    for (int32_t s = 0; s < P; ++s) {
      const int64_t o = r * P + s;
      const int32_t a = in->part[o];
      const double *it_a = items + (int64_t)a * K * D;
      const double *v_a = values + (int64_t)a * K;
      double ctr_t, bev;
      const int32_t it_t = oracle_select(it_a, v_a, K, D, x, &ctr_t, &bev);
      int32_t it;
      double est, tru;
      if (pp->alloc_kind[a] == ORA_ALLOCATOR_ORACLE) {
        it = it_t;
        est = ctr_t;
        tru = ctr_t;
      } else { /* LR-TS: sampled CTRs pick the item, the MAP CTR of it is the estimate */
        /* the agent's own model: its Ka items (the sgemv block / remainder rows and the
         * sigmoid's chunks follow Ka, the tensor torch sees) */
        const int32_t Ka = pp->num_items ? pp->num_items[a] : K;
        const float *m = pp->ts_m + (int64_t)a * K * Do;
        const float *nz = in->ts_noise + o * K * Do;
        float w[64];
        double best_s = 0.0;
        it = 0;
        for (int32_t k = 0; k < Ka; ++k) {
          for (int32_t d = 0; d < Do; ++d) w[d] = m[k * Do + d] + (pp->ts_sample ? nz[k * Do + d] : 0.0f);
          const double sc = (double)ora_ts_ctr(w, xo, Do, k, Ka) * v_a[k];
          if (k == 0 || sc > best_s) {
            best_s = sc;
            it = k;
          }
        }
        est = (double)ora_ts_ctr(m + it * Do, xo, Do, it, Ka);
        tru = it == it_t ? ctr_t : ora_sigmoid(ora_dot(it_a + (int64_t)it * D, x, D));
      }
      const double v = v_a[it];
      double b = v * est; /* Bidder.bid: value * estimated CTR (src/Bidder.py:35,49,173,...) */
      double g = NAN, prop = NAN;
      const int32_t bk = pp->bid_kind[a];
      if (bk >= ORA_BIDDER_VALUE_LEARNING && pp->dr_init && pp->dr_init[a] == 1) { /* fitted policy */
        ora_policy_bid(pp->dr_state + (int64_t)a * 16 + 4, est, v, in->policy_eps[o], &g, &prop);
        b = b * g;
      } else if (bk == ORA_BIDDER_VALUE_LEARNING && pp->dr_init && pp->dr_init[a] == 2) { /* search */
        g = ora_search_gamma(pp->dr_state + (int64_t)a * 16, est, v, in->gamma_grid + (int64_t)o * 128, 1);
        prop = 1.0;
        b = b * g;
      } else if (bk != ORA_BIDDER_TRUTHFUL) {
        g = shading_gamma(bk, in->gamma_raw[o]);
        if (bk != ORA_BIDDER_EMPIRICAL) prop = ora_propensity(pp->prev_gamma[a], pp->gamma_sigma[a], g);
        b = b * g;
      }
      out->item[o] = it;
      out->value[o] = v;
      out->bid[o] = b;
      out->est_ctr[o] = est;
      out->true_ctr[o] = tru;
      out->best_ev[o] = bev;
      if (out->gamma) out->gamma[o] = g;
      if (out->propensity) out->propensity[o] = prop;
      bids[s] = b;
    }
    int32_t w;
    double m1, m2;
    top2(bids, P, &w, &m1, &m2);
    double pr, sp;
    int charged = P >= 2; /* P == 1: empty price arrays -> nobody charged (Auction.py:68) */
    if (pp->mech == ORA_FIRST_PRICE) {
      pr = m1;
      sp = m2;
    } else {
      pr = m2;
      sp = m2;
    }
    out->winner[r] = w;
    out->price[r] = charged ? pr : NAN;
    out->second_price[r] = charged ? sp : NAN;
    int32_t oc = ora_bernoulli(out->true_ctr[r * P + w], in->u[r]);
    out->outcome[r] = (uint8_t)oc;
    /* Agent.charge / set_price (src/Agent.py:70-77) and the metric getters
     * (src/Agent.py:96-118) per log record. */
    for (int32_t s = 0; s < P; ++s) {
      int64_t o = r * P + s;
      int32_t a = in->part[o];
      int won = charged && s == w;
      double lp = charged ? pr : 0.0;  /* logged price */
      double lsp = won ? sp : 0.0;     /* logged second price */
      const double *est_ctr = out->est_ctr, *true_ctr = out->true_ctr, *value = out->value;
      double tv = true_ctr[o] * value[o];
      double t[ORA_NUM_COUNTERS];
      memset(t, 0, sizeof t);
      if (won) {
        double last_value = value[o] * (double)oc;
        t[ORA_C_NET] = last_value - pr;
        t[ORA_C_GROSS] = last_value;
        t[ORA_C_N_WON] = 1.0;
        t[ORA_C_PAID] = pr;
        t[ORA_C_CTR_BIAS] = est_ctr[o] / true_ctr[o];
      }
      t[ORA_C_ALLOC_REGRET] = out->best_ev[o] - tv;
      t[ORA_C_EST_REGRET] = est_ctr[o] * value[o] - tv;
      t[ORA_C_OVERBID] = (lp - lsp) * (double)won;
      t[ORA_C_UNDERBID] = (lp - out->bid[o]) * (double)(!won) * (double)(lp < tv);
      double d = true_ctr[o] - est_ctr[o];
      t[ORA_C_CTR_SQERR] = d * d;
      t[ORA_C_BEST_EV] = out->best_ev[o];
      t[ORA_C_N_LOGS] = 1.0;
      double *C = cnt + (int64_t)a * ORA_NUM_COUNTERS;
      for (int c = 0; c < ORA_NUM_COUNTERS; ++c) C[c] += t[c];
      if (fx) {
        __int128 *F = fx + (int64_t)a * ORA_NUM_COUNTERS;
        for (int c = 0; c < ORA_NUM_COUNTERS; ++c) F[c] += ora_to_fx(t[c]);
        /* fixed-point NET is defined as GROSS - PAID (include/auctiongym.h) */
        F[ORA_C_NET] += -ora_to_fx(t[ORA_C_NET]) + ora_to_fx(t[ORA_C_GROSS]) - ora_to_fx(t[ORA_C_PAID]);
      }
    }
  }
}

void ora_simulate_pop(const ora_pop *pp, const double *items, const double *values, int64_t B,
                      const ora_in *in, const ora_out *out, double *counters, int64_t *counters_fx,
                      int32_t nthreads) {
  const int64_t NC = (int64_t)pp->N * ORA_NUM_COUNTERS;
  if (nthreads < 1) nthreads = 1;
  double *part_cnt = (double *)calloc((size_t)nthreads * NC, sizeof(double));
  __int128 *part_fx = (__int128 *)calloc((size_t)nthreads * NC, sizeof(__int128));
#pragma omp parallel num_threads(nthreads)
  {
#ifdef _OPENMP
    int t = omp_get_thread_num(), nt = omp_get_num_threads();
#else
    int t = 0, nt = 1;
#endif
    int64_t r0 = B * t / nt, r1 = B * (t + 1) / nt;
    simulate_range(pp, items, values, r0, r1, in, out, part_cnt + (int64_t)t * NC,
                   part_fx + (int64_t)t * NC);
  }
  for (int t = 0; t < nthreads; ++t)
    for (int64_t i = 0; i < NC; ++i) {
      counters[i] += part_cnt[(int64_t)t * NC + i];
      if (counters_fx) add_limbs(counters_fx + i * 3, part_fx[(int64_t)t * NC + i]);
    }
  free(part_cnt);
  free(part_fx);
}

void ora_simulate(const ora_shape *s, const double *items, const double *values, int64_t B,
                  const double *ctx, const int32_t *part, const double *u, int32_t *winner,
                  double *price, double *second_price, uint8_t *outcome, int32_t *item,
                  double *value, double *bid, double *est_ctr, double *true_ctr, double *best_ev,
                  double *counters, int64_t *counters_fx, int32_t nthreads) {
  int32_t *ak = (int32_t *)calloc((size_t)s->N, sizeof(int32_t));
  int32_t *bk = (int32_t *)calloc((size_t)s->N, sizeof(int32_t));
  ora_pop pp = {s->N, s->P, s->K, s->E, s->E, s->mech, ak, bk, NULL, NULL, NULL, 0, NULL, NULL, NULL};
  ora_in in = {ctx, part, u, NULL, NULL, NULL, NULL};
  ora_out out = {winner, price, second_price, outcome, item, value, bid, est_ctr, true_ctr,
                 best_ev, NULL, NULL};
  ora_simulate_pop(&pp, items, values, B, &in, &out, counters, counters_fx, nthreads);
  free(ak);
  free(bk);
}

/* ---- synthetic batch generator (integer part), restating ag_generate ---- */

void ora_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
  uint32_t k0 = key[0], k1 = key[1];
  for (int i = 0; i < 10; ++i) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    uint32_t n1 = (uint32_t)p1;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    uint32_t n3 = (uint32_t)p0;
    c0 = n0;
    c1 = n1;
    c2 = n2;
    c3 = n3;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  out[0] = c0;
  out[1] = c1;
  out[2] = c2;
  out[3] = c3;
}

static void block(uint64_t seed, uint64_t idx, uint32_t blk, uint32_t stream, uint32_t out[4]) {
  uint32_t ctr[4] = {(uint32_t)idx, (uint32_t)(idx >> 32), blk, stream};
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  ora_philox4x32_10(ctr, key, out);
}

double ora_gen_uniform(uint64_t seed, uint64_t idx) {
  uint32_t w[4];
  block(seed, idx, 0, 0, w);
  uint64_t v = ((uint64_t)w[0] << 32) | w[1];
  return (double)(v >> 11) * 0x1p-53;
}

/* Floyd's sampling of P distinct agents out of N; slot order = insertion order.
 * Step j (j = N-P .. N-1) draws t = floor(word * (j+1) / 2^32): steps 0 and 1 from words 2-3 of
 * stream 0's block 0 (the call whose words 0-1 make u), later steps from stream 1, four per
 * call (csrc/ag_philox.h gen_auction, round 5). */
void ora_gen_participants(uint64_t seed, uint64_t idx, int32_t N, int32_t P, int32_t *part_out) {
  uint32_t w0[4], w[4];
  int32_t n = 0;
  block(seed, idx, 0, 0, w0);
  for (int32_t j = N - P; j < N; ++j) {
    int32_t step = j - (N - P);
    uint32_t word;
    if (step < 2) {
      word = w0[2 + step];
    } else {
      if (((step - 2) & 3) == 0) block(seed, idx, (uint32_t)((step - 2) >> 2), 1, w);
      word = w[(step - 2) & 3];
    }
    uint32_t t = (uint32_t)(((uint64_t)word * (uint64_t)(j + 1)) >> 32);
    int32_t pick = (int32_t)t;
    for (int32_t q = 0; q < n; ++q)
      if (part_out[q] == pick) {
        pick = j;
        break;
      }
    part_out[n++] = pick;
  }
}

/* ---------------------------------------------------------------------------------------
 * LR-TS allocator update (PyTorchLogisticRegressionAllocator.update,
 * src/BidderAllocation.py:29-65; model src/Models.py:35-48), restated with exact sums.
 *
 * Per epoch (src/BidderAllocation.py:44-55): forward on every won sample, loss = prior +
 * BCE (sum), backward, Adam(lr 2e-3) step, ReduceLROnPlateau('min', factor 0.5) on the
 * loss, early stop when epoch > 1024 and |loss[-100] - loss[-1]| < 1e-6. Then the Laplace
 * update of q per item (:58-61, src/Models.py:43-45) and prev_m = m (:62).
 *
 * Arithmetic (the definition the device kernel follows bit for bit):
 *  - z = x . m[a] in float32, products rounded separately, summed in order; p = 1 / (1 + (float)exp(-(double)z)) in float32.
 *  - BCE term (torch.nn.BCELoss, logs clamped at -100) in double: y ? -max(log p, -100)
 *    : -max(log1p(-p), -100); gradient term (p - y) * x_d, exact in double.
 *  - Sums over samples are EXACT: every term is rounded to a fixed-point grid (BCE 2^-32,
 *    gradient and Laplace 2^-40) and added as integers, so no summation order exists;
 *    a sum S is read back as (double)(S >> 24) * 2^24 + (double)(S & (2^24-1)).
 *  - prior loss 0.5 * sum q (pm - m)^2 and its gradient -q (pm - m) in double (row-major
 *    order); gradient and loss are rounded to float32 once.
 *  - Adam (torch.optim.Adam defaults, single-tensor CPU path) in float32:
 *    ea += 0.1f * (g - ea); es = es * 0.999f + (0.001f * g) * g;
 *    m += (float)(-lr / bc1) * (ea / (sqrtf(es) / (float)pow(bc2, 0.5) + 1e-8f)),
 *    bc1 = 1 - pow(0.9, t), bc2 = 1 - pow(0.999, t) in double (Python floats).
 *  - Laplace: P = 1 / (1 + (float)exp((double)(1 - z))) with z as above (float32),
 *    q[k][d] += (float)sum P (1 - P) x_d^2 (products float32, sum exact).
 * torch sums in float32 in its own order: the reference agrees to float32 rounding per
 * epoch (tests/test_oracle_golden.py pins loss0 / grad0 and the trajectory).
 * ------------------------------------------------------------------------------------- */
#define ORA_LR_EPOCHS 16384

static int64_t fx_round(double v, double scale) { return (int64_t)nearbyint(v * scale); }

/* ---- record-parallel hook (ag_oracle.h ora_set_reduce): exact sums over the ranks ---- */
static ora_reduce_fn g_reduce = NULL;
static int64_t g_n_total = 0;
void ora_set_reduce(ora_reduce_fn fn, int64_t n_total) {
  g_reduce = fn;
  g_n_total = n_total;
}
int ora_reducing(void) { return g_reduce != NULL; }
/* records of the fit over all ranks (the means' denominators, the reference's checks) */
int64_t ora_total(int64_t n) { return g_reduce && g_n_total > 0 ? g_n_total : n; }
/* s[0..k) summed over the ranks, exactly (32-bit halves as int64 words: no overflow) */
void ora_reduce128(__int128 *s, int32_t k) {
  if (!g_reduce || k <= 0) return;
  int64_t *w = malloc(sizeof(int64_t) * 2 * (size_t)k);
  for (int32_t j = 0; j < k; ++j) {
    w[2 * j] = (int64_t)(s[j] >> 32);
    w[2 * j + 1] = (int64_t)(s[j] & 0xffffffff);
  }
  g_reduce(w, 2 * k);
  for (int32_t j = 0; j < k; ++j) s[j] = ((__int128)w[2 * j] << 32) + (__int128)w[2 * j + 1];
  free(w);
}

static double fx_read(__int128 s, double inv_scale) {
  /* the device holds these sums split at bit 24; same read-back */
  int64_t hi = (int64_t)(s >> 24), lo = (int64_t)(s & 0xFFFFFF);
  return ((double)hi * 0x1p24 + (double)lo) * inv_scale;
}

/* One epoch's loss (loss.item()) and float32 gradient g [K][Do] at m. */
static float lrts_loss_grad(int64_t n, int32_t K, int32_t Do, const float *X, const int32_t *A,
                            const uint8_t *y, const float *m, const float *pm, const float *q,
                            __int128 *G, float *g) {
  const int32_t KD = K * Do;
  __int128 L = 0;
  for (int32_t c = 0; c < KD; ++c) G[c] = 0;
  for (int64_t i = 0; i < n; ++i) {
    const float *x = X + i * Do, *w = m + (int64_t)A[i] * Do;
    float z = w[0] * x[0];
    for (int32_t d = 1; d < Do; ++d) z = z + w[d] * x[d];
    float p = 1.0f / (1.0f + (float)exp(-(double)z));
    double t = y[i] ? -fmax(log((double)p), -100.0) : -fmax(log1p(-(double)p), -100.0);
    L += fx_round(t, 0x1p32);
    double gz = (double)p - (double)y[i];
    for (int32_t d = 0; d < Do; ++d) G[A[i] * Do + d] += fx_round(gz * (double)x[d], 0x1p40);
  }
  if (ora_reducing()) { /* one exchange of the KD gradient sums and the loss */
    __int128 *t = malloc(sizeof(__int128) * (size_t)(KD + 1));
    for (int32_t c = 0; c < KD; ++c) t[c] = G[c];
    t[KD] = L;
    ora_reduce128(t, KD + 1);
    for (int32_t c = 0; c < KD; ++c) G[c] = t[c];
    L = t[KD];
    free(t);
  }
  double prior = 0.0;
  for (int32_t k = 0; k < K; ++k)
    for (int32_t d = 0; d < Do - 1; ++d) {
      double df = (double)pm[k * Do + d] - (double)m[k * Do + d];
      prior += (double)q[k * Do + d] * (df * df);
    }
  for (int32_t c = 0; c < KD; ++c) {
    double gp = (c % Do) < Do - 1 ? -(double)q[c] * ((double)pm[c] - (double)m[c]) : 0.0;
    g[c] = (float)(fx_read(G[c], 0x1p-40) + gp);
  }
  return (float)(0.5 * prior + fx_read(L, 0x1p-32));
}

float ora_lrts_loss_grad(int64_t n, int32_t K, int32_t Do, const float *X, const int32_t *A,
                         const uint8_t *y, const float *m, const float *pm, const float *q, float *g) {
  __int128 *G = malloc((size_t)K * Do * sizeof(__int128));
  float loss = lrts_loss_grad(n, K, Do, X, A, y, m, pm, q, G, g);
  free(G);
  return loss;
}

int32_t ora_lrts_update(int64_t n, int32_t K, int32_t Do, const float *X, const int32_t *A,
                        const uint8_t *y, float *m, float *pm, float *q, float *loss_trace) {
  if (ora_total(n) < 2) return 0;
  const int32_t KD = K * Do;
  float *ea = calloc(KD, sizeof(float)), *es = calloc(KD, sizeof(float)), *g = malloc(KD * sizeof(float));
  __int128 *G = malloc(KD * sizeof(__int128));
  double lr = 2e-3, best = INFINITY;
  int32_t bad = 0, epoch = 0;
  float hist[100];
  for (epoch = 0; epoch < ORA_LR_EPOCHS; ++epoch) {
    float loss = lrts_loss_grad(n, K, Do, X, A, y, m, pm, q, G, g);
    const double step = (double)(epoch + 1);
    const double bc1 = 1.0 - pow(0.9, step), bc2s = pow(1.0 - pow(0.999, step), 0.5);
    const float neg_step = (float)(-(lr / bc1)), bc2f = (float)bc2s;
    for (int32_t c = 0; c < KD; ++c) {
      ea[c] = ea[c] + 0.1f * (g[c] - ea[c]);
      es[c] = es[c] * 0.999f + (0.001f * g[c]) * g[c];
      float den = sqrtf(es[c]) / bc2f + 1e-8f;
      m[c] = m[c] + neg_step * (ea[c] / den);
    }
    if (loss_trace) loss_trace[epoch] = loss;
    hist[epoch % 100] = loss;
    /* ReduceLROnPlateau(mode min, threshold 1e-4 rel, patience 10, factor 0.5, eps 1e-8) */
    if ((double)loss < best * (1.0 - 1e-4)) {
      best = (double)loss;
      bad = 0;
    } else {
      ++bad;
    }
    if (bad > 10) {
      double nl = lr * 0.5;
      if (lr - nl > 1e-8) lr = nl;
      bad = 0;
    }
    if (epoch > 1024 && fabs((double)hist[(epoch - 99) % 100] - (double)loss) < 1e-6) {
      ++epoch;
      break;
    }
  }
  /* Laplace approximation of q per item, then the prior update */
  for (int32_t c = 0; c < KD; ++c) G[c] = 0;
  for (int64_t i = 0; i < n; ++i) {
    const float *x = X + i * Do, *w = m + (int64_t)A[i] * Do;
    float z = w[0] * x[0];
    for (int32_t d = 1; d < Do; ++d) z = z + w[d] * x[d];
    float P = 1.0f / (1.0f + (float)exp((double)(1.0f - z)));
    float wgt = P * (1.0f - P);
    for (int32_t d = 0; d < Do; ++d) G[A[i] * Do + d] += fx_round((double)wgt * (double)(x[d] * x[d]), 0x1p40);
  }
  ora_reduce128(G, KD);
  for (int32_t c = 0; c < KD; ++c) {
    q[c] = q[c] + (float)fx_read(G[c], 0x1p-40);
    pm[c] = m[c];
  }
  free(ea);
  free(es);
  free(g);
  free(G);
  return epoch;
}

/* ---------------------------------------------------------------------------------------
 * EmpiricalShadedBidder.update (src/Bidder.py:60-147): bucketise the iteration's shading
 * factors on a 0.005 grid, lower confidence bound of the mean net utility per bucket,
 * move prev_gamma to the best bucket's midpoint.
 *  - num_buckets = int((max - min) // 0.005) + 1 with Python's float floor division,
 *    edges = numpy.linspace(min, max, num_buckets): i * step + min, last = max;
 *  - bucket j holds edge_j <= gamma < edge_{j+1} (the maximum itself falls in none);
 *  - buckets with > 1 sample: mean = S / n, stderr = sqrt(S2 / n) / sqrt(n) with S, S2
 *    exact fixed-point sums (2^-40 grid) of u and (u - mean)^2; U = mean - 1.96 stderr;
 *  - best = the LAST bucket with the largest U (the reference's reversed nanargmax);
 *    prev_gamma = clip(midpoint (hi - lo) / 2 + lo, 0, 1).
 * numpy sums pairwise in float64: means agree to ~1e-16 relative, so the chosen bucket
 * (and prev_gamma, computed from the same edges) is identical unless two buckets' bounds
 * tie within that (tests/test_oracle_golden.py: every case of empirical_update_kat.npz).
 * Returns 0, or the reference's exception: -1 empty logs (np.min of an empty array),
 * -2 no bucket (argmax of an empty sequence), -3 all buckets NaN (All-NaN slice).
 * ------------------------------------------------------------------------------------- */
static double py_floordiv(double vx, double wx) { /* CPython float floor division */
  double mod = fmod(vx, wx);
  double div = (vx - mod) / wx;
  if (mod != 0.0) {
    if ((wx < 0) != (mod < 0)) div -= 1.0;
  }
  double fd;
  if (div != 0.0) {
    fd = floor(div);
    if (div - fd > 0.5) fd += 1.0;
  } else {
    fd = copysign(0.0, vx / wx);
  }
  return fd;
}

int32_t ora_empirical_update(int64_t n, const double *gamma, const double *util, double *prev_gamma) {
  if (n < 1) return -1;
  double lo_g = gamma[0], hi_g = gamma[0];
  for (int64_t i = 1; i < n; ++i) {
    if (gamma[i] < lo_g) lo_g = gamma[i];
    if (gamma[i] > hi_g) hi_g = gamma[i];
  }
  const int64_t nb = (int64_t)py_floordiv(hi_g - lo_g, 0.005) + 1;
  if (nb < 2) return -2;
  const double step = (hi_g - lo_g) / (double)(nb - 1);
  double *edge = malloc(nb * sizeof(double));
  for (int64_t j = 0; j < nb - 1; ++j) edge[j] = (double)j * step + lo_g;
  edge[nb - 1] = hi_g;
  const int64_t M = nb - 1;
  int64_t *cnt = calloc(M, sizeof(int64_t));
  __int128 *S = calloc(M, sizeof(__int128)), *S2 = calloc(M, sizeof(__int128));
  int64_t *bk = malloc(n * sizeof(int64_t));
  for (int64_t i = 0; i < n; ++i) {
    int64_t j = -1;
    for (int64_t b = 0; b < M; ++b)
      if (edge[b] <= gamma[i] && gamma[i] < edge[b + 1]) { j = b; break; }
    bk[i] = j;
    if (j >= 0) {
      cnt[j] += 1;
      S[j] += fx_round(util[i], 0x1p40);
    }
  }
  double *mean = malloc(M * sizeof(double));
  for (int64_t b = 0; b < M; ++b) mean[b] = cnt[b] > 1 ? fx_read(S[b], 0x1p-40) / (double)cnt[b] : 0.0;
  for (int64_t i = 0; i < n; ++i)
    if (bk[i] >= 0 && cnt[bk[i]] > 1) {
      double d = util[i] - mean[bk[i]];
      S2[bk[i]] += fx_round(d * d, 0x1p40);
    }
  int64_t best = -1;
  double bestU = 0.0;
  for (int64_t b = 0; b < M; ++b) {
    if (cnt[b] <= 1) continue;
    double se = sqrt(fx_read(S2[b], 0x1p-40) / (double)cnt[b]) / sqrt((double)cnt[b]);
    double U = mean[b] - 1.96 * se;
    if (best < 0 || U >= bestU) {
      best = b;
      bestU = U;
    }
  }
  int32_t rc = 0;
  if (best < 0) {
    rc = -3;
  } else {
    double g = (edge[best + 1] - edge[best]) / 2.0 + edge[best];
    if (g < 0) g = 0;
    if (g > 1.0) g = 1.0;
    *prev_gamma = g;
  }
  free(edge);
  free(cnt);
  free(S);
  free(S2);
  free(bk);
  free(mean);
  return rc;
}
