/*
 * ag_oracle_dr.c -- TEST INFRASTRUCTURE ONLY (part of the oracle, see ag_oracle.h).
 *
 * CPU restatement of DoublyRobustBidder.update (src/Bidder.py:473-615) with its models
 * (src/Models.py:51-62 PyTorchWinRateEstimator, :92-218 BidShadingContextualBandit):
 *   1. win-rate fit: sigmoid(w . [ctr, value, gamma] + b) by BCE (mean) on the logs plus
 *      the "shade 100% -> lose" augmentation (gamma = 0, y = 0) (:500-514), Adam(lr 3e-3,
 *      weight decay 1e-6, AMSGrad), ReduceLROnPlateau(patience 256, factor 0.2, min_lr
 *      1e-7), early stop after 1024 epochs without a 1e-6 improvement, <= 32768 epochs;
 *   2. estimated utilities W (V - P) of the logged bids with the fitted model (:541-546);
 *   3. first update only: imitation of the logging policy (src/Models.py:106-137): MSE of
 *      mu to the logged gammas + MSE of sigma to 0.05, Adam(lr 1e-3, wd 1e-4, AMSGrad),
 *      early stop after 512 epochs, <= 16384 epochs;
 *   4. DR policy fit (:562-590, src/Models.py:201-218): loss -mean((u - u_hat) clip(pi/pi0,
 *      1/50, 50) + W(ctr, value, clip(mu + sigma eps, 0, 1)) (V - P)), eps the per-epoch
 *      rsample noise (given), Adam(lr 7e-3, wd 1e-4, AMSGrad), ReduceLROnPlateau(patience
 *      100, factor 0.2, min_lr 1e-8, threshold 5e-3), early stop after 512, <= 32768.
 *
 * Arithmetic (the definition the device kernel follows bit for bit): parameters and their
 * Adam state in float32 with torch's single-tensor update (weight decay added to the
 * gradient, AMSGrad max of the second moments); per-sample forward / backward in double
 * from the float32 features and parameters, exp from libm (glibc; the device uses its
 * glibc-identical restatement), log1p inside softplus from the fdlibm algorithm restated
 * below (so host and device agree bit for bit); sums over samples EXACT (terms on a 2^-40
 * grid, added as integers) and divided by the sample count once. torch computes all of
 * this in float32 in its own order, so trajectories agree to float32 rounding per epoch
 * and drift apart chaotically late in long fits (tests pin loss0 / gradients and the
 * trajectories within measured tolerances).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "ag_oracle.h"

/* fdlibm log1p (public-domain algorithm: reduction to 1+f in [sqrt(2)/2, sqrt(2)),
 * s = f/(2+f), odd minimax polynomial in s, correction term c), restated. */
static double fl_log1p(double x) {
  static const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
                      Lp1 = 6.666666666666735130e-01, Lp2 = 3.999999999940941908e-01,
                      Lp3 = 2.857142874366239149e-01, Lp4 = 2.222219843214978396e-01,
                      Lp5 = 1.818357216161805012e-01, Lp6 = 1.531383769920937332e-01,
                      Lp7 = 1.479819860511658591e-01;
  uint64_t bits;
  memcpy(&bits, &x, 8);
  int32_t hx = (int32_t)(bits >> 32), ax = hx & 0x7fffffff, hu = 0, k = 1;
  double f = 0.0, c = 0.0;
  if (hx < 0x3FDA827A) {                    /* 1 + x < sqrt(2)+ */
    if (ax >= 0x3ff00000) return x == -1.0 ? -INFINITY : NAN;
    if (ax < 0x3e200000) {                  /* |x| < 2^-29 */
      if (ax < 0x3c900000) return x;
      return x - x * x * 0.5;
    }
    if (hx > 0 || hx <= (int32_t)0xbfd2bec4) { /* sqrt(2)/2- <= 1 + x < sqrt(2)+ */
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
      uint64_t ub;
      memcpy(&ub, &u, 8);
      hu = (int32_t)(ub >> 32);
      k = (hu >> 20) - 1023;
      c = (k > 0) ? 1.0 - (u - x) : x - (u - 1.0);
      c /= u;
    } else {
      u = x;
      uint64_t ub;
      memcpy(&ub, &u, 8);
      hu = (int32_t)(ub >> 32);
      k = (hu >> 20) - 1023;
      c = 0;
    }
    hu &= 0x000fffff;
    uint64_t ub;
    memcpy(&ub, &u, 8);
    if (hu < 0x6a09e) {
      ub = ((uint64_t)(uint32_t)(hu | 0x3ff00000) << 32) | (ub & 0xffffffffull);
    } else {
      k += 1;
      ub = ((uint64_t)(uint32_t)(hu | 0x3fe00000) << 32) | (ub & 0xffffffffull);
      hu = (0x00100000 - hu) >> 2;
    }
    memcpy(&u, &ub, 8);
    f = u - 1.0;
  }
  const double hfsq = 0.5 * f * f;
  if (hu == 0) { /* |f| < 2^-20 */
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

double ora_log1p_restated(double x) { return fl_log1p(x); }

/* torch.nn.Softplus (beta 1, threshold 20) and its derivative */
static double softplus(double u) { return u > 20.0 ? u : fl_log1p(exp(u)); }
static double dsoftplus(double u) {
  if (u > 20.0) return 1.0;
  const double e = exp(u);
  return e / (e + 1.0);
}

/* the record-parallel hook (ag_oracle.c): sums over the ranks, records over the ranks */
int64_t ora_total(int64_t n);
void ora_reduce128(__int128 *s, int32_t k);

#define DR_GRID 0x1p40
#define DR_INV 0x1p-40

static int64_t fxr(double v) { return (int64_t)nearbyint(v * DR_GRID); }
static double fxv(__int128 s) {
  int64_t hi = (int64_t)(s >> 24), lo = (int64_t)(s & 0xFFFFFF);
  return ((double)hi * 0x1p24 + (double)lo) * DR_INV;
}

/* torch.optim.Adam, single-tensor CPU path, weight decay, AMSGrad (tensors < 16 elements:
 * the scalar loops, no fused multiply-adds) */
typedef struct {
  int32_t np;
  float ea[16], es[16], mx[16];
  double lr, wd;
  int64_t step;
} adam_t;

static void adam_init(adam_t *a, int32_t np, double lr, double wd) {
  memset(a, 0, sizeof *a);
  a->np = np;
  a->lr = lr;
  a->wd = wd;
}

static void adam_step(adam_t *a, float *p, const float *grad) {
  a->step += 1;
  const double t = (double)a->step;
  const double bc1 = 1.0 - pow(0.9, t), bc2s = pow(1.0 - pow(0.999, t), 0.5);
  const float neg_step = (float)(-(a->lr / bc1)), bc2f = (float)bc2s, wdf = (float)a->wd;
  for (int32_t j = 0; j < a->np; ++j) {
    const float g = grad[j] + wdf * p[j];
    a->ea[j] = a->ea[j] + 0.1f * (g - a->ea[j]);
    a->es[j] = a->es[j] * 0.999f + (0.001f * g) * g;
    a->mx[j] = a->mx[j] > a->es[j] ? a->mx[j] : a->es[j];
    const float den = sqrtf(a->mx[j]) / bc2f + 1e-8f;
    p[j] = p[j] + neg_step * (a->ea[j] / den);
  }
}

/* torch.optim.lr_scheduler.ReduceLROnPlateau, mode 'min', threshold_mode 'rel' */
typedef struct {
  double best, threshold, factor, min_lr;
  int32_t bad, patience;
} plateau_t;

static void plateau_init(plateau_t *s, int32_t patience, double factor, double min_lr, double threshold) {
  s->best = INFINITY;
  s->bad = 0;
  s->patience = patience;
  s->factor = factor;
  s->min_lr = min_lr;
  s->threshold = threshold;
}

static void plateau_step(plateau_t *s, float loss, double *lr) {
  if ((double)loss < s->best * (1.0 - s->threshold)) {
    s->best = (double)loss;
    s->bad = 0;
  } else {
    s->bad += 1;
  }
  if (s->bad > s->patience) {
    double nl = *lr * s->factor;
    if (nl < s->min_lr) nl = s->min_lr;
    if (*lr - nl > 1e-8) *lr = nl;
    s->bad = 0;
  }
}

/* the reference's early stop: (best - loss) > 1e-6 resets; stop when epoch - best > wait */
typedef struct {
  double best;
  int32_t best_epoch, wait;
} stopper_t;

static int stop_step(stopper_t *s, int32_t epoch, float loss) {
  if (s->best - (double)loss > 1e-6) {
    s->best_epoch = epoch;
    s->best = (double)loss;
    return 0;
  }
  return epoch - s->best_epoch > s->wait;
}

/* win-rate model W(x) = sigmoid(w0 c + w1 v + w2 g + b) */
static double winrate(const float *wr, double c, double v, double g) {
  const double z = c * (double)wr[0] + v * (double)wr[1] + g * (double)wr[2] + (double)wr[3];
  return 1.0 / (1.0 + exp(-z));
}

/* policy forward: p = [W1 (2x2 row-major), b1 (2), wm (2), bm, ws (2), bs] (the order of
 * BidShadingContextualBandit.parameters()) */
typedef struct {
  double h[2], s[2], am, as, mu, sp_sigma, sigma;
} polf_t;

static void policy_fwd(const float *p, double c, double v, polf_t *f) {
  for (int j = 0; j < 2; ++j) {
    f->h[j] = c * (double)p[2 * j] + v * (double)p[2 * j + 1] + (double)p[4 + j];
    f->s[j] = softplus(f->h[j]);
  }
  f->am = f->s[0] * (double)p[6] + f->s[1] * (double)p[7] + (double)p[8];
  f->as = f->s[0] * (double)p[9] + f->s[1] * (double)p[10] + (double)p[11];
  f->mu = softplus(f->am);
  f->sp_sigma = softplus(f->as);
  f->sigma = f->sp_sigma + 0.01;  /* min_sigma (src/Models.py:104) */
}

/* d(loss_i)/d(params) from d/dmu and d/dsigma of one sample, accumulated as fixed point */
static void policy_bwd(const float *p, double c, double v, const polf_t *f, double dmu, double dsigma,
                       __int128 *G) {
  const double dam = dmu * dsoftplus(f->am), das = dsigma * dsoftplus(f->as);
  double ds[2];
  ds[0] = dam * (double)p[6] + das * (double)p[9];
  ds[1] = dam * (double)p[7] + das * (double)p[10];
  G[6] += fxr(dam * f->s[0]);
  G[7] += fxr(dam * f->s[1]);
  G[8] += fxr(dam);
  G[9] += fxr(das * f->s[0]);
  G[10] += fxr(das * f->s[1]);
  G[11] += fxr(das);
  for (int j = 0; j < 2; ++j) {
    const double dh = ds[j] * dsoftplus(f->h[j]);
    G[2 * j] += fxr(dh * c);
    G[2 * j + 1] += fxr(dh * v);
    G[4 + j] += fxr(dh);
  }
}

/* PyTorchWinRateEstimator fit (src/Bidder.py:229-252 ValueLearningBidder, :500-530
 * DoublyRobustBidder): BCE (mean) over the logs plus the gamma = 0, y = 0 augmentation,
 * Adam(lr 3e-3, weight decay 1e-6, AMSGrad), ReduceLROnPlateau(patience, factor, min_lr
 * 1e-7), early stop after `wait` epochs without a 1e-6 improvement, <= 32768 epochs. */
static int32_t fit_winrate(int64_t n, const float *cf, const float *vf, const float *gf, const uint8_t *won,
                           float *wr, int32_t patience, double factor, int32_t wait, float *trace) {
  const double M = 2.0 * (double)ora_total(n);
  adam_t ad;
  adam_init(&ad, 4, 3e-3, 1e-6);
  plateau_t pl;
  plateau_init(&pl, patience, factor, 1e-7, 1e-4);
  stopper_t st = {INFINITY, -1, wait};
  int32_t e = 0;
  for (; e < 32768; ++e) {
    __int128 L = 0, G[4] = {0, 0, 0, 0};
    for (int64_t r = 0; r < 2 * n; ++r) {
      const int64_t i = r < n ? r : r - n;
      const double c = cf[i], v = vf[i], g = r < n ? gf[i] : 0.0;
      const double y = r < n ? (double)won[i] : 0.0;
      const double z = c * (double)wr[0] + v * (double)wr[1] + g * (double)wr[2] + (double)wr[3];
      /* one exp per row: e = exp(-|z|), L = log1p(e) (the restated log1p: the same bits on
       * the device); p = sigmoid(z) = (z >= 0 ? 1 : e) / (1 + e); BCE with torch's clamp of
       * the logs at -100: -log(p) = softplus(-z), -log(1-p) = softplus(z), where softplus(u)
       * = u past torch's threshold 20, L for u <= 0 and |z| + L for u > 0 */
      const double a = fabs(z), e = exp(-a), Lz = fl_log1p(e);
      const double pw = (z >= 0.0 ? 1.0 : e) / (1.0 + e);
      const double u = y > 0.0 ? -z : z;
      const double t = fmin(u > 20.0 ? u : (u > 0.0 ? a + Lz : Lz), 100.0);
      L += fxr(t);
      const double gz = pw - y;
      G[0] += fxr(gz * c);
      G[1] += fxr(gz * v);
      G[2] += fxr(gz * g);
      G[3] += fxr(gz);
    }
    {
      __int128 t[5] = {L, G[0], G[1], G[2], G[3]};
      ora_reduce128(t, 5);
      L = t[0];
      for (int j = 0; j < 4; ++j) G[j] = t[1 + j];
    }
    const float loss = (float)(fxv(L) / M);
    float grad[4];
    for (int j = 0; j < 4; ++j) grad[j] = (float)(fxv(G[j]) / M);
    adam_step(&ad, wr, grad);
    if (trace) trace[e] = loss;
    plateau_step(&pl, loss, &ad.lr);
    if (stop_step(&st, e, loss)) {
      ++e;
      break;
    }
  }
  return e;
}

/* BidShadingContextualBandit.initialise_policy (src/Models.py:106-137): imitation of the
 * logging policy -- MSE of mu to the logged gammas + MSE of softplus(sigma) (WITHOUT
 * min_sigma, :118) to 0.05, Adam(lr 1e-3, wd 1e-4, AMSGrad), no scheduler, early stop
 * after 512 epochs, <= 16384 epochs. */
static int32_t fit_imitation(int64_t n, const float *cf, const float *vf, const float *gf, float *pol,
                             float *trace) {
  adam_t ad;
  adam_init(&ad, 12, 1e-3, 1e-4);
  stopper_t st = {INFINITY, -1, 512};
  int32_t e = 0;
  for (; e < 16384; ++e) {
    __int128 L1 = 0, L2 = 0, G[12];
    memset(G, 0, sizeof G);
    for (int64_t i = 0; i < n; ++i) {
      polf_t f;
      policy_fwd(pol, cf[i], vf[i], &f);
      const double dm = f.mu - (double)gf[i], dsg = f.sp_sigma - 0.05;
      L1 += fxr(dm * dm);
      L2 += fxr(dsg * dsg);
      policy_bwd(pol, cf[i], vf[i], &f, 2.0 * dm, 2.0 * dsg, G);
    }
    {
      __int128 t[14];
      t[0] = L1;
      t[1] = L2;
      for (int j = 0; j < 12; ++j) t[2 + j] = G[j];
      ora_reduce128(t, 14);
      L1 = t[0];
      L2 = t[1];
      for (int j = 0; j < 12; ++j) G[j] = t[2 + j];
    }
    const double nt = (double)ora_total(n);
    const float loss = (float)(fxv(L1) / nt + fxv(L2) / nt);
    float grad[12];
    for (int j = 0; j < 12; ++j) grad[j] = (float)(fxv(G[j]) / nt);
    adam_step(&ad, pol, grad);
    if (trace) trace[e] = loss;
    if (stop_step(&st, e, loss)) {
      ++e;
      break;
    }
  }
  return e;
}

int32_t ora_dr_update(int64_t n, const double *ctr, const double *value, const double *gamma,
                      const double *prop, const uint8_t *won, const double *util, float *wr, float *pol,
                      int32_t initialised, const float *noise, int64_t noise_epochs, int32_t *epochs,
                      float *wr_trace, float *init_trace, float *dr_trace, double *est_util_out) {
  if (ora_total(n) < 1) return -1;
  float *cf = malloc(n * sizeof(float)), *vf = malloc(n * sizeof(float)), *gf = malloc(n * sizeof(float));
  double *eu = malloc(n * sizeof(double));
  for (int64_t i = 0; i < n; ++i) {
    cf[i] = (float)ctr[i];
    vf[i] = (float)value[i];
    gf[i] = (float)gamma[i];
  }
  /* ---- 1. win-rate fit (initialised bit 1, a test hook: skipped, wr is taken as already
   * fitted -- to run the later fits from the reference's own fitted model) */
  epochs[0] = (initialised & 2) ? 0 : fit_winrate(n, cf, vf, gf, won, wr, 256, 0.2, 1024, wr_trace);
  initialised &= 1;
  /* ---- 2. estimated utilities with the fitted model (float32 W, as .numpy() of it) */
  for (int64_t i = 0; i < n; ++i) {
    const float W = (float)winrate(wr, cf[i], vf[i], gf[i]);
    const double V = ctr[i] * value[i], P = ctr[i] * value[i] * gamma[i];
    eu[i] = (double)W * (V - P);
    if (est_util_out) est_util_out[i] = eu[i];
  }
  /* ---- 3. imitation of the logging policy (first update only) */
  epochs[1] = initialised ? 0 : fit_imitation(n, cf, vf, gf, pol, init_trace);
  /* ---- 4. doubly robust policy fit */
  {
    adam_t ad;
    adam_init(&ad, 12, 7e-3, 1e-4);
    plateau_t pl;
    plateau_init(&pl, 100, 0.2, 1e-8, 5e-3);
    stopper_t st = {INFINITY, -1, 512};
    const double inv_sqrt2pi = 1.0 / sqrt(2.0 * 3.141592653589793);
    int32_t e = 0;
    for (; e < 32768 && e < noise_epochs; ++e) {
      const float *eps = noise + (int64_t)e * n;
      __int128 L = 0, G[12];
      memset(G, 0, sizeof G);
      for (int64_t i = 0; i < n; ++i) {
        polf_t f;
        policy_fwd(pol, cf[i], vf[i], &f);
        const double mu = f.mu, sg = f.sigma, g = (double)gf[i];
        const double zz = (mu - g) / sg;
        const double pdf_raw = exp(-(zz * zz) / 2.0) / sg * inv_sqrt2pi;
        const double pi = pdf_raw < 1e-30 ? 1e-30 : pdf_raw;
        const double p0 = (double)fmaxf((float)prop[i], 1e-15f);
        const double iw = pi / p0;
        const double iwc = iw < 1.0 / 50.0 ? 1.0 / 50.0 : (iw > 50.0 ? 50.0 : iw);
        const double du = (double)(float)util[i] - (double)(float)eu[i];
        const double raw = mu + sg * (double)eps[i];
        const double gs = raw < 0.0 ? 0.0 : (raw > 1.0 ? 1.0 : raw);
        const double c = cf[i], v = vf[i];
        const double Wv = winrate(wr, c, v, gs);
        const double V = c * v;
        const double dm_term = Wv * (V - V * gs);
        L += fxr(-(du * iwc + dm_term));
        /* d(-term)/dmu, d(-term)/dsigma */
        double dpi_dmu = 0.0, dpi_dsg = 0.0;
        if (pdf_raw >= 1e-30 && iw >= 1.0 / 50.0 && iw <= 50.0) {
          const double k = du / p0;              /* d(du * iw)/dpi */
          dpi_dmu = k * pdf_raw * (g - mu) / (sg * sg);
          dpi_dsg = k * pdf_raw * ((g - mu) * (g - mu) / (sg * sg * sg) - 1.0 / sg);
        }
        double ddm_dgs = 0.0;
        if (raw >= 0.0 && raw <= 1.0)
          ddm_dgs = -Wv * V + (V - V * gs) * Wv * (1.0 - Wv) * (double)wr[2];
        const double dmu = -(dpi_dmu + ddm_dgs);
        const double dsg = -(dpi_dsg + ddm_dgs * (double)eps[i]);
        policy_bwd(pol, c, v, &f, dmu, dsg, G);
      }
      {
        __int128 t[13];
        t[0] = L;
        for (int j = 0; j < 12; ++j) t[1 + j] = G[j];
        ora_reduce128(t, 13);
        L = t[0];
        for (int j = 0; j < 12; ++j) G[j] = t[1 + j];
      }
      const float loss = (float)(fxv(L) / (double)ora_total(n));
      float grad[12];
      for (int j = 0; j < 12; ++j) grad[j] = (float)(fxv(G[j]) / (double)ora_total(n));
      adam_step(&ad, pol, grad);
      if (dr_trace) dr_trace[e] = loss;
      plateau_step(&pl, loss, &ad.lr);
      if (stop_step(&st, e, loss)) {
        ++e;
        break;
      }
    }
    epochs[2] = e;
  }
  free(cf);
  free(vf);
  free(gf);
  free(eu);
  return 0;
}

/* Philox4x32-10 (ag_oracle.c) */
void ora_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);

/* Synthetic rsample noise of the DR / DM fits (ag_bidder_update with noise == NULL): record
 * i of epoch e of agent a ~ N(0, 1) by Marsaglia's polar method on Philox4x32-10 (counter (i,
 * e, attempt, a), key = seed): each call gives two candidate pairs (u, v) = (w0, w1), (w2, w3)
 * as 32-bit uniforms on [-1, 1), the first accepted pair is taken; log through the restated
 * log1p, rounded to float32. */
void ora_fit_noise(uint64_t seed, uint32_t agent, int32_t epochs, int64_t n, float *out) {
  const uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  for (int32_t e = 0; e < epochs; ++e)
    for (int64_t i = 0; i < n; ++i) {
      float z = 0.0f;
      for (uint32_t t = 0; t < 32; ++t) {
        const uint32_t ctr[4] = {(uint32_t)i, (uint32_t)e, t, agent};
        uint32_t w[4];
        ora_philox4x32_10(ctr, key, w);
        int found = 0;
        for (int h = 0; h < 2 && !found; ++h) {
          const double u = (double)w[2 * h] * 0x1p-31 - 1.0;
          const double v = (double)w[2 * h + 1] * 0x1p-31 - 1.0;
          const double s = u * u + v * v;
          if (s > 0.0 && s < 1.0) {
            z = (float)(u * sqrt(-2.0 * fl_log1p(s - 1.0) / s));
            found = 1;
          }
        }
        if (found) break;
      }
      out[(int64_t)e * n + i] = z;
    }
}

/* torch's float32 exp on the CPU, as torch.sigmoid's vectorised path computes it (ATen's
 * sigmoid kernel: (1 + exp(-x)).reciprocal() with Vectorized<float>::exp = SLEEF's expf_u10):
 * round(x / ln 2) = q, x - q ln 2 in two fused steps, a degree-5 polynomial by fused Horner,
 * times 2^q in two power-of-two steps; 0 below -104, inf above 100. Pinned against
 * torch.sigmoid in tests/golden (every search-bid grid point of search_bid_kat.npz). */
static float torch_expf(float d) {
  const float q = rintf(d * 1.442695040888963407359924681001892137426645954152985934135449406931f);
  float s = fmaf(q, -0.693145751953125f, d);
  s = fmaf(q, -1.428606765330187045e-06f, s);
  float u = 0.000198527617612853646278381f;
  u = fmaf(u, s, 0.00139304355252534151077271f);
  u = fmaf(u, s, 0.00833336077630519866943359f);
  u = fmaf(u, s, 0.0416664853692054748535156f);
  u = fmaf(u, s, 0.166666671633720397949219f);
  u = fmaf(u, s, 0.5f);
  u = 1.0f + fmaf(s * s, u, s);
  const int e = (int)q, e1 = e >> 1;
  u = u * ldexpf(1.0f, e1) * ldexpf(1.0f, e - e1);
  if (d < -104.0f) u = 0.0f;
  if (d > 100.0f) u = INFINITY;
  return u;
}

float ora_torch_sigmoidf(float z) { return 1.0f / (1.0f + torch_expf(-z)); }

/* ValueLearningBidder 'search' (src/Bidder.py:180-196): prob_win of the 128 grid points is
 * PyTorchWinRateEstimator on float32 rows [ctr, value, gamma] as torch runs it on the CPU --
 * Linear(3, 1) as the BLAS kernel sums it, z = (fma(value, w1, ctr w0) + gamma w2) + b, then
 * the vectorised sigmoid (torch_expf) -- and the utility prob_win (ev - ev gamma) in double;
 * the first maximum in sorted-grid order (the smallest gamma among ties). Reproduces the
 * reference's gamma in every one of the 24000 bids of search_bid_kat.npz. */
double ora_search_gamma(const float *wr, double ctr, double value, const double *grid, int64_t stride) {
  const float c = (float)ctr, v = (float)value;
  const float cv = fmaf(v, wr[1], c * wr[0]);
  const double ev = value * ctr;
  double best_u = -INFINITY, best_g = 0.0;
  for (int j = 0; j < 128; ++j) {
    const double g = grid[(int64_t)j * stride];
    const float z = (cv + (float)g * wr[2]) + wr[3];
    const float pw = ora_torch_sigmoidf(z);
    const double ut = (double)pw * (ev - ev * g);
    if (ut > best_u || (ut == best_u && g < best_g)) {
      best_u = ut;
      best_g = g;
    }
  }
  return best_g;
}

/* DoublyRobustBidder.bid with a fitted policy (src/Bidder.py:466-470, src/Models.py:155-164):
 * x = float32 [estimated CTR, value]; the policy's mu and sigma (double, as in the fit, then
 * rounded to float32 like torch's tensors), the rsample mu + sigma * eps in float32, its
 * Gaussian density exp(log_prob) rounded to float32 (log via the restated log1p), gamma =
 * clip(sample, 0, 1). torch computes every step in float32: bids agree to float32 rounding. */
void ora_policy_bid(const float *p, double ctr, double value, float eps, double *gamma, double *prop) {
  polf_t f;
  policy_fwd(p, (double)(float)ctr, (double)(float)value, &f);
  const float mu = (float)f.mu, sg = (float)f.sigma;
  const float raw = mu + sg * eps;
  const double z = ((double)raw - (double)mu) / (double)sg;
  const double logp = -(z * z) / 2.0 - fl_log1p((double)sg - 1.0) - 0.91893853320467274178;
  *prop = (double)(float)exp(logp);
  *gamma = raw < 0.0f ? 0.0 : (raw > 1.0f ? 1.0 : (double)raw);
}

/* ValueLearningBidder.update for one agent (src/Bidder.py:204-325): no wins -> the
 * reference's fallback (model_initialised = False, nothing trained; returns 1); else the
 * win-rate fit (ReduceLROnPlateau patience 100, factor 0.1; early stop after 512 epochs)
 * and, with inference 'policy', the policy fit (:258-303): loss -mean(W(ctr, value, g~) (V -
 * V g~)), g~ = clip(mu + sigma eps, 0, 1) with the per-epoch rsample noise (given), V = ctr
 * value; Adam(lr 2e-3, wd 1e-6, AMSGrad), ReduceLROnPlateau(patience 100, factor 0.1,
 * min_lr 1e-7), early stop after 256 epochs, <= 16384 epochs. BidShadingPolicy's hidden
 * layers (src/Models.py:72-76) are not on the forward path: they get no gradient and Adam
 * skips them, so pol holds the 12 parameters of the path (shared, mu out, sigma out).
 * Sums as in ora_dr_update (exact fixed point). epochs [3] = (win-rate, 0, policy). */
int32_t ora_vl_update(int64_t n, const double *ctr, const double *value, const double *gamma,
                      const uint8_t *won, float *wr, float *pol, int32_t policy, const float *noise,
                      int64_t noise_epochs, int32_t *epochs, float *wr_trace, float *pol_trace) {
  epochs[0] = epochs[1] = epochs[2] = 0;
  if (ora_total(n) < 1) return -1;
  __int128 wins = 0;
  for (int64_t i = 0; i < n; ++i) wins += won[i] != 0;
  ora_reduce128(&wins, 1);
  if (!wins) return 1;
  float *cf = malloc(n * sizeof(float)), *vf = malloc(n * sizeof(float)), *gf = malloc(n * sizeof(float));
  for (int64_t i = 0; i < n; ++i) {
    cf[i] = (float)ctr[i];
    vf[i] = (float)value[i];
    gf[i] = (float)gamma[i];
  }
  epochs[0] = fit_winrate(n, cf, vf, gf, won, wr, 100, 0.1, 512, wr_trace);
  if (policy) {
    adam_t ad;
    adam_init(&ad, 12, 2e-3, 1e-6);
    plateau_t pl;
    plateau_init(&pl, 100, 0.1, 1e-7, 1e-4);
    stopper_t st = {INFINITY, -1, 256};
    int32_t e = 0;
    for (; e < 16384 && e < noise_epochs; ++e) {
      const float *eps = noise + (int64_t)e * n;
      __int128 L = 0, G[12];
      memset(G, 0, sizeof G);
      for (int64_t i = 0; i < n; ++i) {
        polf_t f;
        const double c = cf[i], v = vf[i];
        policy_fwd(pol, c, v, &f);
        const double raw = f.mu + f.sigma * (double)eps[i];
        const double gs = raw < 0.0 ? 0.0 : (raw > 1.0 ? 1.0 : raw);
        const double Wv = winrate(wr, c, v, gs);
        const double V = c * v;
        L += fxr(-(Wv * (V - V * gs)));
        double ddm_dgs = 0.0;
        if (raw >= 0.0 && raw <= 1.0) ddm_dgs = -Wv * V + (V - V * gs) * Wv * (1.0 - Wv) * (double)wr[2];
        policy_bwd(pol, c, v, &f, -ddm_dgs, -(ddm_dgs * (double)eps[i]), G);
      }
      {
        __int128 t[13];
        t[0] = L;
        for (int j = 0; j < 12; ++j) t[1 + j] = G[j];
        ora_reduce128(t, 13);
        L = t[0];
        for (int j = 0; j < 12; ++j) G[j] = t[1 + j];
      }
      const float loss = (float)(fxv(L) / (double)ora_total(n));
      float grad[12];
      for (int j = 0; j < 12; ++j) grad[j] = (float)(fxv(G[j]) / (double)ora_total(n));
      adam_step(&ad, pol, grad);
      if (pol_trace) pol_trace[e] = loss;
      plateau_step(&pl, loss, &ad.lr);
      if (stop_step(&st, e, loss)) {
        ++e;
        break;
      }
    }
    epochs[2] = e;
  }
  free(cf);
  free(vf);
  free(gf);
  return 0;
}

/* Fixed-order double sums of the policy-learning fits (importance weights are unbounded,
 * so their terms do not fit a fixed-point grid): record i goes to lane i mod 256 and is
 * added in record order; each 64-lane wave is combined by the butterfly v[l] + v[l ^ o],
 * o = 32, 16, ..., 1 (identical on every lane); the four wave totals are added to 0.0 in
 * wave order. This is the device's reduction order exactly (csrc/ag_dr.hip). */
#define PL_LANES 256
#define PL_NV 14
static void pl_lane_sums(double (*acc)[PL_NV], double *tot) {
  for (int j = 0; j < PL_NV; ++j) {
    double t = 0.0;
    for (int w = 0; w < PL_LANES / 64; ++w) {
      double v[64], nv[64];
      for (int l = 0; l < 64; ++l) v[l] = acc[w * 64 + l][j];
      for (int o = 32; o > 0; o >>= 1) {
        for (int l = 0; l < 64; ++l) nv[l] = v[l] + v[l ^ o];
        memcpy(v, nv, sizeof v);
      }
      t += v[0];
    }
    tot[j] = t;
  }
}

/* per-record gradient of a policy loss term given d/dmu and d/dsigma (the order of
 * policy_bwd, in double) */
static void policy_grad(const float *p, double c, double v, const polf_t *f, double dmu, double dsigma,
                        double *g) {
  const double dam = dmu * dsoftplus(f->am), das = dsigma * dsoftplus(f->as);
  double ds[2];
  ds[0] = dam * (double)p[6] + das * (double)p[9];
  ds[1] = dam * (double)p[7] + das * (double)p[10];
  g[6] = dam * f->s[0];
  g[7] = dam * f->s[1];
  g[8] = dam;
  g[9] = das * f->s[0];
  g[10] = das * f->s[1];
  g[11] = das;
  for (int j = 0; j < 2; ++j) {
    const double dh = ds[j] * dsoftplus(f->h[j]);
    g[2 * j] = dh * c;
    g[2 * j + 1] = dh * v;
    g[4 + j] = dh;
  }
}

/* PolicyLearningBidder.update for one agent (src/Bidder.py:364-431, the losses of
 * src/Models.py:174-199): imitation of the logging policy on the first update, then the
 * policy fit with Adam(lr 2e-3, wd 1e-4, AMSGrad), ReduceLROnPlateau(patience 100, factor
 * 0.2, min_lr 1e-8), early stop after 512 epochs, <= 16384 epochs, importance-weight
 * clipping eps 50, KL weight 5e-2. loss_kind: 0 REINFORCE, 1 REINFORCE_offpolicy, 2 TRPO,
 * 3 PPO (AG_PL_LOSS_*). Target propensities are clip(pdf, min 1e-30), logging ones
 * clip(float32, min 1e-15). torch.min's gradient on ties is split half and half, which for
 * PPO makes the gradient flow through iw u whenever iw is inside the clip range or iw u <
 * clip(iw) u. Returns 0, -1 without logs, -2 on a NaN loss (the reference exits). epochs
 * [3] = (0, imitation, policy). */
/* one epoch of a policy-learning loss: the float32 loss and gradient (mean over the n
 * records) at pol */
static float pl_epoch(int64_t n, int32_t nblk, const float *cf, const float *vf, const float *gf,
                      const double *prop, const double *util, const float *pol, int32_t loss_kind,
                      double (*acc)[PL_NV], float *grad) {
  const double inv_sqrt2pi = 1.0 / sqrt(2.0 * 3.141592653589793);
  const int64_t per = (n + nblk - 1) / nblk;
  double tot[PL_NV];
  for (int j = 0; j < PL_NV; ++j) tot[j] = 0.0;
  for (int32_t b = 0; b < nblk; ++b) { /* the device's workgroups, in order */
    const int64_t c0 = (int64_t)b * per < n ? (int64_t)b * per : n;
    const int64_t c1 = c0 + per < n ? c0 + per : n;
    memset(acc, 0, sizeof(double[PL_LANES][PL_NV]));
    for (int64_t i = c0; i < c1; ++i) {
      polf_t f;
      const double c = cf[i], v = vf[i], g = (double)gf[i];
      policy_fwd(pol, c, v, &f);
      const double mu = f.mu, sg = f.sigma;
      const double zz = (mu - g) / sg;
      const double pdf_raw = exp(-(zz * zz) / 2.0) / sg * inv_sqrt2pi;
      const double pi = pdf_raw < 1e-30 ? 1e-30 : pdf_raw;
      const double p0 = (double)fmaxf((float)prop[i], 1e-15f);
      const double u = (double)(float)util[i];
      double term = 0.0, kl = 0.0, dpi = 0.0, dmu = 0.0, dsg = 0.0;
      if (loss_kind == 0) {
        term = -(pi * u);
        dpi = -u;
      } else if (loss_kind == 1 || loss_kind == 2) {
        term = -((pi / p0) * u);
        dpi = -u / p0;
        if (loss_kind == 2) {
          kl = (sg * sg + (mu - g) * (mu - g)) / (2.0 * sg * sg) - 0.5;
          dmu = 5e-2 * ((mu - g) / (sg * sg));
          dsg = 5e-2 * (-((mu - g) * (mu - g)) / (sg * sg * sg));
        }
      } else {
        const double iw = pi / p0;
        const int in_range = iw >= 1.0 / 50.0 && iw <= 50.0;
        const double iwc = iw < 1.0 / 50.0 ? 1.0 / 50.0 : (iw > 50.0 ? 50.0 : iw);
        const double A = iw * u, Bc = iwc * u;
        term = -(A < Bc ? A : Bc);
        dpi = (in_range || A < Bc) ? -u / p0 : 0.0;
      }
      if (pdf_raw >= 1e-30 && dpi != 0.0) {
        dmu += dpi * pdf_raw * (g - mu) / (sg * sg);
        dsg += dpi * pdf_raw * ((g - mu) * (g - mu) / (sg * sg * sg) - 1.0 / sg);
      }
      double gr[12];
      policy_grad(pol, c, v, &f, dmu, dsg, gr);
      double *a = acc[(i - c0) % PL_LANES];
      for (int j = 0; j < 12; ++j) a[j] += gr[j];
      a[12] += term;
      a[13] += kl;
    }
    double bt[PL_NV];
    pl_lane_sums(acc, bt);
    for (int j = 0; j < PL_NV; ++j) tot[j] += bt[j];
  }
  for (int j = 0; j < 12; ++j) grad[j] = (float)(tot[j] / (double)n);
  return (float)(tot[12] / (double)n + (tot[13] / (double)n) * 5e-2);
}

static float *to_f32(int64_t n, const double *x) {
  float *f = malloc(n * sizeof(float));
  for (int64_t i = 0; i < n; ++i) f[i] = (float)x[i];
  return f;
}

float ora_pl_loss_grad(int64_t n, const double *ctr, const double *value, const double *gamma,
                       const double *prop, const double *util, const float *pol, int32_t loss_kind,
                       float *grad) {
  float *cf = to_f32(n, ctr), *vf = to_f32(n, value), *gf = to_f32(n, gamma);
  double (*acc)[PL_NV] = malloc(sizeof(double[PL_LANES][PL_NV]));
  const float loss = pl_epoch(n, 1, cf, vf, gf, prop, util, pol, loss_kind, acc, grad);
  free(acc);
  free(cf);
  free(vf);
  free(gf);
  return loss;
}

int32_t ora_pl_update(int64_t n, const double *ctr, const double *value, const double *gamma,
                      const double *prop, const double *util, float *pol, int32_t initialised,
                      int32_t loss_kind, int32_t nblk, int32_t *epochs, float *init_trace, float *pl_trace) {
  epochs[0] = epochs[1] = epochs[2] = 0;
  if (n < 1) return -1;
  float *cf = to_f32(n, ctr), *vf = to_f32(n, value), *gf = to_f32(n, gamma);
  if (!initialised) epochs[1] = fit_imitation(n, cf, vf, gf, pol, init_trace);
  double (*acc)[PL_NV] = malloc(sizeof(double[PL_LANES][PL_NV]));
  adam_t ad;
  adam_init(&ad, 12, 2e-3, 1e-4);
  plateau_t pl;
  plateau_init(&pl, 100, 0.2, 1e-8, 1e-4);
  stopper_t st = {INFINITY, -1, 512};
  int32_t e = 0, rc = 0;
  for (; e < 16384; ++e) {
    float grad[12];
    const float loss = pl_epoch(n, nblk < 1 ? 1 : nblk, cf, vf, gf, prop, util, pol, loss_kind, acc, grad);
    adam_step(&ad, pol, grad);
    if (pl_trace) pl_trace[e] = loss;
    plateau_step(&pl, loss, &ad.lr);
    const int stop = stop_step(&st, e, loss);
    if (loss != loss) rc = -2;
    if (stop || rc) {
      ++e;
      break;
    }
  }
  epochs[2] = e;
  free(acc);
  free(cf);
  free(vf);
  free(gf);
  return rc;
}
