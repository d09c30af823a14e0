// ag_dr.hip -- DoublyRobustBidder.update on the GPU (Agent.update -> src/Bidder.py:473-615,
// models src/Models.py:51-62, :92-218).
//
// One workgroup per DR agent, persistent over the three fits the reference runs one after
// the other: the win-rate model (BCE on the logs + the gamma = 0 augmentation, <= 32768
// epochs), the policy's imitation of the logging policy (first update only, <= 16384) and
// the doubly robust policy fit (<= 32768, rsample noise per epoch supplied by the caller).
// Everything a fit needs per epoch (Adam with weight decay + AMSGrad, ReduceLROnPlateau,
// the reference's early stop) runs on the device. Sums over the agent's records are exact
// (fixed-point terms added as integers), so the result is independent of record order and
// lane assignment; the arithmetic is oracle/ag_oracle_dr.c ora_dr_update, bit for bit.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <type_traits>
#include <vector>

#include <hipcub/hipcub.hpp>

#include "ag_exp.h"
#include "ag_exp_table.h"
#include "ag_host.h"
#include "ag_log1p.h"
#include "ag_philox.h"
#include "ag_coop.h"
#include "ag_div.h"

namespace {

using agcoop::agent_barrier;
using agcoop::bar_lines;
using agcoop::kBarLineWords;
constexpr int kDrThreads = 256;
constexpr int kWrEpochs = 32768, kInitEpochs = 16384, kDrEpochs = 32768;
constexpr int64_t kBidderChunk = 8192;  // records per workgroup of a PolicyLearningBidder (default)
constexpr int64_t kMinChunk = 1024;     // fewest records per workgroup of an exact-sum learner's split
#ifndef AG_DR_ABLATE_XCHG
#define AG_DR_ABLATE_XCHG 0  // diagnostic (wrong fits by design): each workgroup steps on its own partial sums
#endif
#ifndef AG_DR_WR_RECS
#define AG_DR_WR_RECS 1  // records per iteration of the win-rate loop (2: wr_pair2; A/B)
#endif
#ifndef AG_DR_SLOW_OUTLINE
#define AG_DR_SLOW_OUTLINE 0  // 1: the win-rate rows' rare path out of line (wr_slow; A/B)
#endif
#ifndef AG_DR_SHARED_DIV
#define AG_DR_SHARED_DIV 1  // the win-rate row's two divisions by 1 + e share one reciprocal (ag_div.h)
#endif
#ifndef AG_DR_REC_LDS0
#define AG_DR_REC_LDS0 (32 * 1024)
#endif
constexpr size_t kRecLdsBytes0 = AG_DR_REC_LDS0;  // record cache per workgroup, win-rate phase (4 per CU)
#ifndef AG_DR_REC_LDS
#define AG_DR_REC_LDS (48 * 1024)  // (3 workgroups per CU: profiles/r04r_ab_trainer_*.log)
#endif
#ifndef AG_DR_PH0_MIN_WAVES
#define AG_DR_PH0_MIN_WAVES 4  // the win-rate fits: <= 128 VGPRs
#endif
#ifndef AG_DR_PH1_MIN_WAVES
#define AG_DR_PH1_MIN_WAVES 3  // the later fits: <= 168 VGPRs, 3 waves per SIMD (FP_DR_TS update 1.96 -> 1.69 s)
#endif
constexpr size_t kRecLdsBytes = AG_DR_REC_LDS;  // record cache per workgroup, later fits
constexpr double kGrid = 0x1p40, kInv = 0x1p-40;
constexpr int64_t kLo24 = (int64_t(1) << 24) - 1;

// Fixed-point terms (int64)rint(v * 2^40). For |v * 2^40| < 2^51 (every term in practice)
// adding 1.5 * 2^52 rounds to the integer (nearest, ties to even, as rint) and leaves it in
// the low mantissa bits.
// The accumulators hold them biased: fxb(v) = (int64)rint(v * 2^40) + kFxMagic (mod 2^64),
// kFxMagic = the bits of 1.5 * 2^52 -- for |v * 2^40| < 2^51 simply the bits of v * 2^40 +
// 1.5 * 2^52, so a term costs one add and the 64-bit accumulate (no subtract); a lane that
// added n terms to an accumulator takes n * kFxMagic off once (fx_unbias) before the exact
// sums. Integer arithmetic mod 2^64: the same totals, bit for bit.
constexpr uint64_t kFxMagic = 0x4338000000000000ull;  // asu64(0x1.8p52)
__device__ __forceinline__ int64_t fxb_fast(double v) {  // |v| <= 2^10 guaranteed by the caller
  return (int64_t)agexp::asu64(v * kGrid + 0x1.8p52);
}
__device__ __forceinline__ int64_t fxb(double v) {
  const double x = v * kGrid;
  if (__builtin_expect(__builtin_fabs(x) < 0x1p51, 1)) return (int64_t)agexp::asu64(x + 0x1.8p52);
  return (int64_t)((uint64_t)(int64_t)__builtin_rint(x) + kFxMagic);
}
// fxb's fast path on x = v * 2^40 already formed, and its range test (callers test a
// record's terms together and take fxb for all of them when one is out of range)
__device__ __forceinline__ int64_t fxb_x(double x) { return (int64_t)agexp::asu64(x + 0x1.8p52); }
__device__ __forceinline__ bool fx_in(double x) { return __builtin_fabs(x) < 0x1p51; }
__device__ __forceinline__ void addw(int64_t &a, int64_t t) { a = (int64_t)((uint64_t)a + (uint64_t)t); }
__device__ __forceinline__ void fx_unbias(int64_t &a, int64_t n) {
  a = (int64_t)((uint64_t)a - (uint64_t)n * kFxMagic);
}

__device__ __forceinline__ double fxv(int64_t hi, int64_t lo) {
  hi += lo >> 24;
  lo &= kLo24;
  return ((double)hi * 0x1p24 + (double)lo) * kInv;
}

// softplus(u) = u > 20 ? u : log1p(exp(u)) and its derivative exp(u) / (exp(u) + 1), from
// e = exp(u) (the forward pass keeps it for the backward pass)
__device__ __forceinline__ double dsoftplus_e(double u, double e) { return u > 20.0 ? 1.0 : e / (e + 1.0); }
// log1p_main's divisions for a caller that holds r = the reciprocal of its 1 + x (ag_div.h)
struct SharedDiv {
  double r;
  __device__ double cu(double c, double u) const { return agdiv::div_core(c, u, r); }
  __device__ double fs(double f, double d) const { return agdiv::div_core(f, d, agdiv::recip(d)); }
};

// exp(x) and softplus from the branch-free main paths (the same bits), the rare inputs
// outside them patched with the full functions
using agexp::exp_fast;
// e = exp(u); returns softplus(u)
__device__ __forceinline__ double softplus_fast(double u, double &e, const uint64_t *tab) {
  e = agexp::exp_main(u, tab);
  bool lok;
  double l = aglog1p::log1p_main(e, lok);
  if (__builtin_expect(!(agexp::exp_in_main(u) && (lok || u > 20.0)), 0)) {
    e = agexp::exp(u, tab);
    l = aglog1p::log1p(e);
  }
  return u > 20.0 ? u : l;
}

// Exact block sum of NV per-lane int64 accumulators (each split at bit 24 so nothing can
// overflow): every thread gets the totals as (hi, lo) pairs in s_out.
template <int NV>
__device__ __forceinline__ void block_sums(const int64_t (&v)[NV], int64_t (*s_w)[32], int64_t *s_out) {
  static_assert(2 * NV <= 32, "block_sums: at most 16 sums");
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    int64_t h = v[j] >> 24, l = v[j] & kLo24;
    for (int o = 32; o > 0; o >>= 1) {
      h += __shfl_xor(h, o, 64);
      l += __shfl_xor(l, o, 64);
    }
    if (lane == 0) {
      s_w[wv][2 * j] = h;
      s_w[wv][2 * j + 1] = l;
    }
  }
  __syncthreads();
  if (threadIdx.x < 2 * NV) {
    int64_t t = 0;
    for (int w = 0; w < kDrThreads / 64; ++w) t += s_w[w][threadIdx.x];
    s_out[threadIdx.x] = t;
  }
  __syncthreads();
}

// torch.optim.Adam single-tensor step with weight decay and AMSGrad (thread j: param j)
struct AdamState {
  float ea[16], es[16], mx[16];
};

__device__ __forceinline__ void adam_param(float &p, float grad, int j, AdamState &a, float neg_step, float bc2f,
                                           float wdf) {
  const float g = grad + wdf * p;
  a.ea[j] = a.ea[j] + 0.1f * (g - a.ea[j]);
  a.es[j] = a.es[j] * 0.999f + (0.001f * g) * g;
  a.mx[j] = a.mx[j] > a.es[j] ? a.mx[j] : a.es[j];
  // float32 sqrt correctly rounded (as the CPU's sqrtss): via the refined FP64 sqrt
  const float den = (float)__builtin_sqrt((double)a.mx[j]) / bc2f + 1e-8f;
  p = p + neg_step * (a.ea[j] / den);
}

struct Plateau {
  double best, threshold, factor, min_lr;
  int bad, patience;
};
__device__ __forceinline__ void plateau_step(Plateau &s, float loss, double &lr) {
  if ((double)loss < s.best * (1.0 - s.threshold)) {
    s.best = (double)loss;
    s.bad = 0;
  } else {
    s.bad += 1;
  }
  if (s.bad > s.patience) {
    double nl = lr * s.factor;
    if (nl < s.min_lr) nl = s.min_lr;
    if (lr - nl > 1e-8) lr = nl;
    s.bad = 0;
  }
}
struct Stopper {
  double best;
  int best_epoch, wait;
};
__device__ __forceinline__ bool stop_step(Stopper &s, int epoch, float loss) {
  if (s.best - (double)loss > 1e-6) {
    s.best_epoch = epoch;
    s.best = (double)loss;
    return false;
  }
  return epoch - s.best_epoch > s.wait;
}

// forward values of the policy; eh / eam / eas = exp of h / am / as, kept for the backward
// pass's softplus derivatives
struct PolF {
  double h[2], s[2], am, as, mu, sp_sigma, sigma, eh[2], eam, eas;
  double rh[2], ram, ras;  // policy_fwd_main only: the reciprocals of 1 + eh / eam / eas (ag_div.h)
};
__device__ __forceinline__ void policy_fwd(const float *p, double c, double v, PolF &f, const uint64_t *tab) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    f.h[j] = c * (double)p[2 * j] + v * (double)p[2 * j + 1] + (double)p[4 + j];
    f.s[j] = softplus_fast(f.h[j], f.eh[j], tab);
  }
  f.am = f.s[0] * (double)p[6] + f.s[1] * (double)p[7] + (double)p[8];
  f.as = f.s[0] * (double)p[9] + f.s[1] * (double)p[10] + (double)p[11];
  f.mu = softplus_fast(f.am, f.eam, tab);
  f.sp_sigma = softplus_fast(f.as, f.eas, tab);
  f.sigma = f.sp_sigma + 0.01;  // min_sigma (src/Models.py:104)
}
// softplus through the main paths alone (ok cleared when an input leaves them); r = the
// reciprocal of 1 + e, shared by log1p's c / (1 + e) and the backward pass's e / (e + 1)
// (AG_DR_SHARED_DIV; where ok holds and u <= 20, e is in [2^-29, 2^29]: div_safe's range)
__device__ __forceinline__ double softplus_main(double u, double &e, double &r, const uint64_t *tab, bool &ok) {
  e = agexp::exp_main(u, tab);
  bool lok;
#if AG_DR_SHARED_DIV
  r = agdiv::recip(1.0 + e);
  const double l = aglog1p::log1p_main_t(e, lok, SharedDiv{r});
#else
  r = 0.0;
  const double l = aglog1p::log1p_main(e, lok);
#endif
  ok = (int)ok & (int)agexp::exp_in_main(u) & ((int)lok | (int)(u > 20.0));
  return u > 20.0 ? u : l;
}
// dsoftplus_e from softplus_main's reciprocal (the same bits where its ok holds)
__device__ __forceinline__ double dsoftplus_r(double u, double e, double r) {
#if AG_DR_SHARED_DIV
  return u > 20.0 ? 1.0 : agdiv::div_core(e, e + 1.0, r);
#else
  (void)r;
  return dsoftplus_e(u, e);
#endif
}
// policy_fwd through the main paths alone: true when they gave policy_fwd's values (every
// softplus input inside them), else the caller runs policy_fwd -- one rare branch per record
// instead of one per softplus
__device__ __forceinline__ bool policy_fwd_main(const float *p, double c, double v, PolF &f, const uint64_t *tab) {
  bool ok = true;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    f.h[j] = c * (double)p[2 * j] + v * (double)p[2 * j + 1] + (double)p[4 + j];
    f.s[j] = softplus_main(f.h[j], f.eh[j], f.rh[j], tab, ok);
  }
  f.am = f.s[0] * (double)p[6] + f.s[1] * (double)p[7] + (double)p[8];
  f.as = f.s[0] * (double)p[9] + f.s[1] * (double)p[10] + (double)p[11];
  f.mu = softplus_main(f.am, f.eam, f.ram, tab, ok);
  f.sp_sigma = softplus_main(f.as, f.eas, f.ras, tab, ok);
  f.sigma = f.sp_sigma + 0.01;
  return ok;
}
__device__ __forceinline__ void policy_fwd_fast(const float *p, double c, double v, PolF &f, const uint64_t *tab) {
  if (__builtin_expect(!policy_fwd_main(p, c, v, f, tab), 0)) policy_fwd(p, c, v, f, tab);
}
// policy_bwd's twelve gradient terms as doubles (d[j]: parameter j), the same expressions,
// from policy_fwd_main's values (used only where its ok holds)
__device__ __forceinline__ void policy_terms(const float *p, double c, double v, const PolF &f, double dmu,
                                             double dsigma, double *d) {
  const double dam = dmu * dsoftplus_r(f.am, f.eam, f.ram), das = dsigma * dsoftplus_r(f.as, f.eas, f.ras);
  double ds[2];
  ds[0] = dam * (double)p[6] + das * (double)p[9];
  ds[1] = dam * (double)p[7] + das * (double)p[10];
  d[6] = dam * f.s[0];
  d[7] = dam * f.s[1];
  d[8] = dam;
  d[9] = das * f.s[0];
  d[10] = das * f.s[1];
  d[11] = das;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const double dh = ds[j] * dsoftplus_r(f.h[j], f.eh[j], f.rh[j]);
    d[2 * j] = dh * c;
    d[2 * j + 1] = dh * v;
    d[4 + j] = dh;
  }
}
// a record's N fixed-point terms through fxb's fast path when every one is in its range (ok
// in: the record's main-path test), added to acc[0..N); false (nothing added) otherwise
template <int N>
__device__ __forceinline__ bool fx_add_fast(int64_t (&acc)[16], const double (&d)[N], bool ok) {
  double x[N];
#pragma unroll
  for (int k = 0; k < N; ++k) {
    x[k] = d[k] * kGrid;
    ok = (int)ok & (int)fx_in(x[k]);
  }
  if (__builtin_expect(!ok, 0)) return false;
#pragma unroll
  for (int k = 0; k < N; ++k) addw(acc[k], fxb_x(x[k]));
  return true;
}

__device__ __forceinline__ void policy_bwd(const float *p, double c, double v, const PolF &f, double dmu,
                                           double dsigma, int64_t (&G)[16], int off, const uint64_t *tab) {
  const double dam = dmu * dsoftplus_e(f.am, f.eam), das = dsigma * dsoftplus_e(f.as, f.eas);
  double ds[2];
  ds[0] = dam * (double)p[6] + das * (double)p[9];
  ds[1] = dam * (double)p[7] + das * (double)p[10];
  // biased terms (fxb): one per accumulator per record, fx_unbias'd by the caller
  addw(G[off + 6], fxb(dam * f.s[0]));
  addw(G[off + 7], fxb(dam * f.s[1]));
  addw(G[off + 8], fxb(dam));
  addw(G[off + 9], fxb(das * f.s[0]));
  addw(G[off + 10], fxb(das * f.s[1]));
  addw(G[off + 11], fxb(das));
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const double dh = ds[j] * dsoftplus_e(f.h[j], f.eh[j]);
    addw(G[off + 2 * j], fxb(dh * c));
    addw(G[off + 2 * j + 1], fxb(dh * v));
    addw(G[off + 4 + j], fxb(dh));
  }
}

__device__ __forceinline__ void bias_corrections(int step, const double *adam_tab, float &bc2f, double &bc1) {
  // adam_tab: [0, kDrEpochs): 1 - 0.9^t; [kDrEpochs, 2 kDrEpochs): (1 - 0.999^t)^0.5 (libm pow)
  bc1 = adam_tab[step];
  bc2f = (float)adam_tab[kDrEpochs + step];
}

// records of agent a: SoA, bucketed: ctr, value, gamma, prop, util (f64), won (u8)
struct DrRecords {
  const double *ctr, *value, *gamma, *prop, *util;
  const uint8_t *won;
};

// LDS of one workgroup
struct TrainLds {
  uint64_t tab[256];
  float wr[4], pol[12];
  int64_t w[kDrThreads / 64][32];
  int64_t tot[32];
  double wf[kDrThreads / 64][16];
  double ftot[16];
  AdamState adam;
  int stop;       // a NaN loss
  int exhausted;  // a noise-driven fit ran out of noise epochs before it stopped
  int flag;       // agent_allreduce_i64's broadcast
  uint64_t gprev[2][32];  // agent_allreduce_grouped's row sums of the last two rounds
};

__device__ __forceinline__ void adam_reset(TrainLds &S) {
  if (threadIdx.x < 16) S.adam.ea[threadIdx.x] = S.adam.es[threadIdx.x] = S.adam.mx[threadIdx.x] = 0.0f;
  __syncthreads();
}

// The workgroups training one agent: each owns a contiguous chunk of the agent's records and
// exchanges its per-epoch partial sums through `part` ([2 parities][nblk][32] words) at an
// agent barrier; afterwards every workgroup holds the same totals and runs the same Adam /
// scheduler / early-stop step on its LDS copy of the parameters (the workgroups stay in
// lockstep without a second barrier: an exchange's parity buffer is only rewritten two
// exchanges later, after every workgroup has passed the barrier in between).
struct Coop {
  int rank, nblk;
  int64_t *part;
  unsigned *bar;  // the agent's barrier lines (bar_lines)
  int ph;         // exchanges so far (identical in every workgroup of the agent)
  int64_t *acc;   // exact_totals' accumulator rows [bar_lines][32] (row 0: the totals), zero
                  // between exchanges; AG_COOP_GROUPED: agent_allreduce_grouped's [2][groups][32]
  unsigned *gcnt; // AG_COOP_GROUPED: its group arrival counters (group_lines, after the barrier lines)
  unsigned rnd;   // AG_COOP_GROUPED: exact_totals calls so far
};

// exact totals of NV fixed-point sums over the agent's records (S.tot: hi, lo pairs), summed
// up the agent barrier's combining tree with integer atomics: each workgroup adds its 2 NV
// words to its level-0 node's accumulator row and arrives; the last arriver at a node moves
// the node's row into its parent's (zeroing it) and arrives one level up; the root's last
// arriver publishes the totals in row 0 and releases everyone, who read that one row.
// Integer additions: the totals are exact whatever the order (round 1 had every workgroup
// read every other workgroup's partials after the barrier: nblk lines from other XCDs per
// workgroup per epoch).
template <int NV>
__device__ __forceinline__ void exact_totals(const int64_t (&acc)[NV], TrainLds &S, Coop &C) {
  block_sums<NV>(acc, S.w, S.tot);
  if (C.nblk > 1 && !(AG_DR_ABLATE_XCHG & 1)) {
#if AG_COOP_GROUPED
    agcoop::agent_allreduce_grouped(C.gcnt, C.acc, 32, C.rank, C.nblk, S.tot, 2 * NV, S.tot, ++C.rnd, S.gprev);
#else
    agcoop::agent_allreduce_i64(C.bar, C.acc, 32, C.rank, C.nblk, S.tot, 2 * NV, S.tot, &S.flag);
#endif
    ++C.ph;
  }
}

// Fixed-order double sums (the policy-learning fits: importance weights are unbounded, so
// their terms do not fit a fixed-point grid). In each workgroup, record c0 + j is added by
// thread j mod 256 in record order; each wave combines by the butterfly v + shfl_xor(v, o),
// o = 32 .. 1 (the same value on every lane); the wave totals are added to 0.0 in wave
// order; the workgroup totals are added to 0.0 in workgroup order. oracle/ag_oracle_dr.c
// pl_epoch is this order exactly.
template <int NV>
__device__ __forceinline__ void float_totals(const double (&v)[NV], TrainLds &S, Coop &C) {
  static_assert(NV <= 16, "float_totals: at most 16 sums");
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    double x = v[j];
    for (int o = 32; o > 0; o >>= 1) x = x + __shfl_xor(x, o, 64);
    if (lane == 0) S.wf[wv][j] = x;
  }
  __syncthreads();
  double t = 0.0;
  if (threadIdx.x < NV)
    for (int w = 0; w < kDrThreads / 64; ++w) t += S.wf[w][threadIdx.x];
  if (C.nblk > 1) {
    double *pp = reinterpret_cast<double *>(C.part + (size_t)(C.ph & 1) * C.nblk * 32);
    if (threadIdx.x < NV) pp[C.rank * 32 + threadIdx.x] = t;
    agent_barrier(C.bar, C.rank, C.nblk);
    if (threadIdx.x < NV) {
      double T = 0.0;
      for (int b = 0; b < C.nblk; ++b) T += pp[b * 32 + threadIdx.x];
      S.ftot[threadIdx.x] = T;
    }
    ++C.ph;
  } else if (threadIdx.x < NV) {
    S.ftot[threadIdx.x] = 0.0 + t;
  }
  __syncthreads();
}

// one Adam step of the first np parameters of `par` (thread j: parameter j)
__device__ __forceinline__ void adam_step_block(TrainLds &S, float *par, int np, float grad, int step, double lr,
                                                float wd, const double *adam_tab) {
  double bc1;
  float bc2f;
  bias_corrections(step, adam_tab, bc2f, bc1);
  const float neg_step = (float)(-(lr / bc1));
  if ((int)threadIdx.x < np) {
    float p = par[threadIdx.x];
    adam_param(p, grad, threadIdx.x, S.adam, neg_step, bc2f, wd);
    par[threadIdx.x] = p;
  }
}

// The rsample noise of the DR / DM policy fits: the caller's draws (noise != NULL: agent's
// record i of epoch e at noise[e * n + i]) or synthetic ones -- a standard normal by
// Marsaglia's polar method on Philox4x32-10 (counter (i, e, attempt, agent), key = seed), two
// candidate pairs of 32-bit uniforms per call (a wave's 64 lanes then finish in ~2 calls
// instead of ~4 with one pair), its log through the restated log1p, so the host
// (oracle/ag_oracle_dr.c ora_fit_noise) draws the same bits.
struct FitNoise {
  const float *noise;  // agent's draws or NULL
  int64_t n;           // agent's record count
  uint64_t seed;
  uint32_t agent;
  int epochs;          // epochs available (synthetic: unlimited)
};

__device__ __forceinline__ double fit_eps(const FitNoise &F, int e, int64_t i) {
  if (F.noise) return (double)F.noise[(int64_t)e * F.n + i];
  // the rejection loop only finds the first accepted (u, s); the transform runs once after
  // it for every lane together (a wave's lanes accept at different attempts)
  double u = 0.0, s = 0.0;
  bool found = false;
  for (uint32_t t = 0; t < 32 && !found; ++t) {
    uint32_t w[4];
    philox((uint32_t)i, (uint32_t)e, t, F.agent, (uint32_t)F.seed, (uint32_t)(F.seed >> 32), w);
    const double u0 = (double)w[0] * 0x1p-31 - 1.0, v0 = (double)w[1] * 0x1p-31 - 1.0;
    const double u1 = (double)w[2] * 0x1p-31 - 1.0, v1 = (double)w[3] * 0x1p-31 - 1.0;
    const double s0 = u0 * u0 + v0 * v0, s1 = u1 * u1 + v1 * v1;
    const bool a0 = s0 > 0.0 && s0 < 1.0, a1 = s1 > 0.0 && s1 < 1.0;
    if (a0 || a1) {
      u = a0 ? u0 : u1;
      s = a0 ? s0 : s1;
      found = true;
    }
  }
  if (!found) return 0.0;
  return (double)(float)(u * __builtin_sqrt(-2.0 * aglog1p::log1p(s - 1.0) / s));
}

// records of the workgroup: [c0, c0 + nb) of the agent's n
struct Chunk {
  int64_t c0, nb, n;
};

// The workgroup's records as the fits read them, every epoch: the first `cap` of its chunk
// staged once in LDS as float32 fields (every fit consumes them through a float32 rounding,
// so the staged values are the ones it would compute: (float)ctr, (float)value, ...), the rest
// read from the global store. Local index j = record c0 + j of the agent. Fields [nf][cap]
// floats: ctr, value, gamma, propensity, utility, estimated utility; then won [cap] bytes.
enum { kFCtr = 0, kFVal, kFGam, kFProp, kFUtil, kFEu };
struct RecView {
  DrRecords R;       // the agent's records (global)
  const double *eu;  // the agent's estimated utilities (global, DoublyRobustBidder)
  int64_t c0;
  const float *lf;  // LDS fields
  const uint8_t *lw;
  int64_t cap;      // staged records (a multiple of kDrThreads, so j < cap is block-uniform)
  __device__ __forceinline__ double f(int fld, const double *g, int64_t j) const {
    return j < cap ? (double)lf[(int64_t)fld * cap + j] : (double)(float)g[c0 + j];
  }
  __device__ __forceinline__ double ctr(int64_t j) const { return f(kFCtr, R.ctr, j); }
  __device__ __forceinline__ double val(int64_t j) const { return f(kFVal, R.value, j); }
  __device__ __forceinline__ double gam(int64_t j) const { return f(kFGam, R.gamma, j); }
  __device__ __forceinline__ float prop(int64_t j) const {
    return j < cap ? lf[(int64_t)kFProp * cap + j] : (float)R.prop[c0 + j];
  }
  __device__ __forceinline__ double util(int64_t j) const { return f(kFUtil, R.util, j); }
  __device__ __forceinline__ double eut(int64_t j) const { return f(kFEu, eu, j); }
  __device__ __forceinline__ double won(int64_t j) const { return (double)(j < cap ? lw[j] : R.won[c0 + j]); }
  // the same fields with the LDS / global choice known at compile time (each_record's loops)
  template <bool L>
  __device__ __forceinline__ double fl(int fld, const double *g, int64_t j) const {
    if constexpr (L) return (double)lf[(int64_t)fld * cap + j];
    else return (double)(float)g[c0 + j];
  }
  template <bool L> __device__ __forceinline__ double ctr_(int64_t j) const { return fl<L>(kFCtr, R.ctr, j); }
  template <bool L> __device__ __forceinline__ double val_(int64_t j) const { return fl<L>(kFVal, R.value, j); }
  template <bool L> __device__ __forceinline__ double gam_(int64_t j) const { return fl<L>(kFGam, R.gamma, j); }
  template <bool L> __device__ __forceinline__ double util_(int64_t j) const { return fl<L>(kFUtil, R.util, j); }
  template <bool L> __device__ __forceinline__ double eut_(int64_t j) const { return fl<L>(kFEu, eu, j); }
  template <bool L> __device__ __forceinline__ float prop_(int64_t j) const {
    if constexpr (L) return lf[(int64_t)kFProp * cap + j];
    else return (float)R.prop[c0 + j];
  }
  template <bool L> __device__ __forceinline__ double won_(int64_t j) const {
    if constexpr (L) return (double)lw[j];
    else return (double)R.won[c0 + j];
  }
};

// f(j, std::true_type / std::false_type) for this thread's records j of [0, nb): the staged
// ones (j < cap, read from LDS) then the rest (global) -- two loops with the source known at
// compile time, instead of a per-field test (cap is a multiple of kDrThreads)
template <class F>
__device__ __forceinline__ void each_record(const RecView &V, int64_t nb, F &&f) {
  const int64_t ns = nb < V.cap ? nb : V.cap;
  int64_t j = threadIdx.x;
  for (; j < ns; j += kDrThreads) f(j, std::true_type());
  for (; j < nb; j += kDrThreads) f(j, std::false_type());
}

// One BCE row of the win-rate fit (its loss and gradient terms, biased: see fxb) at the model
// (w0, w1, w2, w3). One exp per row (oracle/ag_oracle_dr.c fit_winrate): e = exp(-|z|), L =
// log1p(e); p = (z >= 0 ? 1 : e) / (1 + e); -log(p) = softplus(-z) for a win, -log(1 - p) =
// softplus(z) otherwise, softplus(u) = L for u <= 0, |z| + L for u > 0 (u past 20: u).
// Branch-free main paths of exp and log1p (the same bits), the rare inputs outside them
// patched with the full functions afterwards. aug: the gamma = 0, y = 0 augmentation row.
// The row in two parts so that a record's two rows (and a lane's records) can be computed
// in one basic block before either takes its rare branch: wr_main is branch-free, wr_finish
// patches (rarely) and adds the terms.
struct WrMain {
  double z, a, e, Lz, pw, u, t, gz, x2, x3;
  bool main;  // exp and log1p on their main paths
  bool ok;    // main, and the checked terms in fxb's fast range
};
__device__ __forceinline__ WrMain wr_main(double c, double v, double g, double y, bool aug, double w0, double w1,
                                          double w2, double w3, const uint64_t *tab) {
  WrMain m;
  m.z = c * w0 + v * w1 + g * w2 + w3;
  m.a = __builtin_fabs(m.z);
  m.e = agexp::exp_main(-m.a, tab);
  bool lok;
  // p's division and log1p's c / u both divide by 1 + e: one reciprocal (ag_div.h; on the main
  // paths e >= exp(-512), c is 0 or >= 2^-81 in magnitude, |f| >= 2^-53: div_safe's range)
#if AG_DR_SHARED_DIV
  const double d1 = 1.0 + m.e, r1 = agdiv::recip(d1);
  m.Lz = aglog1p::log1p_main_t(m.e, lok, SharedDiv{r1});
  m.pw = agdiv::div_core(m.z >= 0.0 ? 1.0 : m.e, d1, r1);
#else
  m.Lz = aglog1p::log1p_main(m.e, lok);
  m.pw = (m.z >= 0.0 ? 1.0 : m.e) / (1.0 + m.e);
#endif
  m.u = y > 0.0 ? -m.z : m.z;
  m.t = fmin(m.u > 20.0 ? m.u : (m.u > 0.0 ? m.a + m.Lz : m.Lz), 100.0);
  m.gz = m.pw - y;
  // |t| <= 100, |pw - y| <= 1, ctr in [0, 1]: those terms are far inside fxb's fast range;
  // gz * value and gz * gamma are checked. ONE rare branch per row (the exp / log1p patch and
  // an out-of-range term together) instead of one per patch: the common path stays straight.
  // (the augmentation row's x3 is gz * 0: always in range, and its term is never added)
  m.x2 = (m.gz * v) * kGrid;
  m.x3 = (m.gz * g) * kGrid;
  m.main = (int)agexp::exp_in_main(m.a) & (int)lok;
  m.ok = (int)m.main & (int)fx_in(m.x2) & ((int)aug | (int)fx_in(m.x3));
  return m;
}
__device__ __forceinline__ void wr_finish(int64_t (&acc)[5], WrMain m, double c, double v, double g, double y,
                                          bool aug, const uint64_t *tab) {
  int64_t t2, t3;
  if (__builtin_expect(m.ok, 1)) {
    t2 = fxb_x(m.x2);
    t3 = fxb_x(m.x3);
  } else {
    if (!m.main) {
      m.e = agexp::exp(-m.a, tab);
      m.Lz = aglog1p::log1p(m.e);
      m.pw = (m.z >= 0.0 ? 1.0 : m.e) / (1.0 + m.e);
      m.t = fmin(m.u > 20.0 ? m.u : (m.u > 0.0 ? m.a + m.Lz : m.Lz), 100.0);
      m.gz = m.pw - y;
    }
    t2 = fxb(m.gz * v);
    t3 = fxb(m.gz * g);
  }
  addw(acc[0], fxb_fast(m.t));
  addw(acc[1], fxb_fast(m.gz * c));
  addw(acc[2], t2);
  if (!aug) addw(acc[3], t3);  // the augmentation row's g = 0 term is +-0: rounds to 0
  addw(acc[4], fxb_fast(m.gz));
}
__device__ __forceinline__ void wr_row(int64_t (&acc)[5], double c, double v, double g, double y, bool aug,
                                       double w0, double w1, double w2, double w3, const uint64_t *tab) {
  wr_finish(acc, wr_main(c, v, g, y, aug, w0, w1, w2, w3, tab), c, v, g, y, aug, tab);
}
// the rare path of a row, out of line (the main path keeps its registers): the row from the
// full exp / log1p and the general fixed-point conversion -- the same terms wr_finish adds
struct WrTerms {
  int64_t t[5];
};
__device__ __noinline__ WrTerms wr_slow(double c, double v, double g, double y, bool aug, double w0, double w1,
                                        double w2, double w3, const uint64_t *tab) {
  const double z = c * w0 + v * w1 + g * w2 + w3;
  const double a = __builtin_fabs(z);
  const double e = agexp::exp(-a, tab);
  const double Lz = aglog1p::log1p(e);
  const double pw = (z >= 0.0 ? 1.0 : e) / (1.0 + e);
  const double u = y > 0.0 ? -z : z;
  const double t = fmin(u > 20.0 ? u : (u > 0.0 ? a + Lz : Lz), 100.0);
  const double gz = pw - y;
  WrTerms r;
  r.t[0] = fxb(t);
  r.t[1] = fxb(gz * c);
  r.t[2] = fxb(gz * v);
  r.t[3] = aug ? 0 : fxb(gz * g);
  r.t[4] = fxb(gz);
  return r;
}

// a record's logged row and its gamma = 0, y = 0 augmentation row, both main paths first
__device__ __forceinline__ void wr_pair(int64_t (&acc)[5], double c, double v, double g, double y, double w0,
                                        double w1, double w2, double w3, const uint64_t *tab) {
  const WrMain A = wr_main(c, v, g, y, false, w0, w1, w2, w3, tab);
  const WrMain B = wr_main(c, v, 0.0, 0.0, true, w0, w1, w2, w3, tab);
  if (__builtin_expect((int)A.ok & (int)B.ok, 1)) {  // one branch for both rows
    addw(acc[0], fxb_fast(A.t));
    addw(acc[1], fxb_fast(A.gz * c));
    addw(acc[2], fxb_x(A.x2));
    addw(acc[3], fxb_x(A.x3));
    addw(acc[4], fxb_fast(A.gz));
    addw(acc[0], fxb_fast(B.t));
    addw(acc[1], fxb_fast(B.gz * c));
    addw(acc[2], fxb_x(B.x2));
    addw(acc[4], fxb_fast(B.gz));
  } else {
#if AG_DR_SLOW_OUTLINE
    const WrTerms ta = wr_slow(c, v, g, y, false, w0, w1, w2, w3, tab);
    const WrTerms tb = wr_slow(c, v, 0.0, 0.0, true, w0, w1, w2, w3, tab);
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      addw(acc[k], ta.t[k]);
      if (k != 3) addw(acc[k], tb.t[k]);
    }
#else
    wr_finish(acc, A, c, v, g, y, false, tab);
    wr_finish(acc, B, c, v, 0.0, 0.0, true, tab);
#endif
  }
}
// two records' four rows, main paths first, one rare branch (AG_DR_WR_RECS = 2)
__device__ __forceinline__ void wr_pair2(int64_t (&acc)[5], double c0, double v0, double g0, double y0, double c1,
                                         double v1, double g1, double y1, double w0, double w1, double w2, double w3,
                                         const uint64_t *tab) {
  const WrMain A0 = wr_main(c0, v0, g0, y0, false, w0, w1, w2, w3, tab);
  const WrMain B0 = wr_main(c0, v0, 0.0, 0.0, true, w0, w1, w2, w3, tab);
  const WrMain A1 = wr_main(c1, v1, g1, y1, false, w0, w1, w2, w3, tab);
  const WrMain B1 = wr_main(c1, v1, 0.0, 0.0, true, w0, w1, w2, w3, tab);
  if (__builtin_expect((int)A0.ok & (int)B0.ok & (int)A1.ok & (int)B1.ok, 1)) {
    addw(acc[0], fxb_fast(A0.t));
    addw(acc[1], fxb_fast(A0.gz * c0));
    addw(acc[2], fxb_x(A0.x2));
    addw(acc[3], fxb_x(A0.x3));
    addw(acc[4], fxb_fast(A0.gz));
    addw(acc[0], fxb_fast(B0.t));
    addw(acc[1], fxb_fast(B0.gz * c0));
    addw(acc[2], fxb_x(B0.x2));
    addw(acc[4], fxb_fast(B0.gz));
    addw(acc[0], fxb_fast(A1.t));
    addw(acc[1], fxb_fast(A1.gz * c1));
    addw(acc[2], fxb_x(A1.x2));
    addw(acc[3], fxb_x(A1.x3));
    addw(acc[4], fxb_fast(A1.gz));
    addw(acc[0], fxb_fast(B1.t));
    addw(acc[1], fxb_fast(B1.gz * c1));
    addw(acc[2], fxb_x(B1.x2));
    addw(acc[4], fxb_fast(B1.gz));
  } else {
    const WrTerms t[4] = {wr_slow(c0, v0, g0, y0, false, w0, w1, w2, w3, tab),
                          wr_slow(c0, v0, 0.0, 0.0, true, w0, w1, w2, w3, tab),
                          wr_slow(c1, v1, g1, y1, false, w0, w1, w2, w3, tab),
                          wr_slow(c1, v1, 0.0, 0.0, true, w0, w1, w2, w3, tab)};
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int k = 0; k < 5; ++k)
        if (k != 3 || (r & 1) == 0) addw(acc[k], t[r].t[k]);
  }
}

// a lane that ran wr_row for nrec records (both rows each): its accumulators unbiased
__device__ __forceinline__ void wr_unbias(int64_t (&acc)[5], int64_t nrec) {
  fx_unbias(acc[0], 2 * nrec);
  fx_unbias(acc[1], 2 * nrec);
  fx_unbias(acc[2], 2 * nrec);
  fx_unbias(acc[3], nrec);
  fx_unbias(acc[4], 2 * nrec);
}

// PyTorchWinRateEstimator fit (src/Bidder.py:229-252 ValueLearningBidder, :500-530
// DoublyRobustBidder): BCE (mean) over the logs plus the gamma = 0, y = 0 augmentation,
// Adam(lr 3e-3, wd 1e-6, AMSGrad), ReduceLROnPlateau(patience, factor, min_lr 1e-7),
// early stop after `wait` epochs without a 1e-6 improvement, <= 32768 epochs.
__device__ int fit_winrate(const RecView &V, const Chunk &K, TrainLds &S, Coop &C, int patience, double factor,
                           int wait, const double *adam_tab, float *tr) {
  const int tid = threadIdx.x;
  adam_reset(S);
  double lr = 3e-3;
  Plateau pl{INFINITY, 1e-4, factor, 1e-7, 0, patience};
  Stopper sp{INFINITY, -1, wait};
  const double M = 2.0 * (double)K.n;
  int e = 0;
  for (; e < kWrEpochs; ++e) {
    int64_t acc[5] = {0, 0, 0, 0, 0};
    const double w0 = (double)S.wr[0], w1 = (double)S.wr[1], w2 = (double)S.wr[2], w3 = (double)S.wr[3];
    // record j's logged row and its gamma = 0, y = 0 augmentation row together (two
    // independent chains for the scheduler; the sums are exact, so any order)
    int64_t nrec = 0;
#if AG_DR_WR_RECS == 2
    if (!(AG_DR_ABLATE_XCHG & 2)) {  // two staged records per iteration, then as each_record
      const int64_t ns = K.nb < V.cap ? K.nb : V.cap;
      int64_t j = tid;
      for (; j + kDrThreads < ns; j += 2 * kDrThreads) {
        const int64_t k = j + kDrThreads;
        wr_pair2(acc, V.template ctr_<true>(j), V.template val_<true>(j), V.template gam_<true>(j),
                 V.template won_<true>(j), V.template ctr_<true>(k), V.template val_<true>(k),
                 V.template gam_<true>(k), V.template won_<true>(k), w0, w1, w2, w3, S.tab);
        nrec += 2;
      }
      for (; j < ns; j += kDrThreads, ++nrec)
        wr_pair(acc, V.template ctr_<true>(j), V.template val_<true>(j), V.template gam_<true>(j),
                V.template won_<true>(j), w0, w1, w2, w3, S.tab);
      for (; j < K.nb; j += kDrThreads, ++nrec)
        wr_pair(acc, V.template ctr_<false>(j), V.template val_<false>(j), V.template gam_<false>(j),
                V.template won_<false>(j), w0, w1, w2, w3, S.tab);
    }
#else
    if (!(AG_DR_ABLATE_XCHG & 2))  // diagnostic: 2 = no records (the epoch's fixed cost alone)
    each_record(V, K.nb, [&](int64_t j, auto L) {
      constexpr bool l = decltype(L)::value;
      const double c = V.template ctr_<l>(j), v = V.template val_<l>(j);
      wr_pair(acc, c, v, V.template gam_<l>(j), V.template won_<l>(j), w0, w1, w2, w3, S.tab);
      ++nrec;
    });
#endif
    wr_unbias(acc, nrec);
    exact_totals<5>(acc, S, C);
    // every thread: the same loss; threads 0..3 step their parameter
    const float loss = (float)(fxv(S.tot[0], S.tot[1]) / M);
    const float g = tid < 4 ? (float)(fxv(S.tot[2 + 2 * tid], S.tot[3 + 2 * tid]) / M) : 0.0f;
    adam_step_block(S, S.wr, 4, g, e, lr, (float)1e-6, adam_tab);
    if (tid == 0 && tr) tr[e] = loss;
    plateau_step(pl, loss, lr);  // every thread keeps the same scheduler state
    const bool stop = stop_step(sp, e, loss);
    __syncthreads();
    if (stop) return e + 1;
  }
  return e;
}

// one record of the imitation fit: MSE terms of mu to the logged gamma and of softplus(sigma)
// to 0.05 (acc[12], acc[13]) and their gradient (acc[0..11]), biased
__device__ __noinline__ void imit_rec_exact(int64_t (&acc)[16], const float *pol, double c, double v, double g,
                                            const uint64_t *tab) {
  PolF f;
  policy_fwd(pol, c, v, f, tab);
  const double dm = f.mu - g, dsg = f.sp_sigma - 0.05;
  addw(acc[12], fxb(dm * dm));
  addw(acc[13], fxb(dsg * dsg));
  policy_bwd(pol, c, v, f, 2.0 * dm, 2.0 * dsg, acc, 0, tab);
}
// the common path: main-path functions and fast fixed-point terms, imit_rec_exact (the same
// terms) when a record leaves them
__device__ __forceinline__ void imit_rec(int64_t (&acc)[16], const float *pol, double c, double v, double g,
                                         const uint64_t *tab) {
  PolF f;
  const bool ok = policy_fwd_main(pol, c, v, f, tab);
  const double dm = f.mu - g, dsg = f.sp_sigma - 0.05;
  double d[14];
  policy_terms(pol, c, v, f, 2.0 * dm, 2.0 * dsg, d);
  d[12] = dm * dm;
  d[13] = dsg * dsg;
  if (__builtin_expect(!fx_add_fast<14>(acc, d, ok), 0)) {  // (a separate array: acc stays in registers)
    int64_t t[16] = {};
    imit_rec_exact(t, pol, c, v, g, tab);
#pragma unroll
    for (int k = 0; k < 14; ++k) addw(acc[k], t[k]);
  }
}

// BidShadingContextualBandit.initialise_policy (src/Models.py:106-137): imitation of the
// logging policy, MSE of mu to the logged gammas + MSE of softplus(sigma) (without
// min_sigma) to 0.05; Adam(lr 1e-3, wd 1e-4, AMSGrad), early stop after 512 epochs.
__device__ int fit_imitation(const RecView &V, const Chunk &K, TrainLds &S, Coop &C, const double *adam_tab,
                             float *tr) {
  const int tid = threadIdx.x;
  adam_reset(S);
  Stopper sp{INFINITY, -1, 512};
  const double n = (double)K.n;
  int e = 0;
  for (; e < kInitEpochs; ++e) {
    int64_t acc[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = 0;
    each_record(V, K.nb, [&](int64_t j, auto L) {
      constexpr bool l = decltype(L)::value;
      imit_rec(acc, S.pol, V.template ctr_<l>(j), V.template val_<l>(j), V.template gam_<l>(j), S.tab);
    });
    const int64_t nrec = K.nb > tid ? (K.nb - tid + kDrThreads - 1) / kDrThreads : 0;
#pragma unroll
    for (int q = 0; q < 14; ++q) fx_unbias(acc[q], nrec);
    exact_totals<16>(acc, S, C);
    const float loss = (float)(fxv(S.tot[24], S.tot[25]) / n + fxv(S.tot[26], S.tot[27]) / n);
    const float g = tid < 12 ? (float)(fxv(S.tot[2 * tid], S.tot[2 * tid + 1]) / n) : 0.0f;
    adam_step_block(S, S.pol, 12, g, e, 1e-3, (float)1e-4, adam_tab);
    if (tid == 0 && tr) tr[e] = loss;
    const bool stop = stop_step(sp, e, loss);
    __syncthreads();
    if (stop) return e + 1;
  }
  return e;
}

// one record of the DR policy fit (fit_dr): its loss term (acc[12]) and gradient (acc[0..11]),
// biased; du = utility - estimated utility, ep = the epoch's rsample draw
__device__ __noinline__ void dr_rec_exact(int64_t (&acc)[16], const float *pol, const float *wr, double c,
                                          double v, double g, float prop, double du, double ep, const uint64_t *tab) {
  const double inv_sqrt2pi = 1.0 / __builtin_sqrt(2.0 * 3.141592653589793);
  PolF f;
  policy_fwd(pol, c, v, f, tab);
  const double mu = f.mu, sg = f.sigma;
  const double zz = (mu - g) / sg;
  const double pdf_raw = exp_fast(-(zz * zz) / 2.0, tab) / sg * inv_sqrt2pi;
  const double pi = pdf_raw < 1e-30 ? 1e-30 : pdf_raw;
  const double p0 = (double)fmaxf(prop, 1e-15f);
  const double iw = pi / p0;
  const double iwc = iw < 1.0 / 50.0 ? 1.0 / 50.0 : (iw > 50.0 ? 50.0 : iw);
  const double raw = mu + sg * ep;
  const double gs = raw < 0.0 ? 0.0 : (raw > 1.0 ? 1.0 : raw);
  const double zw = c * (double)wr[0] + v * (double)wr[1] + gs * (double)wr[2] + (double)wr[3];
  const double Wv = 1.0 / (1.0 + exp_fast(-zw, tab));
  const double V = c * v;
  addw(acc[12], fxb(-(du * iwc + Wv * (V - V * gs))));
  double dpi_dmu = 0.0, dpi_dsg = 0.0;
  if (pdf_raw >= 1e-30 && iw >= 1.0 / 50.0 && iw <= 50.0) {
    const double k = du / p0;
    dpi_dmu = k * pdf_raw * (g - mu) / (sg * sg);
    dpi_dsg = k * pdf_raw * ((g - mu) * (g - mu) / (sg * sg * sg) - 1.0 / sg);
  }
  double ddm = 0.0;
  if (raw >= 0.0 && raw <= 1.0) ddm = -Wv * V + (V - V * gs) * Wv * (1.0 - Wv) * (double)wr[2];
  policy_bwd(pol, c, v, f, -(dpi_dmu + ddm), -(dpi_dsg + ddm * ep), acc, 0, tab);
}
// the common path of dr_rec_exact (main-path exp / softplus, fast fixed-point terms; the
// same expressions), dr_rec_exact when a record leaves it
__device__ __forceinline__ void dr_rec(int64_t (&acc)[16], const float *pol, const float *wr, double c, double v,
                                       double g, float prop, double du, double ep, const uint64_t *tab) {
  const double inv_sqrt2pi = 1.0 / __builtin_sqrt(2.0 * 3.141592653589793);
  PolF f;
  bool ok = policy_fwd_main(pol, c, v, f, tab);
  const double mu = f.mu, sg = f.sigma;
  const double p0 = (double)fmaxf(prop, 1e-15f);
#if AG_DR_SHARED_DIV
  // three divisions by sg, two by p0: one reciprocal each (ag_div.h; a record whose operands
  // leave div_safe's range takes dr_rec_exact)
  const double rsg = agdiv::recip(sg), rp0 = agdiv::recip(p0);
  const double zz = agdiv::div_core(mu - g, sg, rsg);
  const double xp = -(zz * zz) / 2.0;
  const double ex = agexp::exp_main(xp, tab);
  const double pdf_raw = agdiv::div_core(ex, sg, rsg) * inv_sqrt2pi;
  const double pi = pdf_raw < 1e-30 ? 1e-30 : pdf_raw;
  const double iw = agdiv::div_core(pi, p0, rp0);
  ok = (int)ok & (int)agdiv::div_safe(mu - g, sg) & (int)agdiv::div_safe(ex, sg) & (int)agdiv::div_safe(pi, p0) &
       (int)agdiv::div_safe(du, p0);
#else
  const double zz = (mu - g) / sg;
  const double xp = -(zz * zz) / 2.0;
  const double pdf_raw = agexp::exp_main(xp, tab) / sg * inv_sqrt2pi;
  const double pi = pdf_raw < 1e-30 ? 1e-30 : pdf_raw;
  const double iw = pi / p0;
#endif
  const double iwc = iw < 1.0 / 50.0 ? 1.0 / 50.0 : (iw > 50.0 ? 50.0 : iw);
  const double raw = mu + sg * ep;
  const double gs = raw < 0.0 ? 0.0 : (raw > 1.0 ? 1.0 : raw);
  const double zw = c * (double)wr[0] + v * (double)wr[1] + gs * (double)wr[2] + (double)wr[3];
  const double Wv = 1.0 / (1.0 + agexp::exp_main(-zw, tab));
  ok = (int)ok & (int)agexp::exp_in_main(xp) & (int)agexp::exp_in_main(-zw);
  const double V = c * v;
  double d[13];
  d[12] = -(du * iwc + Wv * (V - V * gs));
  double dpi_dmu = 0.0, dpi_dsg = 0.0;
  if (pdf_raw >= 1e-30 && iw >= 1.0 / 50.0 && iw <= 50.0) {
#if AG_DR_SHARED_DIV
    const double k = agdiv::div_core(du, p0, rp0);
    dpi_dmu = k * pdf_raw * (g - mu) / (sg * sg);
    dpi_dsg = k * pdf_raw * ((g - mu) * (g - mu) / (sg * sg * sg) - agdiv::div_core(1.0, sg, rsg));
#else
    const double k = du / p0;
    dpi_dmu = k * pdf_raw * (g - mu) / (sg * sg);
    dpi_dsg = k * pdf_raw * ((g - mu) * (g - mu) / (sg * sg * sg) - 1.0 / sg);
#endif
  }
  double ddm = 0.0;
  if (raw >= 0.0 && raw <= 1.0) ddm = -Wv * V + (V - V * gs) * Wv * (1.0 - Wv) * (double)wr[2];
  policy_terms(pol, c, v, f, -(dpi_dmu + ddm), -(dpi_dsg + ddm * ep), d);
  if (__builtin_expect(!fx_add_fast<13>(acc, d, ok), 0)) {
    int64_t t[16] = {};
    dr_rec_exact(t, pol, wr, c, v, g, prop, du, ep, tab);
#pragma unroll
    for (int k = 0; k < 13; ++k) addw(acc[k], t[k]);
  }
}

// DoublyRobustBidder's policy fit (src/Bidder.py:562-590, src/Models.py:201-218): loss
// -mean((u - u^) clip(pi / pi0, 1/50, 50) + W(ctr, value, g~) (V - V g~)), g~ = clip(mu +
// sigma eps, 0, 1); Adam(lr 7e-3, wd 1e-4, AMSGrad), ReduceLROnPlateau(patience 100, factor
// 0.2, min_lr 1e-8, threshold 5e-3), early stop after 512 epochs, <= 32768 epochs.
__device__ int fit_dr(const RecView &V, const Chunk &K, TrainLds &S, Coop &C,
                      const FitNoise &F, const double *adam_tab, float *tr) {
  const int tid = threadIdx.x;
  adam_reset(S);
  double lr = 7e-3;
  Plateau pl{INFINITY, 5e-3, 0.2, 1e-8, 0, 100};
  Stopper sp{INFINITY, -1, 512};
  const double n = (double)K.n;
  int e = 0;
  for (; e < kDrEpochs && e < F.epochs; ++e) {
    int64_t acc[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = 0;
    each_record(V, K.nb, [&](int64_t j, auto L) {
      constexpr bool l = decltype(L)::value;
      dr_rec(acc, S.pol, S.wr, V.template ctr_<l>(j), V.template val_<l>(j), V.template gam_<l>(j),
             V.template prop_<l>(j), V.template util_<l>(j) - V.template eut_<l>(j), fit_eps(F, e, K.c0 + j), S.tab);
    });
    const int64_t nrec = K.nb > tid ? (K.nb - tid + kDrThreads - 1) / kDrThreads : 0;
#pragma unroll
    for (int q = 0; q < 13; ++q) fx_unbias(acc[q], nrec);
    exact_totals<16>(acc, S, C);
    const float loss = (float)(fxv(S.tot[24], S.tot[25]) / n);
    const float g = tid < 12 ? (float)(fxv(S.tot[2 * tid], S.tot[2 * tid + 1]) / n) : 0.0f;
    adam_step_block(S, S.pol, 12, g, e, lr, (float)1e-4, adam_tab);
    if (tid == 0 && tr) tr[e] = loss;
    plateau_step(pl, loss, lr);
    const bool stop = stop_step(sp, e, loss);
    if (tid == 0 && loss != loss) S.stop = 1;  // NaN: the reference exits (src/Bidder.py:592-600)
    __syncthreads();
    if (stop || S.stop) return e + 1;
  }
  if (e < kDrEpochs && tid == 0) S.exhausted = 1;
  return e;
}

// one record of the ValueLearningBidder policy fit (fit_dm), biased
__device__ __noinline__ void dm_rec_exact(int64_t (&acc)[16], const float *pol, const float *wr, double c,
                                          double v, double ep, const uint64_t *tab) {
  PolF f;
  policy_fwd(pol, c, v, f, tab);
  const double raw = f.mu + f.sigma * ep;
  const double gs = raw < 0.0 ? 0.0 : (raw > 1.0 ? 1.0 : raw);
  const double zw = c * (double)wr[0] + v * (double)wr[1] + gs * (double)wr[2] + (double)wr[3];
  const double Wv = 1.0 / (1.0 + exp_fast(-zw, tab));
  const double V = c * v;
  addw(acc[12], fxb(-(Wv * (V - V * gs))));
  double ddm = 0.0;
  if (raw >= 0.0 && raw <= 1.0) ddm = -Wv * V + (V - V * gs) * Wv * (1.0 - Wv) * (double)wr[2];
  policy_bwd(pol, c, v, f, -ddm, -(ddm * ep), acc, 0, tab);
}
// the common path of dm_rec_exact, dm_rec_exact when a record leaves it
__device__ __forceinline__ void dm_rec(int64_t (&acc)[16], const float *pol, const float *wr, double c, double v,
                                       double ep, const uint64_t *tab) {
  PolF f;
  bool ok = policy_fwd_main(pol, c, v, f, tab);
  const double raw = f.mu + f.sigma * ep;
  const double gs = raw < 0.0 ? 0.0 : (raw > 1.0 ? 1.0 : raw);
  const double zw = c * (double)wr[0] + v * (double)wr[1] + gs * (double)wr[2] + (double)wr[3];
  const double Wv = 1.0 / (1.0 + agexp::exp_main(-zw, tab));
  ok = (int)ok & (int)agexp::exp_in_main(-zw);
  const double V = c * v;
  double d[13];
  d[12] = -(Wv * (V - V * gs));
  double ddm = 0.0;
  if (raw >= 0.0 && raw <= 1.0) ddm = -Wv * V + (V - V * gs) * Wv * (1.0 - Wv) * (double)wr[2];
  policy_terms(pol, c, v, f, -ddm, -(ddm * ep), d);
  if (__builtin_expect(!fx_add_fast<13>(acc, d, ok), 0)) {
    int64_t t[16] = {};
    dm_rec_exact(t, pol, wr, c, v, ep, tab);
#pragma unroll
    for (int k = 0; k < 13; ++k) addw(acc[k], t[k]);
  }
}

// ValueLearningBidder's policy fit (inference 'policy', src/Bidder.py:258-303): loss
// -mean(W(ctr, value, g~) (V - V g~)), g~ = clip(mu + sigma eps, 0, 1); Adam(lr 2e-3, wd
// 1e-6, AMSGrad), ReduceLROnPlateau(patience 100, factor 0.1, min_lr 1e-7), early stop after
// 256 epochs, <= 16384 epochs. Exact fixed-point sums (bounded terms).
__device__ int fit_dm(const RecView &V, const Chunk &K, TrainLds &S, Coop &C, const FitNoise &F,
                      const double *adam_tab, float *tr) {
  const int tid = threadIdx.x;
  adam_reset(S);
  double lr = 2e-3;
  Plateau pl{INFINITY, 1e-4, 0.1, 1e-7, 0, 100};
  Stopper sp{INFINITY, -1, 256};
  const double n = (double)K.n;
  int e = 0;
  for (; e < kInitEpochs && e < F.epochs; ++e) {
    int64_t acc[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = 0;
    if (!(AG_DR_ABLATE_XCHG & 2))
    each_record(V, K.nb, [&](int64_t j, auto L) {
      constexpr bool l = decltype(L)::value;
      dm_rec(acc, S.pol, S.wr, V.template ctr_<l>(j), V.template val_<l>(j), fit_eps(F, e, K.c0 + j), S.tab);
    });
    const int64_t nrec = K.nb > tid ? (K.nb - tid + kDrThreads - 1) / kDrThreads : 0;
#pragma unroll
    for (int q = 0; q < 13; ++q) fx_unbias(acc[q], nrec);
    exact_totals<16>(acc, S, C);
    const float loss = (float)(fxv(S.tot[24], S.tot[25]) / n);
    const float g = tid < 12 ? (float)(fxv(S.tot[2 * tid], S.tot[2 * tid + 1]) / n) : 0.0f;
    adam_step_block(S, S.pol, 12, g, e, lr, (float)1e-6, adam_tab);
    if (tid == 0 && tr) tr[e] = loss;
    plateau_step(pl, loss, lr);
    const bool stop = stop_step(sp, e, loss);
    __syncthreads();
    if (stop) return e + 1;
  }
  if (e < kInitEpochs && tid == 0) S.exhausted = 1;
  return e;
}

// per-record gradient of a policy loss term from d/dmu and d/dsigma (policy_bwd's order)
__device__ __forceinline__ void policy_grad(const float *p, double c, double v, const PolF &f, double dmu,
                                            double dsigma, double (&G)[14], const uint64_t *tab) {
  const double dam = dmu * dsoftplus_e(f.am, f.eam), das = dsigma * dsoftplus_e(f.as, f.eas);
  double ds[2];
  ds[0] = dam * (double)p[6] + das * (double)p[9];
  ds[1] = dam * (double)p[7] + das * (double)p[10];
  G[6] += dam * f.s[0];
  G[7] += dam * f.s[1];
  G[8] += dam;
  G[9] += das * f.s[0];
  G[10] += das * f.s[1];
  G[11] += das;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const double dh = ds[j] * dsoftplus_e(f.h[j], f.eh[j]);
    G[2 * j] += dh * c;
    G[2 * j + 1] += dh * v;
    G[4 + j] += dh;
  }
}

// PolicyLearningBidder's policy fit (src/Bidder.py:376-407, the losses of src/Models.py:
// 174-199; AG_PL_LOSS_* kinds): Adam(lr 2e-3, wd 1e-4, AMSGrad), ReduceLROnPlateau
// (patience 100, factor 0.2, min_lr 1e-8), early stop after 512 epochs, <= 16384 epochs.
// oracle/ag_oracle_dr.c pl_epoch, term for term, with the same fixed-order sums.
__device__ int fit_pl(const RecView &V, const Chunk &K, TrainLds &S, Coop &C, int kind, const double *adam_tab,
                      float *tr) {
  const int tid = threadIdx.x;
  adam_reset(S);
  double lr = 2e-3;
  Plateau pl{INFINITY, 1e-4, 0.2, 1e-8, 0, 100};
  Stopper sp{INFINITY, -1, 512};
  const double inv_sqrt2pi = 1.0 / __builtin_sqrt(2.0 * 3.141592653589793);
  const double n = (double)K.n;
  int e = 0;
  for (; e < kInitEpochs; ++e) {
    double acc[14];
#pragma unroll
    for (int j = 0; j < 14; ++j) acc[j] = 0.0;
    for (int64_t j = tid; j < K.nb; j += kDrThreads) {
      const double c = V.ctr(j), v = V.val(j), g = V.gam(j);
      PolF f;
      policy_fwd_fast(S.pol, c, v, f, S.tab);
      const double mu = f.mu, sg = f.sigma;
      const double zz = (mu - g) / sg;
      const double pdf_raw = exp_fast(-(zz * zz) / 2.0, S.tab) / sg * inv_sqrt2pi;
      const double pi = pdf_raw < 1e-30 ? 1e-30 : pdf_raw;
      const double p0 = (double)fmaxf(V.prop(j), 1e-15f);
      const double u = V.util(j);
      double term = 0.0, kl = 0.0, dpi = 0.0, dmu = 0.0, dsg = 0.0;
      if (kind == AG_PL_LOSS_REINFORCE) {
        term = -(pi * u);
        dpi = -u;
      } else if (kind == AG_PL_LOSS_REINFORCE_OFFPOLICY || kind == AG_PL_LOSS_TRPO) {
        term = -((pi / p0) * u);
        dpi = -u / p0;
        if (kind == AG_PL_LOSS_TRPO) {
          kl = (sg * sg + (mu - g) * (mu - g)) / (2.0 * sg * sg) - 0.5;
          dmu = 5e-2 * ((mu - g) / (sg * sg));
          dsg = 5e-2 * (-((mu - g) * (mu - g)) / (sg * sg * sg));
        }
      } else {  // PPO
        const double iw = pi / p0;
        const bool in_range = iw >= 1.0 / 50.0 && iw <= 50.0;
        const double iwc = iw < 1.0 / 50.0 ? 1.0 / 50.0 : (iw > 50.0 ? 50.0 : iw);
        const double A = iw * u, Bc = iwc * u;
        term = -(A < Bc ? A : Bc);
        dpi = (in_range || A < Bc) ? -u / p0 : 0.0;
      }
      if (pdf_raw >= 1e-30 && dpi != 0.0) {
        dmu += dpi * pdf_raw * (g - mu) / (sg * sg);
        dsg += dpi * pdf_raw * ((g - mu) * (g - mu) / (sg * sg * sg) - 1.0 / sg);
      }
      double gr[14];
#pragma unroll
      for (int q = 0; q < 14; ++q) gr[q] = 0.0;
      policy_grad(S.pol, c, v, f, dmu, dsg, gr, S.tab);
#pragma unroll
      for (int q = 0; q < 12; ++q) acc[q] += gr[q];
      acc[12] += term;
      acc[13] += kl;
    }
    float_totals<14>(acc, S, C);
    const float loss = (float)(S.ftot[12] / n + (S.ftot[13] / n) * 5e-2);
    const float g = tid < 12 ? (float)(S.ftot[tid] / n) : 0.0f;
    adam_step_block(S, S.pol, 12, g, e, lr, (float)1e-4, adam_tab);
    if (tid == 0 && tr) tr[e] = loss;
    plateau_step(pl, loss, lr);
    const bool stop = stop_step(sp, e, loss);
    if (tid == 0 && loss != loss) S.stop = 1;  // NaN: the reference exits (src/Bidder.py:409-417)
    __syncthreads();
    if (stop || S.stop) return e + 1;
  }
  return e;
}

// The workgroups of the learning bidders (ValueLearning, PolicyLearning, DoublyRobust): block
// b trains agent blk_agent[b] as workgroup blk_rank[b] of agent_nblk[agent] over the agent's
// records, running its fits in the reference's order, in two launches:
//   PH = 0: the win-rate fits (ValueLearning, DoublyRobust; a ValueLearningBidder without
//           wins falls back, status 1) -> wr_ws, epochs [a][0]; a register-lean loop, 4 waves
//           per SIMD;
//   PH = 1: everything after (estimated utilities, imitation, the policy fits) from wr_ws,
//           then the agent's state.
// status: 0 trained, 1 ValueLearningBidder fallback (no wins: nothing trained), -1 no logs,
// -2 NaN loss, -3 out of noise epochs (state not written); epochs [3] = (win-rate,
// imitation, policy fit); traces [3][32768] (workgroup 0).
template <int PH>
__global__ __launch_bounds__(kDrThreads, PH == 0 ? AG_DR_PH0_MIN_WAVES : AG_DR_PH1_MIN_WAVES) void k_bidder_train(
    const int32_t *__restrict__ bkind, const int32_t *__restrict__ bmode, const int32_t *__restrict__ blk_agent,
    const int32_t *__restrict__ blk_rank, const int32_t *__restrict__ agent_nblk,
    const int64_t *__restrict__ offsets, DrRecords R0, double *__restrict__ eu_ws, float *__restrict__ state,
    float *__restrict__ wr_ws, const int32_t *__restrict__ initialised, const float *__restrict__ noise,
    const int64_t *__restrict__ noise_off, int noise_epochs, uint64_t noise_seed, const double *__restrict__ adam_tab,
    int32_t *__restrict__ epochs_out, int32_t *__restrict__ status, float *__restrict__ traces,
    int64_t *__restrict__ partials, unsigned *__restrict__ barriers, const int32_t *__restrict__ bar_off, int nf,
    int64_t cap) {
  const int a = blk_agent[blockIdx.x], rank = blk_rank[blockIdx.x], nblk = agent_nblk[a];
  const int tid = threadIdx.x;
  const int bk = bkind[a];
  const int64_t s0 = offsets[a], n = offsets[a + 1] - s0;
  const bool lead = rank == 0;
  const bool has_wr = bk == AG_BIDDER_DOUBLY_ROBUST || bk == AG_BIDDER_VALUE_LEARNING;
  if (n == 0) {
    // no logs: a ValueLearningBidder falls back (its won mask sums to 0, src/Bidder.py:206-
    // 211); the other learners fail in the reference
    if (PH == 1 && lead && tid == 0) {
      epochs_out[3 * a] = epochs_out[3 * a + 1] = epochs_out[3 * a + 2] = 0;
      status[a] = bk == AG_BIDDER_VALUE_LEARNING ? 1 : -1;
    }
    return;
  }
  if (PH == 1 && bk == AG_BIDDER_VALUE_LEARNING && status[a] == 1) return;  // fallback: state unchanged
  __shared__ TrainLds S;
  for (int i = tid; i < 256; i += kDrThreads) S.tab[i] = ag_exp_tab[i];
  float *st = state + (size_t)a * 16;
  if (tid < 4) S.wr[tid] = (PH == 1 && has_wr) ? wr_ws[(size_t)a * 4 + tid] : st[tid];
  if (tid < 12) S.pol[tid] = st[4 + tid];
  if (tid == 0) S.stop = S.exhausted = 0;
  __syncthreads();
  DrRecords R{R0.ctr + s0, R0.value + s0, R0.gamma + s0, R0.prop + s0, R0.util + s0, R0.won + s0};
  const int64_t per = (n + nblk - 1) / nblk;
  const int64_t c0 = (int64_t)rank * per < n ? (int64_t)rank * per : n;
  const Chunk K{c0, (c0 + per < n ? c0 + per : n) - c0, n};
  // the agent's exchange region [2][nblk][32] (its workgroups have consecutive block indices)
  // the agent's exchange region: [2][nblk][32] parity buffers, then [nblk][32] accumulator rows
  int64_t *preg = partials + (size_t)(blockIdx.x - rank) * 3 * 32;
  unsigned *abar = barriers + (size_t)bar_off[a] * kBarLineWords;
  Coop C{rank, nblk, preg, abar, 0, preg + (size_t)2 * nblk * 32, abar + (size_t)bar_lines(nblk) * kBarLineWords, 0u};
  if (tid < 64) S.gprev[tid >> 5][tid & 31] = 0;
  // stage the chunk's first `cap` records in LDS (the fields this phase's fits read)
  extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];
  float *lf = reinterpret_cast<float *>(s_dyn);
  uint8_t *lw = reinterpret_cast<uint8_t *>(lf + (size_t)nf * cap);
  {
    const int64_t ns = K.nb < cap ? K.nb : cap;
    const bool full = PH == 1 && bk != AG_BIDDER_VALUE_LEARNING;  // propensity, utility
    const bool won = PH == 0 || bk == AG_BIDDER_DOUBLY_ROBUST;
    for (int64_t j = tid; j < ns; j += kDrThreads) {
      const int64_t i = K.c0 + j;
      lf[kFCtr * cap + j] = (float)R.ctr[i];
      lf[kFVal * cap + j] = (float)R.value[i];
      lf[kFGam * cap + j] = (float)R.gamma[i];
      if (full) {
        lf[kFProp * cap + j] = (float)R.prop[i];
        lf[kFUtil * cap + j] = (float)R.util[i];
      }
      if (won) lw[j] = R.won[i];
    }
    __syncthreads();
  }
  const RecView V{R, eu_ws + s0, K.c0, lf, lw, cap};
  float *tr = (traces && lead) ? traces + (size_t)a * 3 * kDrEpochs : nullptr;
  if constexpr (PH == 0) {
    int ep0 = 0, stat = 0;
    if (bk == AG_BIDDER_DOUBLY_ROBUST) {
      ep0 = fit_winrate(V, K, S, C, 256, 0.2, 1024, adam_tab, tr);
    } else {  // ValueLearningBidder
      int64_t acc[1] = {0};
      each_record(V, K.nb, [&](int64_t j, auto L) { acc[0] += V.template won_<decltype(L)::value>(j) != 0.0 ? 1 : 0; });
      exact_totals<1>(acc, S, C);
      if (S.tot[0] == 0 && S.tot[1] == 0)
        stat = 1;  // src/Bidder.py:206-211: revert to Gaussian shading, nothing trained
      else
        ep0 = fit_winrate(V, K, S, C, 100, 0.1, 512, adam_tab, tr);
    }
    if (!lead) return;
    if (tid == 0) {
      epochs_out[3 * a] = ep0;
      status[a] = stat;
    }
    if (tid < 4) wr_ws[(size_t)a * 4 + tid] = S.wr[tid];
  } else {
    const FitNoise F{noise ? noise + noise_off[a] : nullptr, n, noise_seed, (uint32_t)a,
                     noise ? noise_epochs : 1 << 30};
    int ep1 = 0, ep2 = 0;
    int stat = 0;
    if (bk == AG_BIDDER_DOUBLY_ROBUST) {
      // estimated utilities of this workgroup's records with the fitted model (src/Bidder.py:541-546)
      double *eu = eu_ws + s0;
      for (int64_t j = tid; j < K.nb; j += kDrThreads) {
        const int64_t i = K.c0 + j;
        const double c = (double)(float)R.ctr[i], v = (double)(float)R.value[i], g = (double)(float)R.gamma[i];
        const double z = c * (double)S.wr[0] + v * (double)S.wr[1] + g * (double)S.wr[2] + (double)S.wr[3];
        const float W = (float)(1.0 / (1.0 + agexp::exp(-z, S.tab)));
        const double Vv = R.ctr[i] * R.value[i], P = R.ctr[i] * R.value[i] * R.gamma[i];
        eu[i] = (double)W * (Vv - P);
        if (j < cap) lf[kFEu * cap + j] = (float)eu[i];
      }
      __syncthreads();
      if (!initialised[a]) ep1 = fit_imitation(V, K, S, C, adam_tab, tr ? tr + kDrEpochs : nullptr);
      ep2 = fit_dr(V, K, S, C, F, adam_tab, tr ? tr + 2 * kDrEpochs : nullptr);
      stat = S.stop ? -2 : 0;
    } else if (bk == AG_BIDDER_VALUE_LEARNING) {
      if (bmode[a] == AG_VL_POLICY) ep2 = fit_dm(V, K, S, C, F, adam_tab, tr ? tr + 2 * kDrEpochs : nullptr);
    } else {  // PolicyLearningBidder
      if (!initialised[a]) ep1 = fit_imitation(V, K, S, C, adam_tab, tr ? tr + kDrEpochs : nullptr);
      ep2 = fit_pl(V, K, S, C, bmode[a], adam_tab, tr ? tr + 2 * kDrEpochs : nullptr);
      stat = S.stop ? -2 : 0;
    }
    __syncthreads();
    if (S.exhausted) stat = -3;  // not applied: the caller supplies more noise epochs
    if (!lead) return;
    if (tid == 0) {
      epochs_out[3 * a + 1] = ep1;
      epochs_out[3 * a + 2] = ep2;
      status[a] = stat;
    }
    if (stat == -3) return;
    if (tid < 4) st[tid] = S.wr[tid];
    if (tid < 12) st[4 + tid] = S.pol[tid];
  }
}

// ---------------------------------------------------------------------------------------
// Resumable, record-parallel training (ag_bidder_rp_*): the exact-sum learners' fits --
// ValueLearningBidder (win count, win-rate fit, 'policy' fit) and DoublyRobustBidder (win-rate
// fit, estimated utilities, imitation, DR policy fit) -- as ONE LAUNCH PER EPOCH, the whole
// training state of a learner (FitSt) in HBM between launches. Launch k, every workgroup of
// every learner:
//   1. steps the learner's state with the summed partials of launch k - 1 (summed over this
//      rank's workgroups by launch k - 1's tree root, then over the ranks by the caller's
//      all-reduce of those int64 words): loss, Adam, scheduler, early stop and the move to the
//      next fit, exactly as the persistent fits do it -- every workgroup computes the same
//      step from the same integers;
//   2. adds its records' exact fixed-point terms of the next epoch at the new state;
//   3. sums them up the agent's combining tree without waiting (agent_reduce_nowait): the
//      root stores the rank's totals for launch k + 1 (or the caller's all-reduce).
// No workgroup waits for another: no co-residency, no device-wide barrier. The sums are
// integers, so a rank holding a shard of the records (its records' global indices keep the
// synthetic rsample draws) steps to the model one process fits on all of them, bit for bit --
// and that model is the persistent fits' (k_bidder_train), which the GPU tests check.
// A policy fit that runs out of host-drawn noise epochs (ag_bidder_rp_noise) waits, with its
// state kept, for the next window: the drop-in update draws the reference's torch noise
// window by window and never re-runs a fit.
enum { kFitWins = 0, kFitWr, kFitEu, kFitInit, kFitPol, kFitDone };
struct FitSt {
  int32_t fit, epoch, status, have_tot, need_noise, pad0;
  int32_t ep[3], pad1;
  double lr;
  Plateau pl;
  Stopper sp;
  float wr[4], pol[12];
  AdamState adam;
};

// the learner's state on entering `fit` (the persistent fits' initialisations)
__device__ __forceinline__ void fit_enter(FitSt &st, int fit, int bk, int mode) {
  st.fit = fit;
  st.epoch = 0;
  for (int j = 0; j < 16; ++j) st.adam.ea[j] = st.adam.es[j] = st.adam.mx[j] = 0.0f;
  const bool dr = bk == AG_BIDDER_DOUBLY_ROBUST;
  if (fit == kFitWr) {
    st.lr = 3e-3;
    st.pl = dr ? Plateau{INFINITY, 1e-4, 0.2, 1e-7, 0, 256} : Plateau{INFINITY, 1e-4, 0.1, 1e-7, 0, 100};
    st.sp = Stopper{INFINITY, -1, dr ? 1024 : 512};
  } else if (fit == kFitInit) {
    st.lr = 1e-3;
    st.sp = Stopper{INFINITY, -1, 512};
  } else if (fit == kFitPol) {
    if (dr) {
      st.lr = 7e-3;
      st.pl = Plateau{INFINITY, 5e-3, 0.2, 1e-8, 0, 100};
      st.sp = Stopper{INFINITY, -1, 512};
    } else {
      st.lr = 2e-3;
      st.pl = Plateau{INFINITY, 1e-4, 0.1, 1e-7, 0, 100};
      st.sp = Stopper{INFINITY, -1, 256};
    }
  }
  (void)mode;
}

// the fit after `st.fit` ended (the reference's order, src/Bidder.py:229-325, :500-615)
__device__ __forceinline__ void fit_after(FitSt &st, int bk, int mode, int init) {
  int nxt = kFitDone;
  switch (st.fit) {
    case kFitWins: nxt = kFitWr; break;
    case kFitWr: nxt = bk == AG_BIDDER_DOUBLY_ROBUST ? kFitEu : (mode == AG_VL_POLICY ? kFitPol : kFitDone); break;
    case kFitEu: nxt = init ? kFitPol : kFitInit; break;
    case kFitInit: nxt = kFitPol; break;
    default: nxt = kFitDone;
  }
  fit_enter(st, nxt, bk, mode);
}

__device__ __forceinline__ int fit_max_epochs(int fit, int bk) {
  if (fit == kFitWr) return kWrEpochs;
  if (fit == kFitInit) return kInitEpochs;
  return bk == AG_BIDDER_DOUBLY_ROBUST ? kDrEpochs : kInitEpochs;
}

// step 1 (thread 0 with threads 0..15 for Adam): the learner's state after the epoch whose
// summed partials are tot (hi, lo pairs); n: the learner's records over all ranks
__device__ __forceinline__ void fit_step(FitSt &st, const int64_t *tot, double n, int bk, int mode, int init, const double *adam_tab,
                         float *s_grad, float *s_loss, int *s_np, float *tr, const double *bcp = nullptr) {
  const int tid = threadIdx.x;
  if (tid == 0) {
    *s_np = 0;
    if (st.fit == kFitWins) {
      if (tot[0] == 0 && tot[1] == 0) {  // no wins: revert to Gaussian shading (src/Bidder.py:206-211)
        st.status = 1;
        fit_enter(st, kFitDone, bk, mode);
      } else {
        fit_after(st, bk, mode, init);
      }
    } else if (st.fit == kFitWr) {
      const double M = 2.0 * n;
      *s_loss = (float)(fxv(tot[0], tot[1]) / M);
      for (int j = 0; j < 4; ++j) s_grad[j] = (float)(fxv(tot[2 + 2 * j], tot[3 + 2 * j]) / M);
      *s_np = 4;
    } else {  // imitation / policy fits: 12 parameters
      *s_loss = st.fit == kFitInit ? (float)(fxv(tot[24], tot[25]) / n + fxv(tot[26], tot[27]) / n)
                                   : (float)(fxv(tot[24], tot[25]) / n);
      for (int j = 0; j < 12; ++j) s_grad[j] = (float)(fxv(tot[2 * j], tot[2 * j + 1]) / n);
      *s_np = 12;
    }
  }
  __syncthreads();
  const int np = *s_np;
  if (np == 0) return;
  // Adam: thread j steps parameter j (adam_step_block's arithmetic)
  const int e = st.epoch;
  const float wd = st.fit == kFitWr ? (float)1e-6 : (st.fit == kFitInit || bk == AG_BIDDER_DOUBLY_ROBUST ? (float)1e-4
                                                                                                         : (float)1e-6);
  double bc1;
  float bc2f;
  if (bcp) {  // adam_tab[e], adam_tab[kDrEpochs + e] fetched by the caller
    bc1 = bcp[0];
    bc2f = (float)bcp[1];
  } else {
    bias_corrections(e, adam_tab, bc2f, bc1);
  }
  const float neg_step = (float)(-(st.lr / bc1));
  float *par = st.fit == kFitWr ? st.wr : st.pol;
  __syncthreads();
  if (tid < np) {
    float p = par[tid];
    adam_param(p, s_grad[tid], tid, st.adam, neg_step, bc2f, wd);
    par[tid] = p;
  }
  __syncthreads();
  if (tid == 0) {
    const float loss = *s_loss;
    if (tr) tr[e] = loss;
    if (st.fit != kFitInit) plateau_step(st.pl, loss, st.lr);
    const bool stop = stop_step(st.sp, e, loss);
    const bool nan = loss != loss && st.fit == kFitPol && bk == AG_BIDDER_DOUBLY_ROBUST;
    st.epoch = e + 1;
    if (stop || nan || st.epoch >= fit_max_epochs(st.fit, bk)) {
      st.ep[st.fit == kFitWr ? 0 : (st.fit == kFitInit ? 1 : 2)] = st.epoch;
      if (nan) {
        st.status = -2;  // the reference exits (src/Bidder.py:592-600)
        fit_enter(st, kFitDone, bk, mode);
      } else {
        fit_after(st, bk, mode, init);
      }
    }
  }
  __syncthreads();
}

// step 2: this workgroup's exact partial sums (S.tot, 2 NV words) of the learner's epoch
template <int NV>
__device__ __forceinline__ void rp_block(const int64_t (&acc)[NV], TrainLds &S) {
  block_sums<NV>(acc, S.w, S.tot);
}

__global__ __launch_bounds__(kDrThreads) void k_bidder_epoch(
    const int32_t *__restrict__ bkind, const int32_t *__restrict__ bmode, const int32_t *__restrict__ initialised,
    const int32_t *__restrict__ blk_agent, const int32_t *__restrict__ blk_rank,
    const int32_t *__restrict__ agent_nblk, const int64_t *__restrict__ offsets, const int64_t *__restrict__ n_total,
    const int64_t *__restrict__ g_base, DrRecords R0, double *__restrict__ eu_ws, const FitSt *__restrict__ st_in,
    FitSt *__restrict__ st_out, const int64_t *__restrict__ tot_in, int64_t *__restrict__ tot_out,
    int64_t *__restrict__ acc_rows, unsigned *__restrict__ bars, const int32_t *__restrict__ bar_off,
    const float *__restrict__ noise, int64_t noise_n, int32_t noise_e0, int32_t noise_epochs, uint64_t noise_seed,
    const double *__restrict__ adam_tab, float *__restrict__ traces) {
  const int a = blk_agent[blockIdx.x], rank = blk_rank[blockIdx.x], nblk = agent_nblk[a];
  const int tid = threadIdx.x;
  const int bk = bkind[a], mode = bmode[a], init = initialised[a];
  __shared__ TrainLds S;
  __shared__ FitSt st;
  __shared__ float s_grad[16], s_loss;
  __shared__ int s_np;
  for (int i = tid; i < 256; i += kDrThreads) S.tab[i] = ag_exp_tab[i];
  if (tid == 0) st = st_in[a];
  __syncthreads();
  const double n = (double)n_total[a];
  if (st.fit != kFitDone && st.have_tot) {
    float *tr = (traces && g_base[a] == 0 && rank == 0 && st.fit >= kFitWr)
                    ? traces + ((size_t)a * 3 + (st.fit == kFitWr ? 0 : (st.fit == kFitInit ? 1 : 2))) * kDrEpochs
                    : nullptr;
    fit_step(st, tot_in + (size_t)a * 32, n, bk, mode, init, adam_tab, s_grad, &s_loss, &s_np, tr);
  }
  const int64_t s0 = offsets[a], nl = offsets[a + 1] - s0;
  const int64_t per = (nl + nblk - 1) / nblk;
  const int64_t c0 = (int64_t)rank * per < nl ? (int64_t)rank * per : nl;
  const int64_t nb = (c0 + per < nl ? c0 + per : nl) - c0;
  const DrRecords R{R0.ctr + s0 + c0, R0.value + s0 + c0, R0.gamma + s0 + c0, R0.prop + s0 + c0, R0.util + s0 + c0,
                    R0.won + s0 + c0};
  double *eu = eu_ws + s0 + c0;
  if (st.fit == kFitEu) {
    // estimated utilities of this workgroup's records with the fitted win-rate model
    // (src/Bidder.py:541-546; k_bidder_train<1>'s arithmetic); the same thread reads them back
    for (int64_t j = tid; j < nb; j += kDrThreads) {
      const double c = (double)(float)R.ctr[j], v = (double)(float)R.value[j], g = (double)(float)R.gamma[j];
      const double z = c * (double)st.wr[0] + v * (double)st.wr[1] + g * (double)st.wr[2] + (double)st.wr[3];
      const float W = (float)(1.0 / (1.0 + agexp::exp(-z, S.tab)));
      const double Vv = R.ctr[j] * R.value[j], P = R.ctr[j] * R.value[j] * R.gamma[j];
      eu[j] = (double)W * (Vv - P);
    }
    __syncthreads();
    if (tid == 0) fit_after(st, bk, mode, init);
    __syncthreads();
  }
  const bool noisy = st.fit == kFitPol;  // the DR / DM policy fits draw an rsample per record per epoch
  if (tid == 0)
    st.need_noise = noisy && noise && (st.epoch < noise_e0 || st.epoch >= noise_e0 + noise_epochs) ? 1 : 0;
  __syncthreads();
  const bool active = st.fit != kFitDone && !st.need_noise;
  if (active) {
    const FitNoise F{noise ? noise - (int64_t)noise_e0 * noise_n : nullptr, noise_n, noise_seed, (uint32_t)a,
                     1 << 30};
    const int64_t gb = g_base[a] + c0;  // the global index of record 0 of this chunk (the noise's)
    const int e = st.epoch;
    const int64_t nrec = nb > tid ? (nb - tid + kDrThreads - 1) / kDrThreads : 0;
    if (st.fit == kFitWins) {
      int64_t acc[1] = {0};
      for (int64_t j = tid; j < nb; j += kDrThreads) acc[0] += R.won[j] != 0 ? 1 : 0;
      rp_block<1>(acc, S);
    } else if (st.fit == kFitWr) {
      int64_t acc[5] = {0, 0, 0, 0, 0};
      const double w0 = (double)st.wr[0], w1 = (double)st.wr[1], w2 = (double)st.wr[2], w3 = (double)st.wr[3];
      for (int64_t j = tid; j < nb; j += kDrThreads) {
        const double c = (double)(float)R.ctr[j], v = (double)(float)R.value[j];
        wr_row(acc, c, v, (double)(float)R.gamma[j], (double)R.won[j], false, w0, w1, w2, w3, S.tab);
        wr_row(acc, c, v, 0.0, 0.0, true, w0, w1, w2, w3, S.tab);
      }
      wr_unbias(acc, nrec);
      rp_block<5>(acc, S);
    } else {
      int64_t acc[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[j] = 0;
      if (st.fit == kFitInit) {
        for (int64_t j = tid; j < nb; j += kDrThreads)
          imit_rec(acc, st.pol, (double)(float)R.ctr[j], (double)(float)R.value[j], (double)(float)R.gamma[j], S.tab);
#pragma unroll
        for (int q = 0; q < 14; ++q) fx_unbias(acc[q], nrec);
      } else if (bk == AG_BIDDER_DOUBLY_ROBUST) {
        for (int64_t j = tid; j < nb; j += kDrThreads)
          dr_rec(acc, st.pol, st.wr, (double)(float)R.ctr[j], (double)(float)R.value[j], (double)(float)R.gamma[j],
                 (float)R.prop[j], (double)(float)R.util[j] - (double)(float)eu[j], fit_eps(F, e, gb + j), S.tab);
#pragma unroll
        for (int q = 0; q < 13; ++q) fx_unbias(acc[q], nrec);
      } else {
        for (int64_t j = tid; j < nb; j += kDrThreads)
          dm_rec(acc, st.pol, st.wr, (double)(float)R.ctr[j], (double)(float)R.value[j], fit_eps(F, e, gb + j), S.tab);
#pragma unroll
        for (int q = 0; q < 13; ++q) fx_unbias(acc[q], nrec);
      }
      rp_block<16>(acc, S);
    }
    const int W = st.fit == kFitWins ? 2 : (st.fit == kFitWr ? 10 : 32);
    // the agent's region: accumulator rows [bar_lines(nblk)][32], barrier lines
    agcoop::agent_reduce_nowait(bars + (size_t)bar_off[a] * agcoop::kBarLineWords,
                                acc_rows + (size_t)bar_off[a] * 32, 32, rank, nblk, S.tot, W,
                                tot_out + (size_t)a * 32, &S.flag);
  }
  if (rank == 0 && tid == 0) {
    st.have_tot = active ? 1 : 0;
    st_out[a] = st;
  }
}

// ---------------------------------------------------------------------------------------
// Pipelined persistent training (ag_bidder_rp_run; ag_bidder_update's exact-sum learners):
// the FitSt state machine of k_bidder_epoch inside ONE cooperative launch per phase, every
// workgroup holding a contiguous slice of EVERY learner's records (slot i: learner
// agents[i]). A round visits the learners in turn: finish learner i's last epoch sum (its
// combining tree, agent_allreduce_finish), step its state (fit_step: loss, Adam, scheduler,
// early stop, next fit -- every workgroup the same integers, so the same step), add this
// workgroup's exact terms of its next epoch and start that sum up the tree
// (agent_allreduce_start) -- then the next learner. A learner's sum climbs the tree while the
// workgroups compute the OTHER learners' epochs, so the cross-workgroup latency that one
// learner per launch (k_bidder_train) or per epoch (k_bidder_epoch) waits out is hidden
// behind useful work. Integer sums: the same models, epochs and status bit for bit as both.
//   PH = 0: the win count and the win-rate fit (4 workgroups per CU, <= 128 VGPRs);
//   PH = 1: estimated utilities, imitation, the policy fits (3 per CU).
// A policy fit whose host-drawn noise window ends waits with its state kept (need_noise);
// the launch ends when no learner has an epoch left in its phase.
constexpr int kPipeMaxAgents = 16;
constexpr int kPipeFanIn = 32;  // the trees' fan-in: 2 levels up to 1024 workgroups
struct PipeArgs {
  int NA;                       // learners in the launch (<= kPipeMaxAgents)
  const int32_t *agents;        // [NA] their agent indices
  const int32_t *bkind, *bmode, *initialised;
  const int64_t *offsets;       // [N + 1] sorted records
  const int64_t *n_total;       // [N] the learners' record counts (fit_step's n)
  DrRecords R0;
  double *eu_ws;
  FitSt *st;                    // [N] in / out
  const int64_t *tot_in;        // [N][32] totals pending from ag_bidder_rp_epoch (have_tot)
  int64_t *acc;                 // [NA][lines][32] combining-tree rows
  unsigned *bars;               // [NA][lines][kBarLineWords]
  int lines;
  const int32_t *lds_off;       // [NA] record-cache byte offsets (dynamic LDS, after the FitSt copies)
  const int32_t *lds_cap;       // [NA] records cached per workgroup
  const float *noise;           // host-drawn draws or NULL (synthetic)
  const int64_t *noise_off;     // [N] per-learner offsets (NULL: 0)
  int64_t noise_stride;         // floats per epoch (0: the learner's record count)
  int32_t noise_e0, noise_epochs;
  uint64_t noise_seed;
  const double *adam_tab;
  float *traces;                // [N][3][kDrEpochs] or NULL
  long long *prof;              // diagnostics (AG_PIPE_PROF): [G][8] wall-clock ticks per part, or NULL
};

// this workgroup's slice [c0, c0 + nb) of n records over G workgroups
__device__ __forceinline__ void pipe_chunk(int64_t n, int G, int rank, int64_t &c0, int64_t &nb) {
  const int64_t per = (n + G - 1) / G;
  c0 = (int64_t)rank * per < n ? (int64_t)rank * per : n;
  nb = (c0 + per < n ? c0 + per : n) - c0;
}

template <int PH>
__device__ __forceinline__ bool pipe_in_phase(int fit) {
  return PH == 0 ? (fit == kFitWins || fit == kFitWr) : (fit == kFitEu || fit == kFitInit || fit == kFitPol);
}

// this workgroup's exact partial sums of the learner's current epoch -> S.tot; returns the
// words to sum (k_bidder_epoch's step 2)
template <int PH>
__device__ __forceinline__ int pipe_partial(const FitSt &st, const RecView &V, int64_t nb, int bk, const FitNoise &F,
                                            TrainLds &S) {
  const int tid = threadIdx.x;
  const int64_t nrec = nb > tid ? (nb - tid + kDrThreads - 1) / kDrThreads : 0;
  if constexpr (PH == 0) {
    if (st.fit == kFitWins) {
      int64_t acc[1] = {0};
      each_record(V, nb, [&](int64_t j, auto L) { acc[0] += V.template won_<decltype(L)::value>(j) != 0.0 ? 1 : 0; });
      block_sums<1>(acc, S.w, S.tot);
      return 2;
    }
    int64_t acc[5] = {0, 0, 0, 0, 0};
    const double w0 = (double)st.wr[0], w1 = (double)st.wr[1], w2 = (double)st.wr[2], w3 = (double)st.wr[3];
    each_record(V, nb, [&](int64_t j, auto L) {
      constexpr bool l = decltype(L)::value;
      const double c = V.template ctr_<l>(j), v = V.template val_<l>(j);
      wr_pair(acc, c, v, V.template gam_<l>(j), V.template won_<l>(j), w0, w1, w2, w3, S.tab);
    });
    wr_unbias(acc, nrec);
    block_sums<5>(acc, S.w, S.tot);
    return 10;
  } else {
    int64_t acc[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = 0;
    const int e = st.epoch;
    if (st.fit == kFitInit) {
      each_record(V, nb, [&](int64_t j, auto L) {
        constexpr bool l = decltype(L)::value;
        imit_rec(acc, st.pol, V.template ctr_<l>(j), V.template val_<l>(j), V.template gam_<l>(j), S.tab);
      });
#pragma unroll
      for (int q = 0; q < 14; ++q) fx_unbias(acc[q], nrec);
    } else if (bk == AG_BIDDER_DOUBLY_ROBUST) {
      each_record(V, nb, [&](int64_t j, auto L) {
        constexpr bool l = decltype(L)::value;
        dr_rec(acc, st.pol, st.wr, V.template ctr_<l>(j), V.template val_<l>(j), V.template gam_<l>(j),
               V.template prop_<l>(j), V.template util_<l>(j) - V.template eut_<l>(j), fit_eps(F, e, V.c0 + j), S.tab);
      });
#pragma unroll
      for (int q = 0; q < 13; ++q) fx_unbias(acc[q], nrec);
    } else {
      each_record(V, nb, [&](int64_t j, auto L) {
        constexpr bool l = decltype(L)::value;
        dm_rec(acc, st.pol, st.wr, V.template ctr_<l>(j), V.template val_<l>(j), fit_eps(F, e, V.c0 + j), S.tab);
      });
#pragma unroll
      for (int q = 0; q < 13; ++q) fx_unbias(acc[q], nrec);
    }
    block_sums<16>(acc, S.w, S.tot);
    return 32;
  }
}

// a slot's constants, read once into LDS (the rounds read nothing from global memory but the
// records beyond the cache and the Adam table)
struct PipeSlot {
  int64_t s0, c0, nb, cap;  // the learner's first sorted record; this workgroup's slice; cached records
  double n;                 // records (fit_step's n)
  uint32_t off;             // record cache: byte offset in the dynamic LDS (not a pointer: kept
                            // an LDS address, ds_read, not a flat load through a generic pointer)
  int a, bk, mode, init, nf;
};

template <int PH>
__global__ __launch_bounds__(kDrThreads, PH == 0 ? 4 : AG_DR_PH1_MIN_WAVES) void k_bidder_pipe(PipeArgs A) {
  __shared__ TrainLds S;
  __shared__ float s_grad[16], s_loss;
  __shared__ int s_np;
  __shared__ unsigned s_gen[kPipeMaxAgents];
  __shared__ PipeSlot s_slot[kPipeMaxAgents];
  __shared__ double s_bc[kPipeMaxAgents][2];  // the Adam bias corrections of each slot's epoch in flight
  extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];
  FitSt *fst = reinterpret_cast<FitSt *>(s_dyn);
  const int tid = threadIdx.x, G = gridDim.x, rank = blockIdx.x, NA = A.NA;
  for (int i = tid; i < 256; i += kDrThreads) S.tab[i] = ag_exp_tab[i];
  for (int i = tid; i < NA; i += kDrThreads) {
    const int a = A.agents[i], bk = A.bkind[a];
    fst[i] = A.st[a];
    PipeSlot &P = s_slot[i];
    P.a = a;
    P.bk = bk;
    P.mode = A.bmode[a];
    P.init = A.initialised[a];
    P.n = (double)A.n_total[a];
    P.s0 = A.offsets[a];
    pipe_chunk(A.offsets[a + 1] - P.s0, G, rank, P.c0, P.nb);
    P.cap = A.lds_cap[i];
    P.off = (uint32_t)A.lds_off[i];
    P.nf = PH == 0 ? 3 : (bk == AG_BIDDER_DOUBLY_ROBUST ? 6 : 2);
  }
  __syncthreads();
  // stage every slot's cached records (this phase's fields)
  for (int i = 0; i < NA; ++i) {
    const PipeSlot &P = s_slot[i];
    const int64_t cap = P.cap, ns = P.nb < cap ? P.nb : cap;
    float *lf = reinterpret_cast<float *>(s_dyn + P.off);
    const bool dr = P.bk == AG_BIDDER_DOUBLY_ROBUST;
    uint8_t *lw = reinterpret_cast<uint8_t *>(lf + (size_t)P.nf * cap);
    const bool eu_ready = dr && fst[i].fit > kFitEu && fst[i].fit != kFitDone;
    for (int64_t j = tid; j < ns; j += kDrThreads) {
      const int64_t r = P.s0 + P.c0 + j;
      lf[kFCtr * cap + j] = (float)A.R0.ctr[r];
      lf[kFVal * cap + j] = (float)A.R0.value[r];
      if (PH == 0 || dr) lf[kFGam * cap + j] = (float)A.R0.gamma[r];
      if (PH == 0) lw[j] = A.R0.won[r];
      if (PH == 1 && dr) {
        lf[kFProp * cap + j] = (float)A.R0.prop[r];
        lf[kFUtil * cap + j] = (float)A.R0.util[r];
        if (eu_ready) lf[kFEu * cap + j] = (float)A.eu_ws[r];
      }
    }
  }
  __syncthreads();
  // AG_PIPE_PROF: finish, step, partial, start, total, finishes (thread 0's; LDS, not registers)
  __shared__ long long pr[8];
  if (tid < 8) pr[tid] = 0;
  auto view = [&](const PipeSlot &P) -> RecView {
    const int64_t s0 = P.s0;
    const DrRecords R{A.R0.ctr + s0, A.R0.value + s0, A.R0.gamma + s0, A.R0.prop + s0, A.R0.util + s0, A.R0.won + s0};
    const float *lf = reinterpret_cast<const float *>(s_dyn + P.off);
    return RecView{R, A.eu_ws + s0, P.c0, lf, reinterpret_cast<const uint8_t *>(lf + (size_t)P.nf * P.cap), P.cap};
  };
  auto tr_of = [&](int a, const FitSt &st) -> float * {
    if (!A.traces || rank != 0 || st.fit < kFitWr) return nullptr;
    return A.traces + ((size_t)a * 3 + (st.fit == kFitWr ? 0 : (st.fit == kFitInit ? 1 : 2))) * kDrEpochs;
  };
  auto step = [&](int i, const int64_t *tot, bool prefetched) {
    const PipeSlot &P = s_slot[i];
    fit_step(fst[i], tot, P.n, P.bk, P.mode, P.init, A.adam_tab, s_grad, &s_loss, &s_np, tr_of(P.a, fst[i]),
             prefetched ? s_bc[i] : nullptr);
  };
  // the next epoch of slot i: estimated utilities when its fit reaches them, then its partial
  // sums started up its tree; false when it has no epoch left in this phase (or waits for noise)
  auto begin = [&](int i, bool &root) -> bool {
    FitSt &st = fst[i];
    const PipeSlot &P = s_slot[i];
    const int a = P.a, bk = P.bk;
    const int64_t nb = P.nb;
    const RecView V = view(P);
    if (PH == 1 && st.fit == kFitEu) {
      // src/Bidder.py:541-546 with the fitted win-rate model (k_bidder_epoch's arithmetic);
      // each_record's thread mapping, so a thread reads back what it wrote
      double *eu = A.eu_ws + P.s0;
      float *lfe = reinterpret_cast<float *>(s_dyn + P.off) + (size_t)kFEu * V.cap;
      for (int64_t j = tid; j < nb; j += kDrThreads) {
        const int64_t r = V.c0 + j;
        const double c = (double)(float)V.R.ctr[r], v = (double)(float)V.R.value[r], g = (double)(float)V.R.gamma[r];
        const double z = c * (double)st.wr[0] + v * (double)st.wr[1] + g * (double)st.wr[2] + (double)st.wr[3];
        const float W = (float)(1.0 / (1.0 + agexp::exp(-z, S.tab)));
        const double Vv = V.R.ctr[r] * V.R.value[r], Pp = V.R.ctr[r] * V.R.value[r] * V.R.gamma[r];
        eu[r] = (double)W * (Vv - Pp);
        if (j < V.cap) lfe[j] = (float)eu[r];
      }
      __syncthreads();
      if (tid == 0) fit_after(st, bk, P.mode, P.init);
      __syncthreads();
    }
    if (!pipe_in_phase<PH>(st.fit) || st.fit == kFitEu) return false;
    const bool wait = PH == 1 && st.fit == kFitPol && A.noise &&
                      (st.epoch < A.noise_e0 || st.epoch >= A.noise_e0 + A.noise_epochs);
    __syncthreads();
    if (tid == 0) st.need_noise = wait ? 1 : 0;
    __syncthreads();
    if (wait) return false;
    // this epoch's Adam bias corrections, loaded now and stored after the partial sums (the
    // load's latency hidden behind them); fit_step reads them from LDS
    const int e = st.epoch;
    double b1 = 0.0, b2 = 0.0;
    if (tid == 0 && st.fit != kFitWins) {
      b1 = A.adam_tab[e];
      b2 = A.adam_tab[kDrEpochs + e];
    }
    const int64_t stride = A.noise_stride ? A.noise_stride : (int64_t)P.n;
    const FitNoise F{A.noise ? A.noise + (A.noise_off ? A.noise_off[a] : 0) - (int64_t)A.noise_e0 * stride : nullptr,
                     stride, A.noise_seed, (uint32_t)a, 1 << 30};
    long long tp = A.prof && tid == 0 ? wall_clock64() : 0;
    const int W = pipe_partial<PH>(st, V, nb, bk, F, S);
    if (tid == 0) {
      s_bc[i][0] = b1;
      s_bc[i][1] = b2;
    }
    if (A.prof) {
      __syncthreads();
      if (tid == 0) {
        const long long tq = wall_clock64();
        pr[2] += tq - tp;
        tp = tq;
      }
    }
    root = agcoop::agent_allreduce_start<kPipeFanIn>(A.bars + (size_t)i * A.lines * kBarLineWords, A.acc + (size_t)i * A.lines * 32,
                                         32, rank, G, S.tot, W, &s_gen[i], &S.flag);
    if (A.prof && tid == 0) pr[3] += wall_clock64() - tp;
    return true;
  };
  // totals left by ag_bidder_rp_epoch launches
  for (int i = 0; i < NA; ++i)
    if (fst[i].have_tot && fst[i].fit != kFitDone) step(i, A.tot_in + (size_t)s_slot[i].a * 32, false);
  uint32_t pend = 0, roots = 0;
  const long long t_start = A.prof ? wall_clock64() : 0;
  for (int i = 0; i < NA; ++i) {
    bool root = false;
    if (begin(i, root)) pend |= 1u << i;
    if (root) roots |= 1u << i;
  }
  while (pend) {
    for (int i = 0; i < NA; ++i) {
      if (!(pend >> i & 1)) continue;
      const int W = fst[i].fit == kFitWins ? 2 : (fst[i].fit == kFitWr ? 10 : 32);
      long long tf = A.prof && tid == 0 ? wall_clock64() : 0;
      agcoop::agent_allreduce_finish(A.bars + (size_t)i * A.lines * kBarLineWords, A.acc + (size_t)i * A.lines * 32, G,
                                     roots >> i & 1, &s_gen[i], W, S.tot);
      if (A.prof && tid == 0) {
        const long long tg = wall_clock64();
        pr[0] += tg - tf;
        tf = tg;
        pr[5] += 1;
      }
      step(i, S.tot, true);
      if (A.prof) {
        __syncthreads();
        if (tid == 0) pr[1] += wall_clock64() - tf;
      }
      bool root = false;
      pend &= ~(1u << i);
      roots &= ~(1u << i);
      if (begin(i, root)) pend |= 1u << i;
      if (root) roots |= 1u << i;
    }
  }
  __syncthreads();
  if (A.prof && tid == 0) {
    pr[4] = wall_clock64() - t_start;
    for (int k = 0; k < 8; ++k) A.prof[(size_t)rank * 8 + k] = pr[k];
  }
  if (rank == 0)
    for (int i = tid; i < NA; i += kDrThreads) {
      FitSt f = fst[i];
      f.have_tot = 0;
      A.st[s_slot[i].a] = f;
    }
}

// the learners' FitSt at the start of a resumable update (state16: win-rate model, policy)
__global__ void k_rp_init(int N, const int32_t *__restrict__ bkind, const int32_t *__restrict__ bmode,
                          const int32_t *__restrict__ mask, const float *__restrict__ state, FitSt *__restrict__ st,
                          int parities) {
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= N) return;
  FitSt f;
  memset(&f, 0, sizeof f);
  for (int j = 0; j < 4; ++j) f.wr[j] = state[(size_t)a * 16 + j];
  for (int j = 0; j < 12; ++j) f.pol[j] = state[(size_t)a * 16 + 4 + j];
  const int bk = bkind[a];
  if (mask[a])
    fit_enter(f, bk == AG_BIDDER_DOUBLY_ROBUST ? kFitWr : kFitWins, bk, bmode[a]);
  else
    fit_enter(f, kFitDone, bk, bmode[a]);
  st[a] = f;
  if (parities == 2) st[N + a] = f;  // [2][N] states: parity 1 too -- the epoch launches never
                                     // write unmasked agents' rows
}

__global__ __launch_bounds__(kDrThreads) void k_sh_hist(const int32_t *__restrict__ agent, int64_t n, int N,
                                                        int64_t *__restrict__ counts) {
  extern __shared__ unsigned int s_hist[];
  for (int a = threadIdx.x; a < N; a += kDrThreads) s_hist[a] = 0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * kDrThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kDrThreads)
    atomicAdd(&s_hist[agent[i]], 1u);
  __syncthreads();
  for (int a = threadIdx.x; a < N; a += kDrThreads)
    if (s_hist[a]) atomicAdd((unsigned long long *)&counts[a], (unsigned long long)s_hist[a]);
}

// records in (agent, log order): sort keys agent << 40 | order, gather every field
__global__ __launch_bounds__(kDrThreads) void k_sh_keys(ag_shading_samples s, int64_t n, uint64_t *__restrict__ key,
                                                        uint32_t *__restrict__ idx) {
  for (int64_t i = (int64_t)blockIdx.x * kDrThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kDrThreads) {
    key[i] = ((uint64_t)(uint32_t)s.agent[i] << 40) | (s.order[i] & ((1ull << 40) - 1));
    idx[i] = (uint32_t)i;
  }
}

__global__ __launch_bounds__(kDrThreads) void k_sh_gather(ag_shading_samples s, int64_t n,
                                                          const uint32_t *__restrict__ idx,
                                                          double *__restrict__ o_ctr, double *__restrict__ o_val,
                                                          double *__restrict__ o_gam, double *__restrict__ o_prop,
                                                          double *__restrict__ o_util, uint8_t *__restrict__ o_won) {
  for (int64_t j = (int64_t)blockIdx.x * kDrThreads + threadIdx.x; j < n; j += (int64_t)gridDim.x * kDrThreads) {
    const uint32_t i = idx[j];
    o_ctr[j] = s.ctr[i];
    o_val[j] = s.value[i];
    o_gam[j] = s.gamma[i];
    o_prop[j] = s.propensity[i];
    o_util[j] = s.utility[i];
    o_won[j] = s.won[i];
  }
}

int grid_over(int64_t n) {
  int64_t g = (n + kDrThreads - 1) / kDrThreads;
  if (g > 4096) g = 4096;
  return (int)(g < 1 ? 1 : g);
}

}  // namespace

void ag_dr_release(ag_ctx *c) {
  ag_dr_ws &w = c->dr;
  (void)hipFree(w.buf);
  (void)hipFree(w.counts);
  (void)hipFree(w.adam_tab);
  (void)hipFree(w.state);
  (void)hipFree(w.init);
  (void)hipFree(w.mode);
  (void)hipFree(w.scratch);
  (void)hipFree(w.coop);
  (void)hipFree(w.rp.st);
  (void)hipFree(w.rp.acc);
  (void)hipFree(w.rp.tables);
  (void)hipFree(w.rp.pipe);
  (void)hipFree(w.rp.pipe_st);
  w = ag_dr_ws();
}

// The sorted record arrays of the workspace (sort_records' layout) for n records
static DrRecords sorted_view(ag_dr_ws &w, int64_t n, double **eu) {
  const int64_t cap = n > 0 ? n : 1;
  double *b = (double *)w.buf;
  *eu = b + 5 * cap;
  return DrRecords{b, b + cap, b + 2 * cap, b + 3 * cap, b + 4 * cap,
                   (const uint8_t *)((uint32_t *)((uint64_t *)(b + 6 * cap) + 2 * cap) + 2 * cap)};
}

// k_bidder_pipe's record-cache budgets (dynamic LDS per workgroup: 4 / 3 per CU) and the
// records per workgroup it aims at (AG_PIPE_RECS overrides, for tuning): fewer workgroups for
// small learners -- a shorter tree to climb each epoch -- and the whole resident grid for
// large ones
constexpr size_t kPipeLds[2] = {32 * 1024, 44 * 1024};
constexpr int64_t kPipeRecs = 512;

struct PipeNoise {
  const float *noise = nullptr;
  const int64_t *noise_off = nullptr;
  int64_t stride = 0;
  int32_t e0 = 0, epochs = 0;
};

// Runs the learners `slots` (agent indices; FitSt in d_st) through k_bidder_pipe's phases
// `phases` (bit p: phase p), one cooperative launch each.
static int pipe_run(ag_ctx *c, const std::vector<int32_t> &slots, const std::vector<int64_t> &cnt, const DrRecords &R,
                    double *eu, const int64_t *d_off, const int64_t *d_ntot, FitSt *d_st, const int64_t *tot_in,
                    const PipeNoise &nz, float *traces, int phases, hipStream_t st) {
  ag_dr_ws &w = c->dr;
  ag_dr_rp &rp = w.rp;
  const int NA = (int)slots.size();
  if (NA == 0) return AG_OK;
  if (NA > kPipeMaxAgents) return ag_set_error(AG_ERR_UNSUPPORTED, "k_bidder_pipe: > %d learners", kPipeMaxAgents);
  int64_t recs = 0;
  for (int a : slots) recs += cnt[a];
  int64_t want_recs = kPipeRecs;
  if (const char *e = getenv("AG_PIPE_RECS")) want_recs = std::max<int64_t>(1, atoll(e));
  for (int ph = 0; ph < 2; ++ph)
    if (!rp.pipe_blocks[ph]) {
      const void *fn = ph == 0 ? (const void *)k_bidder_pipe<0> : (const void *)k_bidder_pipe<1>;
      int per_cu = 0, cus = 0;
      AG_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kPipeLds[ph]));
      AG_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kDrThreads, kPipeLds[ph]));
      AG_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device));
      rp.pipe_blocks[ph] = std::max(1, per_cu * cus);
    }
  // device tables, sized once for the largest grid: [3][kPipeMaxAgents] i32 per phase, then
  // per phase the acc rows [kPipeMaxAgents][lines][32] i64 and barrier lines (the two
  // launches of a run never share a word)
  const size_t lines_max = (size_t)std::max(1, bar_lines(std::max(rp.pipe_blocks[0], rp.pipe_blocks[1]), kPipeFanIn));
  const size_t rows_max = (size_t)kPipeMaxAgents * lines_max * 32;
  const size_t per_ph = 3 * kPipeMaxAgents * sizeof(int32_t) + rows_max * (sizeof(int64_t) + sizeof(unsigned)) + 64;
  if (2 * per_ph > rp.pipe_bytes) {
    (void)hipFree(rp.pipe);  // (synchronises: no launch of an earlier run uses it any more)
    rp.pipe = nullptr;
    rp.pipe_bytes = 0;
    AG_HIP(hipMalloc(&rp.pipe, 2 * per_ph));
    rp.pipe_bytes = 2 * per_ph;
  }
  for (int ph = 0; ph < 2; ++ph) {
    if (!(phases >> ph & 1)) continue;
    const void *fn = ph == 0 ? (const void *)k_bidder_pipe<0> : (const void *)k_bidder_pipe<1>;
    const int G = (int)std::max<int64_t>(1, std::min<int64_t>(rp.pipe_blocks[ph], (recs + want_recs - 1) / want_recs));
    const int lines = std::max(1, bar_lines(G, kPipeFanIn));
    // record caches after the FitSt copies: slot i caches min(chunk, share) records
    const size_t fst_bytes = ((size_t)NA * sizeof(FitSt) + 15) / 16 * 16;
    const size_t budget = kPipeLds[ph] - fst_bytes;
    std::vector<int64_t> chunk(NA), bytes(NA);
    double total = 0.0;
    for (int i = 0; i < NA; ++i) {
      const int bk = c->h_bkind[slots[i]];
      chunk[i] = (cnt[slots[i]] + G - 1) / G;
      bytes[i] = ph == 0 ? 13 : (bk == AG_BIDDER_DOUBLY_ROBUST ? 24 : 8);
      total += (double)(chunk[i] * bytes[i] + 16);
    }
    const double f = total > (double)budget ? (double)budget / total : 1.0;
    std::vector<int32_t> tab(3 * kPipeMaxAgents, 0);
    size_t off = fst_bytes;
    for (int i = 0; i < NA; ++i) {
      const int64_t cap = std::min<int64_t>(chunk[i], (int64_t)((double)chunk[i] * f));
      tab[i] = slots[i];
      tab[kPipeMaxAgents + i] = (int32_t)off;
      tab[2 * kPipeMaxAgents + i] = (int32_t)cap;
      off += ((size_t)cap * bytes[i] + 15) / 16 * 16;
    }
    if (off > kPipeLds[ph])
      return ag_set_error(AG_ERR_UNSUPPORTED, "k_bidder_pipe: record cache plan %zu > %zu", off, kPipeLds[ph]);
    int32_t *d_tab = (int32_t *)((char *)rp.pipe + ph * per_ph);
    int64_t *d_acc = (int64_t *)(((uintptr_t)(d_tab + 3 * kPipeMaxAgents) + 15) & ~(uintptr_t)15);
    const size_t rows = (size_t)NA * lines * 32;
    unsigned *d_bar = (unsigned *)(d_acc + rows);
    AG_HIP(hipMemcpyAsync(d_tab, tab.data(), sizeof(int32_t) * tab.size(), hipMemcpyHostToDevice, st));
    AG_HIP(hipMemsetAsync(d_acc, 0, rows * (sizeof(int64_t) + sizeof(unsigned)), st));
    PipeArgs A;
    A.NA = NA;
    A.agents = d_tab;
    A.bkind = c->d_bkind;
    A.bmode = w.mode;
    A.initialised = w.init;
    A.offsets = d_off;
    A.n_total = d_ntot;
    A.R0 = R;
    A.eu_ws = eu;
    A.st = d_st;
    A.tot_in = tot_in;
    A.acc = d_acc;
    A.bars = d_bar;
    A.lines = lines;
    A.lds_off = d_tab + kPipeMaxAgents;
    A.lds_cap = d_tab + 2 * kPipeMaxAgents;
    A.noise = nz.noise;
    A.noise_off = nz.noise_off;
    A.noise_stride = nz.stride;
    A.noise_e0 = nz.e0;
    A.noise_epochs = nz.epochs;
    A.noise_seed = c->fit_noise_seed;
    A.adam_tab = w.adam_tab;
    A.traces = traces;
    A.prof = nullptr;
    const bool prof = getenv("AG_PIPE_PROF") != nullptr;
    if (prof) AG_HIP(hipMalloc(&A.prof, sizeof(long long) * 8 * G));
    void *args[] = {&A};
    AG_HIP(hipLaunchCooperativeKernel(fn, dim3(G), dim3(kDrThreads), args, kPipeLds[ph], st));
    if (prof) {  // diagnostics: mean over workgroups of each part, microseconds (100 MHz clock)
      std::vector<long long> h(8 * (size_t)G);
      AG_HIP(hipMemcpy(h.data(), A.prof, sizeof(long long) * 8 * G, hipMemcpyDeviceToHost));
      (void)hipFree(A.prof);
      double m[8] = {0};
      for (int b = 0; b < G; ++b)
        for (int k = 0; k < 8; ++k) m[k] += (double)h[8 * (size_t)b + k] / G;
      fprintf(stderr, "k_bidder_pipe<%d> G=%d NA=%d: finish-wait %.0f us, step %.0f us, partial %.0f us, start %.0f "
              "us, total %.0f us, finishes %.0f\n", ph, G, NA, m[0] / 100, m[1] / 100, m[2] / 100, m[3] / 100,
              m[4] / 100, m[5]);
    }
  }
  return AG_OK;
}

// FitSt [N] then a mask [N] for ag_bidder_update's pipe run (its own buffer: pipe_run may
// reallocate the tables)
static FitSt *pipe_fitst(ag_ctx *c) {
  ag_dr_rp &rp = c->dr.rp;
  const size_t N = (size_t)c->shape.num_agents;
  if (!rp.pipe_st && hipMalloc(&rp.pipe_st, (sizeof(FitSt) + sizeof(int32_t)) * N) != hipSuccess) return nullptr;
  return (FitSt *)rp.pipe_st;
}

// which agents bid from a fitted policy / a win-rate search (ag_simulate checks its inputs)
static void learner_flags(ag_ctx *c, const int32_t *init) {
  c->dr_any_init = c->vl_any_search = false;
  for (int a = 0; a < c->shape.num_agents; ++a) {
    const int bk = c->h_bkind ? c->h_bkind[a] : -1;
    const bool learner = bk == AG_BIDDER_VALUE_LEARNING || bk == AG_BIDDER_POLICY_LEARNING || bk == AG_BIDDER_DOUBLY_ROBUST;
    if (learner && init[a] == AG_LEARNER_POLICY) c->dr_any_init = true;
    if (bk == AG_BIDDER_VALUE_LEARNING && init[a] == AG_LEARNER_SEARCH) c->vl_any_search = true;
  }
}

// workspace: counts / offsets / cursors, the Adam bias-correction table, the learner state
static int dr_ws_ready(ag_ctx *c) {
  ag_dr_ws &w = c->dr;
  if (w.adam_tab) return AG_OK;
  const int N = c->shape.num_agents;
  double *tab = new double[2 * kDrEpochs];
  for (int t = 0; t < kDrEpochs; ++t) {  // torch.optim.Adam: Python floats, libm pow
    tab[t] = 1.0 - pow(0.9, (double)(t + 1));
    tab[kDrEpochs + t] = pow(1.0 - pow(0.999, (double)(t + 1)), 0.5);
  }
  hipError_t e = hipMalloc(&w.adam_tab, sizeof(double) * 2 * kDrEpochs);
  if (e == hipSuccess) e = hipMemcpy(w.adam_tab, tab, sizeof(double) * 2 * kDrEpochs, hipMemcpyHostToDevice);
  delete[] tab;
  if (e == hipSuccess) e = hipMalloc(&w.counts, sizeof(int64_t) * (3 * (size_t)N + 1));
  if (e == hipSuccess) e = hipMalloc(&w.state, sizeof(float) * 16 * (size_t)N);
  if (e == hipSuccess) e = hipMemset(w.state, 0, sizeof(float) * 16 * (size_t)N);
  if (e == hipSuccess) e = hipMalloc(&w.init, sizeof(int32_t) * (size_t)N);
  if (e == hipSuccess) e = hipMemset(w.init, 0, sizeof(int32_t) * (size_t)N);
  if (e == hipSuccess) e = hipMalloc(&w.mode, sizeof(int32_t) * (size_t)N);
  if (e == hipSuccess) {  // defaults: ValueLearningBidder 'search', PolicyLearningBidder 'PPO'
    std::vector<int32_t> m(N, AG_VL_SEARCH);
    for (int a = 0; a < N; ++a)
      if (c->h_bkind && c->h_bkind[a] == AG_BIDDER_POLICY_LEARNING) m[a] = AG_PL_LOSS_PPO;
    e = hipMemcpy(w.mode, m.data(), sizeof(int32_t) * N, hipMemcpyHostToDevice);
  }
  if (e == hipSuccess) e = hipMalloc(&w.scratch, sizeof(int64_t) * (size_t)N + sizeof(int32_t) * 5 * (size_t)N);
  if (e != hipSuccess) {
    ag_dr_release(c);
    return ag_set_error(AG_ERR_HIP, "DR workspace: %s", hipGetErrorString(e));
  }
  return AG_OK;
}

// The learning bidders' records of a store sorted into (agent, log order) in the workspace
// (radix sort on agent << 40 | order, then every field gathered): cnt / off host [N] / [N + 1];
// SortedRecs: device arrays [n] (eu: the estimated-utility workspace) and d_off [N + 1].
struct SortedRecs {
  double *ctr, *val, *gam, *prop, *util, *eu;
  uint8_t *won;
  int64_t *d_off;
  int64_t n;
};
static int sort_records(ag_ctx *c, const ag_shading_samples *s, std::vector<int64_t> &cnt, std::vector<int64_t> &off,
                        SortedRecs &out, hipStream_t st) {
  const int N = c->shape.num_agents;
  if (int rc = ag_shading_counts(c, s, cnt.data(), st)) return rc;
  int64_t n = 0;
  for (int a = 0; a < N; ++a) n += cnt[a];
  ag_dr_ws &w = c->dr;
  off.assign((size_t)N + 1, 0);
  for (int a = 0; a < N; ++a) off[a + 1] = off[a] + cnt[a];
  int64_t *d_off = w.counts + N;  // [N + 1] offsets
  AG_HIP(hipMemcpyAsync(d_off, off.data(), sizeof(int64_t) * ((size_t)N + 1), hipMemcpyHostToDevice, st));
  if (n >= ((int64_t)1 << 32)) return ag_set_error(AG_ERR_UNSUPPORTED, "learning bidders' update: >= 2^32 records");
  // radix-sort workspace: keys in/out (8 B), indices in/out (4 B), then hipcub's temp
  size_t sort_tmp = 0;
  AG_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_tmp, (uint64_t *)nullptr, (uint64_t *)nullptr,
                                            (uint32_t *)nullptr, (uint32_t *)nullptr, (int)(n > 0 ? n : 1), 0, 64,
                                            st));
  const size_t rec_bytes = (size_t)6 * sizeof(double) + 1;
  const size_t need = (size_t)(n > 0 ? n : 1) * (rec_bytes + 24) + sort_tmp + 256;
  if (need > w.buf_bytes) {
    (void)hipFree(w.buf);
    w.buf = nullptr;
    const size_t bytes = need + (need >> 2);
    AG_HIP(hipMalloc(&w.buf, bytes));
    w.buf_bytes = bytes;
  }
  const size_t cap = (size_t)(n > 0 ? n : 1);
  double *b_ctr = (double *)w.buf, *b_val = b_ctr + cap, *b_gam = b_val + cap, *b_prop = b_gam + cap,
         *b_util = b_prop + cap, *b_eu = b_util + cap;
  uint64_t *k_in = (uint64_t *)(b_eu + cap), *k_out = k_in + cap;
  uint32_t *i_in = (uint32_t *)(k_out + cap), *i_out = i_in + cap;
  uint8_t *b_won = (uint8_t *)(i_out + cap);
  void *tmp = (void *)(((uintptr_t)(b_won + cap) + 255) & ~(uintptr_t)255);
  if (n > 0) {
    if (!s->order) return ag_set_error(AG_ERR_INVALID, "learning bidders' update: the store needs order");
    hipLaunchKernelGGL(k_sh_keys, dim3(grid_over(n)), dim3(kDrThreads), 0, st, *s, n, k_in, i_in);
    AG_HIP(hipGetLastError());
    int end_bit = 40;
    while ((1ll << (end_bit - 40)) < N) ++end_bit;
    AG_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, sort_tmp, k_in, k_out, i_in, i_out, (int)n, 0, end_bit, st));
    hipLaunchKernelGGL(k_sh_gather, dim3(grid_over(n)), dim3(kDrThreads), 0, st, *s, n, i_out, b_ctr, b_val, b_gam,
                       b_prop, b_util, b_won);
    AG_HIP(hipGetLastError());
  }
  out = SortedRecs{b_ctr, b_val, b_gam, b_prop, b_util, b_eu, b_won, d_off, n};
  return AG_OK;
}

extern "C" {

int ag_set_dr_state(ag_ctx *c, const float *state, const int32_t *initialised) {
  if (!c || !state || !initialised) return ag_set_error(AG_ERR_INVALID, "ag_set_dr_state: null argument");
  AgDeviceGuard g(c->device);
  if (int rc = dr_ws_ready(c)) return rc;
  const int N = c->shape.num_agents;
  AG_HIP(hipMemcpy(c->dr.state, state, sizeof(float) * 16 * N, hipMemcpyHostToDevice));
  AG_HIP(hipMemcpy(c->dr.init, initialised, sizeof(int32_t) * N, hipMemcpyHostToDevice));
  c->dr_loaded = true;
  learner_flags(c, initialised);
  return AG_OK;
}

int ag_get_dr_state(ag_ctx *c, float *state, int32_t *initialised) {
  if (!c) return ag_set_error(AG_ERR_INVALID, "ag_get_dr_state: null ctx");
  AgDeviceGuard g(c->device);
  if (int rc = dr_ws_ready(c)) return rc;
  const int N = c->shape.num_agents;
  AG_HIP(hipDeviceSynchronize());
  if (state) AG_HIP(hipMemcpy(state, c->dr.state, sizeof(float) * 16 * N, hipMemcpyDeviceToHost));
  if (initialised) AG_HIP(hipMemcpy(initialised, c->dr.init, sizeof(int32_t) * N, hipMemcpyDeviceToHost));
  return AG_OK;
}

int ag_shading_counts(ag_ctx *c, const ag_shading_samples *s, int64_t *counts, void *stream) {
  if (!c || !s || !counts) return ag_set_error(AG_ERR_INVALID, "ag_shading_counts: null argument");
  AG_CHECK_STRUCT(s, "ag_shading_counts", "ag_shading_samples");
  AgDeviceGuard g(c->device);
  if (int rc = dr_ws_ready(c)) return rc;
  const int N = c->shape.num_agents;
  hipStream_t st = (hipStream_t)stream;
  uint64_t n = 0;
  AG_HIP(hipMemcpyAsync(&n, s->count, sizeof n, hipMemcpyDeviceToHost, st));
  AG_HIP(hipStreamSynchronize(st));
  if ((int64_t)n > s->capacity)
    return ag_set_error(AG_ERR_INVALID, "ag_shading_counts: %llu records overflowed the store (capacity %lld)",
                        (unsigned long long)n, (long long)s->capacity);
  int64_t *d_counts = c->dr.counts;
  AG_HIP(hipMemsetAsync(d_counts, 0, sizeof(int64_t) * N, st));
  if (n > 0) {
    if ((size_t)N * 4 > 64 * 1024) return ag_set_error(AG_ERR_UNSUPPORTED, "ag_shading_counts: N > 16384");
    hipLaunchKernelGGL(k_sh_hist, dim3(grid_over((int64_t)n)), dim3(kDrThreads), (size_t)N * 4, st, s->agent,
                       (int64_t)n, N, d_counts);
    AG_HIP(hipGetLastError());
  }
  AG_HIP(hipMemcpyAsync(counts, d_counts, sizeof(int64_t) * N, hipMemcpyDeviceToHost, st));
  AG_HIP(hipStreamSynchronize(st));
  return AG_OK;
}

int ag_bidder_update(ag_ctx *c, const ag_shading_samples *s, const int32_t *agents, const float *noise,
                     const int64_t *noise_offsets, int32_t noise_epochs, int32_t *epochs, int32_t *status,
                     float *traces, void *stream) {
  if (!c || !s || !noise_offsets) return ag_set_error(AG_ERR_INVALID, "ag_bidder_update: null argument");
  AG_CHECK_STRUCT(s, "ag_bidder_update", "ag_shading_samples");
  if (!s->ctr || !s->value || !s->propensity || !s->won || !s->order)
    return ag_set_error(AG_ERR_INVALID, "ag_bidder_update: the store needs ctr, value, propensity, won, order");
  if (!c->dr_loaded) return ag_set_error(AG_ERR_STATE, "ag_bidder_update: ag_set_dr_state not called");
  AgDeviceGuard g(c->device);
  const int N = c->shape.num_agents;
  hipStream_t st = (hipStream_t)stream;
  std::vector<int64_t> cnt(N), off;
  SortedRecs SR;
  if (int rc = sort_records(c, s, cnt, off, SR, st)) return rc;
  ag_dr_ws &w = c->dr;
  const int64_t *d_off = SR.d_off;
  double *b_ctr = SR.ctr, *b_val = SR.val, *b_gam = SR.gam, *b_prop = SR.prop, *b_util = SR.util, *b_eu = SR.eu;
  uint8_t *b_won = SR.won;
  int64_t *d_noff = w.scratch;                       // [N] noise offsets
  int32_t *d_epochs = (int32_t *)(w.scratch + N);     // [N][3] epochs, then [N] status
  int32_t *d_stat = d_epochs + 3 * (size_t)N;
  AG_HIP(hipMemcpyAsync(d_noff, noise_offsets, sizeof(int64_t) * N, hipMemcpyHostToDevice, st));
  AG_HIP(hipMemsetAsync(d_epochs, 0, sizeof(int32_t) * 4 * N, st));
  // Workgroups per learning bidder, co-resident (cooperative launch) when an agent has
  // several; capped to the resident grid (occupancy with the phase's largest record cache).
  // With AG_OPT_BIDDER_BLOCK_SAMPLES set: one per that many records. By default the
  // exact-sum learners (ValueLearning, DoublyRobust: results independent of the split)
  // share the resident grid in proportion to their records, >= kMinChunk records per
  // workgroup; a PolicyLearningBidder (fixed-order float sums: its result follows the split)
  // keeps one workgroup per kBidderChunk records. Both phases use the same rule with their
  // own grid.
  // k_bidder_train, one group of workgroups per learner, by default: measured on the bench's
  // populations (profiles/r04j_*), the pipelined launches (k_bidder_pipe, every learner in
  // every workgroup) lose -- each round pays one epoch's serial step and tree climb per
  // learner on 1/A of the work, 1.4-3.4x the time. AG_BIDDER_PIPE=1 takes the pipe for the
  // exact-sum learners (A/B); ag_bidder_rp_run (one learner of the drop-in update at a time,
  // where the alternative is a launch per epoch) always does.
  std::vector<int32_t> pipe_slots, pipe_mask(N, 0);
  {
    const char *e = getenv("AG_BIDDER_PIPE");
    const bool off = !(e && e[0] == '1') || c->bidder_chunk > 0;
    for (int a = 0; a < N && !off; ++a) {
      const int bk = c->h_bkind[a];
      // (a learner without logs takes k_bidder_train's no-logs path: fallback or error)
      if ((bk == AG_BIDDER_VALUE_LEARNING || bk == AG_BIDDER_DOUBLY_ROBUST) && !(agents && !agents[a]) && cnt[a] > 0)
        pipe_slots.push_back(a);
    }
    if ((int)pipe_slots.size() > kPipeMaxAgents) pipe_slots.clear();
    for (int a : pipe_slots) pipe_mask[a] = 1;
  }
  auto is_learner = [&](int a) {
    const int bk = c->h_bkind[a];
    return (bk == AG_BIDDER_VALUE_LEARNING || bk == AG_BIDDER_POLICY_LEARNING || bk == AG_BIDDER_DOUBLY_ROBUST) &&
           !(agents && !agents[a]) && !pipe_mask[a];
  };
  struct Plan {
    const void *fn = nullptr;
    std::vector<int32_t> nblk, blk_agent, blk_rank, bar_off;
    int G = 0, lines = 0, nf = 0;
    bool multi = false;
    int64_t rcap = 0;
    size_t dyn = 0;
  };
  auto plan = [&](int ph, Plan &P) -> int {
    P.fn = ph == 0 ? (const void *)k_bidder_train<0> : (const void *)k_bidder_train<1>;
    const size_t lds_budget = ph == 0 ? kRecLdsBytes0 : kRecLdsBytes;
    int &coop_blocks = ph == 0 ? w.coop_blocks0 : w.coop_blocks;
    if (!coop_blocks) {
      int per_cu = 0, cus = 0;
      AG_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, P.fn, kDrThreads, lds_budget));
      AG_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device));
      coop_blocks = per_cu * cus > 0 ? per_cu * cus : 1;
    }
    std::vector<int32_t> &nblk = P.nblk;
    nblk.assign(N, 0);
    int64_t want = 0, exact_recs = 0, fixed_blocks = 0;
    int nf = 0;  // float fields of the record cache: 3 (win-rate, ValueLearning), 5 (PolicyLearning), 6 (DR)
    for (int a = 0; a < N; ++a) {
      const int bk = c->h_bkind[a];
      if (!is_learner(a) || (ph == 0 && bk == AG_BIDDER_POLICY_LEARNING)) continue;
      nf = std::max(nf, ph == 0 ? 3 : (bk == AG_BIDDER_DOUBLY_ROBUST ? 6 : (bk == AG_BIDDER_POLICY_LEARNING ? 5 : 3)));
      if (c->bidder_chunk > 0 || bk == AG_BIDDER_POLICY_LEARNING) {
        const int64_t chunk = c->bidder_chunk > 0 ? c->bidder_chunk : kBidderChunk;
        nblk[a] = cnt[a] > 0 ? (int32_t)((cnt[a] + chunk - 1) / chunk) : 1;
        fixed_blocks += nblk[a];
      } else {
        exact_recs += cnt[a];
        nblk[a] = -1;
      }
    }
    for (int a = 0; a < N; ++a) {
      if (nblk[a] < 0) {
        const int64_t avail = std::max<int64_t>(1, coop_blocks - fixed_blocks);
        const int64_t share = exact_recs > 0 ? (int64_t)((double)avail * (double)cnt[a] / (double)exact_recs) : 1;
        nblk[a] = (int32_t)std::max<int64_t>(1, std::min<int64_t>((cnt[a] + kMinChunk - 1) / kMinChunk, share));
      }
      want += nblk[a];
    }
    if (want > coop_blocks) {  // share the resident grid out
      const double f = (double)coop_blocks / (double)want;
      for (int a = 0; a < N; ++a)
        if (nblk[a] > 1) nblk[a] = (int32_t)(nblk[a] * f) > 1 ? (int32_t)(nblk[a] * f) : 1;
    }
    int64_t most = 0;  // records of the largest workgroup chunk
    P.bar_off.assign(N, 0);
    for (int a = 0; a < N; ++a) {
      P.multi |= nblk[a] > 1;
      if (nblk[a]) most = std::max<int64_t>(most, (cnt[a] + nblk[a] - 1) / nblk[a]);
      P.bar_off[a] = P.lines;
      P.lines += bar_lines(nblk[a]) + agcoop::group_lines(nblk[a]);  // (the tree's, then the grouped sums')
      for (int r = 0; r < nblk[a]; ++r) {
        P.blk_agent.push_back(a);
        P.blk_rank.push_back(r);
      }
    }
    P.G = (int)P.blk_agent.size();
    if (P.multi && P.G > coop_blocks)
      return ag_set_error(AG_ERR_UNSUPPORTED, "ag_bidder_update: %d learning bidders need more co-resident "
                          "workgroups (%d) than the device holds (%d)", N, P.G, coop_blocks);
    // record cache: [nf][cap] floats + [cap] bytes, cap a multiple of the block size
    const int64_t rcap_fit = nf ? (int64_t)lds_budget / (4 * nf + 1) / kDrThreads * kDrThreads : 0;
    P.rcap = std::min<int64_t>(rcap_fit, (most + kDrThreads - 1) / kDrThreads * kDrThreads);
    if (c->bidder_cache >= 0) P.rcap = std::min<int64_t>(P.rcap, c->bidder_cache / kDrThreads * kDrThreads);
    P.nf = nf;
    P.dyn = ((size_t)P.rcap * (4 * nf + 1) + 15) / 16 * 16;
    return AG_OK;
  };
  Plan P0, P1;
  if (int rc = plan(0, P0)) return rc;
  if (int rc = plan(1, P1)) return rc;
  // device tables (shared by the two launches, rewritten in stream order): exchange
  // partials [G][2][32] i64; barrier lines [lines][32] u32; blk_agent [G], blk_rank [G],
  // agent_nblk [N], bar_off [N] i32; win-rate models [N][4] f32 (phase 0 -> phase 1)
  const size_t gmax = (size_t)std::max(P0.G, P1.G), lmax = (size_t)std::max(P0.lines, P1.lines);
  const size_t need_coop = sizeof(int64_t) * 96 * gmax + sizeof(unsigned) * kBarLineWords * lmax +
                           sizeof(int32_t) * (2 * gmax + 2 * (size_t)N) + sizeof(float) * 4 * N + 64;
  if (need_coop > w.coop_bytes) {
    (void)hipFree(w.coop);
    w.coop = nullptr;
    w.coop_bytes = 0;
    AG_HIP(hipMalloc(&w.coop, need_coop));
    w.coop_bytes = need_coop;
  }
  int64_t *d_part = (int64_t *)w.coop;
  unsigned *d_bar = (unsigned *)(d_part + 96 * gmax);
  int32_t *d_bagent = (int32_t *)(d_bar + kBarLineWords * lmax);
  int32_t *d_brank = d_bagent + gmax;
  int32_t *d_nblk = d_brank + gmax;
  int32_t *d_baroff = d_nblk + N;
  float *d_wr = (float *)(d_baroff + N);
  auto launch = [&](const Plan &P) -> int {
    if (P.G == 0) return AG_OK;
    AG_HIP(hipMemcpyAsync(d_bagent, P.blk_agent.data(), sizeof(int32_t) * P.G, hipMemcpyHostToDevice, st));
    AG_HIP(hipMemcpyAsync(d_brank, P.blk_rank.data(), sizeof(int32_t) * P.G, hipMemcpyHostToDevice, st));
    AG_HIP(hipMemcpyAsync(d_nblk, P.nblk.data(), sizeof(int32_t) * N, hipMemcpyHostToDevice, st));
    AG_HIP(hipMemcpyAsync(d_baroff, P.bar_off.data(), sizeof(int32_t) * N, hipMemcpyHostToDevice, st));
    if (P.lines) AG_HIP(hipMemsetAsync(d_bar, 0, sizeof(unsigned) * kBarLineWords * P.lines, st));
    if (P.multi) AG_HIP(hipMemsetAsync(d_part, 0, sizeof(int64_t) * 96 * (size_t)P.G, st));  // accumulators
    DrRecords R{b_ctr, b_val, b_gam, b_prop, b_util, b_won};
    const int32_t *cbk = c->d_bkind, *cmode = w.mode, *cinit = w.init, *cbo = d_baroff;
    const int64_t *coff = d_off, *cnoff = d_noff;
    double *ceu = b_eu;
    float *cstate = w.state, *ctr = traces, *cwr = d_wr;
    int cne = noise_epochs;
    uint64_t cseed = c->fit_noise_seed;
    const double *ctab = w.adam_tab;
    int cnf = P.nf;
    int64_t ccap = P.rcap;
    void *args[] = {&cbk,  &cmode,  &d_bagent, &d_brank, &d_nblk, &coff,  &R,        &ceu,
                    &cstate, &cwr,  &cinit,    &noise,   &cnoff,  &cne,   &cseed,    &ctab,
                    &d_epochs, &d_stat, &ctr,  &d_part,  &d_bar,  &cbo,   &cnf,      &ccap};
    if (P.multi)  // workgroups of one agent wait for each other: they must all be resident
      AG_HIP(hipLaunchCooperativeKernel(P.fn, dim3(P.G), dim3(kDrThreads), args, P.dyn, st));
    else
      AG_HIP(hipLaunchKernel(P.fn, dim3(P.G), dim3(kDrThreads), args, P.dyn, st));
    return AG_OK;
  };
  FitSt *pst = nullptr;
  if (!pipe_slots.empty()) {
    pst = pipe_fitst(c);
    if (!pst) return ag_set_error(AG_ERR_HIP, "ag_bidder_update: FitSt allocation failed");
    int32_t *d_pmask = (int32_t *)(pst + N);
    AG_HIP(hipMemcpyAsync(d_pmask, pipe_mask.data(), sizeof(int32_t) * N, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_rp_init, dim3((N + 255) / 256), dim3(256), 0, st, N, c->d_bkind, w.mode, d_pmask, w.state,
                       pst, 1);
    AG_HIP(hipGetLastError());
    // n_total = the counts (w.counts [N]); noise: agent a's draws of epoch e at noise_offsets[a] + e n_a
    PipeNoise nz;
    nz.noise = noise;
    nz.noise_off = d_noff;
    nz.stride = 0;
    nz.e0 = 0;
    nz.epochs = noise_epochs;
    const DrRecords R{b_ctr, b_val, b_gam, b_prop, b_util, b_won};
    if (int rc = pipe_run(c, pipe_slots, cnt, R, b_eu, d_off, w.counts, pst, nullptr, nz, traces, 3, st)) return rc;
  }
  if (int rc = launch(P0)) return rc;
  if (int rc = launch(P1)) return rc;
  std::vector<int32_t> h(4 * (size_t)N);
  AG_HIP(hipMemcpyAsync(h.data(), d_epochs, sizeof(int32_t) * 4 * N, hipMemcpyDeviceToHost, st));
  AG_HIP(hipStreamSynchronize(st));
  if (pst) {  // the pipe's learners: epochs, status and (unless out of noise) their models
    std::vector<FitSt> fs(N);
    std::vector<float> state(16 * (size_t)N);
    AG_HIP(hipMemcpy(fs.data(), pst, sizeof(FitSt) * N, hipMemcpyDeviceToHost));
    AG_HIP(hipMemcpy(state.data(), w.state, sizeof(float) * 16 * N, hipMemcpyDeviceToHost));
    for (int a : pipe_slots) {
      const FitSt &f = fs[a];
      for (int j = 0; j < 3; ++j) h[3 * a + j] = f.ep[j];
      int stt = f.status;
      if (f.fit != kFitDone) {  // waits for noise epochs past noise_epochs: not applied
        stt = -3;
        h[3 * a + 2] = f.epoch;
      } else if (stt != 1) {
        for (int j = 0; j < 4; ++j) state[16 * (size_t)a + j] = f.wr[j];
        for (int j = 0; j < 12; ++j) state[16 * (size_t)a + 4 + j] = f.pol[j];
      }
      h[3 * (size_t)N + a] = stt;
    }
    AG_HIP(hipMemcpy(w.state, state.data(), sizeof(float) * 16 * N, hipMemcpyHostToDevice));
  }
  if (epochs) memcpy(epochs, h.data(), sizeof(int32_t) * 3 * N);
  if (status) memcpy(status, h.data() + 3 * (size_t)N, sizeof(int32_t) * N);
  static const char *names[] = {"", "", "ValueLearningBidder", "PolicyLearningBidder", "DoublyRobustBidder"};
  for (int a = 0; a < N; ++a) {
    const int bk = c->h_bkind[a];
    if (h[3 * N + a] == -1)
      return ag_set_error(AG_ERR_INVALID, "agent %d: %s.update without logs", a, names[bk]);
    if (h[3 * N + a] == -2)
      return ag_set_error(AG_ERR_INVALID, "agent %d: %s: NAN DETECTED! in losses (src/Bidder.py:%d)", a, names[bk],
                          bk == AG_BIDDER_DOUBLY_ROBUST ? 592 : 409);
  }
  // from now on the agents bid from what they fitted (src/Bidder.py:321, :430, :612-613):
  // 1 = the policy, 2 = the win-rate search (ValueLearningBidder 'search'); 0 after the
  // ValueLearningBidder's no-win fallback (:206-211)
  std::vector<int32_t> init(N), mode(N);
  AG_HIP(hipMemcpy(init.data(), w.init, sizeof(int32_t) * N, hipMemcpyDeviceToHost));
  AG_HIP(hipMemcpy(mode.data(), w.mode, sizeof(int32_t) * N, hipMemcpyDeviceToHost));
  for (int a = 0; a < N; ++a) {
    const int bk = c->h_bkind[a];
    if ((agents && !agents[a]) || h[3 * N + a] == -3) continue;  // not updated
    if (bk == AG_BIDDER_DOUBLY_ROBUST || bk == AG_BIDDER_POLICY_LEARNING)
      init[a] = AG_LEARNER_POLICY;
    else if (bk == AG_BIDDER_VALUE_LEARNING)
      init[a] = h[3 * N + a] == 1 ? AG_LEARNER_UNINITIALISED
                                  : (mode[a] == AG_VL_POLICY ? AG_LEARNER_POLICY : AG_LEARNER_SEARCH);
  }
  AG_HIP(hipMemcpy(w.init, init.data(), sizeof(int32_t) * N, hipMemcpyHostToDevice));
  learner_flags(c, init.data());
  return AG_OK;
}

int ag_dr_update(ag_ctx *c, const ag_shading_samples *s, const float *noise, const int64_t *noise_offsets,
                 int32_t noise_epochs, int32_t *epochs, float *traces, void *stream) {
  std::vector<int32_t> stat(c->shape.num_agents);
  if (int rc = ag_bidder_update(c, s, nullptr, noise, noise_offsets, noise_epochs, epochs, stat.data(), traces, stream))
    return rc;
  for (int a = 0; a < c->shape.num_agents; ++a)
    if (stat[a] == -3)
      return ag_set_error(AG_ERR_INVALID, "agent %d: the DR fit needs more than %d noise epochs", a, noise_epochs);
  return AG_OK;
}

// ---- resumable / record-parallel training (k_bidder_epoch) ----
int ag_bidder_rp_begin(ag_ctx *c, const ag_shading_samples *s, const int32_t *agents, const int64_t *records_total,
                       const int64_t *records_base, int64_t *totals, void *stream) {
  if (!c || !s || !totals) return ag_set_error(AG_ERR_INVALID, "ag_bidder_rp_begin: null argument");
  AG_CHECK_STRUCT(s, "ag_bidder_rp_begin", "ag_shading_samples");
  if (!s->ctr || !s->value || !s->propensity || !s->won || !s->order)
    return ag_set_error(AG_ERR_INVALID, "ag_bidder_rp_begin: the store needs ctr, value, propensity, won, order");
  if (!c->dr_loaded) return ag_set_error(AG_ERR_STATE, "ag_bidder_rp_begin: ag_set_dr_state not called");
  AgDeviceGuard g(c->device);
  const int N = c->shape.num_agents;
  hipStream_t st = (hipStream_t)stream;
  ag_dr_ws &w = c->dr;
  ag_dr_rp &rp = w.rp;
  std::vector<int32_t> mode(N), mask(N, 0);
  AG_HIP(hipMemcpy(mode.data(), w.mode, sizeof(int32_t) * N, hipMemcpyDeviceToHost));
  for (int a = 0; a < N; ++a) {
    const int bk = c->h_bkind ? c->h_bkind[a] : -1;
    if (agents && !agents[a]) continue;
    if (bk == AG_BIDDER_DOUBLY_ROBUST || bk == AG_BIDDER_VALUE_LEARNING) mask[a] = 1;
    else if (bk == AG_BIDDER_POLICY_LEARNING && agents)
      return ag_set_error(AG_ERR_UNSUPPORTED, "ag_bidder_rp_begin: agent %d: PolicyLearningBidder fits use "
                          "fixed-order float sums (their result follows the record split): ag_bidder_update", a);
  }
  std::vector<int64_t> cnt(N), off;
  SortedRecs SR;
  if (int rc = sort_records(c, s, cnt, off, SR, st)) return rc;
  // workgroups: one per kRpChunk of an agent's records on this rank, at least one per trained
  // agent (a rank without records of it still steps its state and adds zeros)
  constexpr int64_t kRpChunk = 2048;
  std::vector<int32_t> nblk(N, 0), blk_agent, blk_rank, bar_off(N, 0);
  int lines = 0;
  for (int a = 0; a < N; ++a) {
    if (!mask[a]) continue;
    nblk[a] = (int32_t)std::max<int64_t>(1, (cnt[a] + kRpChunk - 1) / kRpChunk);
    bar_off[a] = lines;
    lines += std::max(1, agcoop::bar_lines(nblk[a]));
    for (int r = 0; r < nblk[a]; ++r) {
      blk_agent.push_back(a);
      blk_rank.push_back(r);
    }
  }
  const int G = (int)blk_agent.size();
  if ((size_t)G > rp.cap_g || (size_t)lines > rp.cap_lines || !rp.st || !rp.acc || !rp.tables) {
    (void)hipFree(rp.st);
    (void)hipFree(rp.acc);
    (void)hipFree(rp.tables);
    rp.st = nullptr;
    rp.acc = nullptr;
    rp.tables = nullptr;
    // capacities zero until every buffer is allocated: a failed allocation leaves the
    // workspace empty, and the next call allocates it again
    rp.cap_g = 0;
    rp.cap_lines = 0;
    const size_t cap_g = (size_t)G + 64, cap_lines = (size_t)lines + 16;
    AG_HIP(hipMalloc(&rp.st, sizeof(FitSt) * 2 * (size_t)N));
    // accumulator rows and barrier lines: [cap_lines][32] each
    AG_HIP(hipMalloc(&rp.acc, (sizeof(int64_t) + sizeof(unsigned)) * 32 * cap_lines));
    AG_HIP(hipMalloc(&rp.tables, sizeof(int32_t) * (2 * cap_g + 3 * (size_t)N) + sizeof(int64_t) * 2 * N + 16));
    rp.cap_g = cap_g;
    rp.cap_lines = cap_lines;
  }
  rp.bar = (unsigned *)(rp.acc + 32 * rp.cap_lines);
  int32_t *d_bagent = rp.tables, *d_brank = d_bagent + rp.cap_g, *d_nblk = d_brank + rp.cap_g,
          *d_baroff = d_nblk + N, *d_mask = d_baroff + N;
  rp.ntot = (int64_t *)(((uintptr_t)(d_mask + N) + 15) & ~(uintptr_t)15);
  rp.mask = d_mask;
  AG_HIP(hipMemcpyAsync(d_bagent, blk_agent.data(), sizeof(int32_t) * G, hipMemcpyHostToDevice, st));
  AG_HIP(hipMemcpyAsync(d_brank, blk_rank.data(), sizeof(int32_t) * G, hipMemcpyHostToDevice, st));
  AG_HIP(hipMemcpyAsync(d_nblk, nblk.data(), sizeof(int32_t) * N, hipMemcpyHostToDevice, st));
  AG_HIP(hipMemcpyAsync(d_baroff, bar_off.data(), sizeof(int32_t) * N, hipMemcpyHostToDevice, st));
  AG_HIP(hipMemcpyAsync(d_mask, mask.data(), sizeof(int32_t) * N, hipMemcpyHostToDevice, st));
  std::vector<int64_t> nt(2 * (size_t)N);
  for (int a = 0; a < N; ++a) {
    nt[a] = records_total ? records_total[a] : cnt[a];
    nt[N + a] = records_base ? records_base[a] : 0;
    if (mask[a] && nt[a] < 1)
      return ag_set_error(AG_ERR_INVALID, "agent %d: %s.update without logs", a,
                          c->h_bkind[a] == AG_BIDDER_DOUBLY_ROBUST ? "DoublyRobustBidder" : "ValueLearningBidder");
    if (nt[N + a] < 0 || nt[N + a] + cnt[a] > nt[a])
      return ag_set_error(AG_ERR_INVALID, "ag_bidder_rp_begin: agent %d: records_base %lld + %lld local records "
                          "> records_total %lld", a, (long long)nt[N + a], (long long)cnt[a], (long long)nt[a]);
  }
  AG_HIP(hipMemcpyAsync(rp.ntot, nt.data(), sizeof(int64_t) * 2 * N, hipMemcpyHostToDevice, st));
  if (lines) AG_HIP(hipMemsetAsync(rp.acc, 0, (sizeof(int64_t) + sizeof(unsigned)) * 32 * rp.cap_lines, st));
  AG_HIP(hipMemsetAsync(totals, 0, sizeof(int64_t) * 2 * 32 * (size_t)N, st));
  hipLaunchKernelGGL(k_rp_init, dim3((N + 255) / 256), dim3(256), 0, st, N, c->d_bkind, w.mode, d_mask, w.state,
                     (FitSt *)rp.st, 2);
  AG_HIP(hipGetLastError());
  if (int rc = dr_ws_ready(c)) return rc;  // the Adam table
  rp.G = G;
  rp.lines = lines;
  rp.k = 0;
  rp.totals = totals;
  rp.noise = nullptr;
  rp.noise_n = 0;
  rp.noise_e0 = rp.noise_epochs = 0;
  rp.n_local = SR.n;
  rp.single = true;
  for (int a = 0; a < N; ++a)
    if (mask[a] && (nt[a] != cnt[a] || nt[N + a] != 0)) rp.single = false;
  rp.active = true;
  (void)mode;
  return AG_OK;
}

// The rest of a one-rank resumable update in persistent launches (k_bidder_pipe): every
// learner under training runs until it is done or waits for the next noise window
// (ag_bidder_rp_noise) -- ag_bidder_rp_poll tells which; ag_bidder_rp_end applies the result.
// The launches read and write the same FitSt as ag_bidder_rp_epoch (which it may follow or
// precede), so the two mix freely.
int ag_bidder_rp_run(ag_ctx *c, float *traces, void *stream) {
  if (!c || !c->dr.rp.active) return ag_set_error(AG_ERR_STATE, "ag_bidder_rp_run: no ag_bidder_rp_begin");
  ag_dr_ws &w = c->dr;
  ag_dr_rp &rp = w.rp;
  if (!rp.single)
    return ag_set_error(AG_ERR_UNSUPPORTED, "ag_bidder_rp_run: this rank holds part of the learners' records "
                        "(records_total / records_base): the ranks' sums meet per epoch, ag_bidder_rp_epoch");
  AgDeviceGuard g(c->device);
  const int N = c->shape.num_agents;
  hipStream_t st = (hipStream_t)stream;
  std::vector<int32_t> mask(N);
  std::vector<int64_t> cnt(N + 1);
  std::vector<FitSt> h(N);
  FitSt *S = (FitSt *)rp.st + (size_t)(rp.k & 1) * N;
  AG_HIP(hipMemcpyAsync(mask.data(), rp.mask, sizeof(int32_t) * N, hipMemcpyDeviceToHost, st));
  AG_HIP(hipMemcpyAsync(cnt.data(), w.counts + N, sizeof(int64_t) * (N + 1), hipMemcpyDeviceToHost, st));
  AG_HIP(hipMemcpyAsync(h.data(), S, sizeof(FitSt) * N, hipMemcpyDeviceToHost, st));
  AG_HIP(hipStreamSynchronize(st));
  std::vector<int32_t> slots;
  std::vector<int64_t> n(N, 0);
  bool ph0 = false;
  for (int a = 0; a < N; ++a) {
    n[a] = cnt[a + 1] - cnt[a];
    if (mask[a] && h[a].fit != kFitDone) {
      slots.push_back(a);
      ph0 |= h[a].fit == kFitWins || h[a].fit == kFitWr;
    }
  }
  if (slots.empty()) return AG_OK;
  if ((int)slots.size() > kPipeMaxAgents) {  // per-epoch launches, polled, until done or waiting
    std::vector<int32_t> fit(N), ep(N), need(N);
    for (;;) {
      if (int rc = ag_bidder_rp_epoch(c, 64, nullptr, traces, stream)) return rc;
      if (int rc = ag_bidder_rp_poll(c, fit.data(), ep.data(), need.data(), stream)) return rc;
      bool busy = false;
      for (int a = 0; a < N; ++a) busy |= mask[a] && fit[a] >= 0 && need[a] < 0;
      if (!busy) return AG_OK;
    }
  }
  double *eu = nullptr;
  const DrRecords R = sorted_view(w, rp.n_local, &eu);
  PipeNoise nz;
  nz.noise = rp.noise;
  nz.stride = rp.noise_n;
  nz.e0 = rp.noise_e0;
  nz.epochs = rp.noise_epochs;
  return pipe_run(c, slots, n, R, eu, w.counts + N, rp.ntot, S, rp.totals + (size_t)((rp.k + 1) & 1) * 32 * N, nz,
                  traces, ph0 ? 3 : 2, st);
}

int ag_bidder_rp_noise(ag_ctx *c, const float *noise, int64_t noise_n, int32_t first_epoch, int32_t epochs) {
  if (!c || !c->dr.rp.active) return ag_set_error(AG_ERR_STATE, "ag_bidder_rp_noise: no ag_bidder_rp_begin");
  if (noise && (noise_n < 1 || first_epoch < 0 || epochs < 0))
    return ag_set_error(AG_ERR_INVALID, "ag_bidder_rp_noise: bad window");
  ag_dr_rp &rp = c->dr.rp;
  rp.noise = noise;
  rp.noise_n = noise_n;
  rp.noise_e0 = first_epoch;
  rp.noise_epochs = epochs;
  return AG_OK;
}

int ag_bidder_rp_epoch(ag_ctx *c, int32_t launches, int64_t *launch_index, float *traces, void *stream) {
  if (!c || !c->dr.rp.active) return ag_set_error(AG_ERR_STATE, "ag_bidder_rp_epoch: no ag_bidder_rp_begin");
  if (launches < 0) return ag_set_error(AG_ERR_INVALID, "ag_bidder_rp_epoch: launches < 0");
  AgDeviceGuard g(c->device);
  const int N = c->shape.num_agents;
  hipStream_t st = (hipStream_t)stream;
  ag_dr_ws &w = c->dr;
  ag_dr_rp &rp = w.rp;
  const int64_t cap = rp.n_local > 0 ? rp.n_local : 1;
  double *b_ctr = (double *)w.buf;
  DrRecords R{b_ctr, b_ctr + cap, b_ctr + 2 * cap, b_ctr + 3 * cap, b_ctr + 4 * cap,
              (const uint8_t *)((uint32_t *)((uint64_t *)(b_ctr + 6 * cap) + 2 * cap) + 2 * cap)};
  double *b_eu = b_ctr + 5 * cap;
  int32_t *d_bagent = rp.tables, *d_brank = d_bagent + rp.cap_g, *d_nblk = d_brank + rp.cap_g, *d_baroff = d_nblk + N;
  FitSt *S = (FitSt *)rp.st;
  for (int32_t l = 0; l < launches; ++l) {
    const int64_t k = rp.k;
    if (rp.G > 0)
      hipLaunchKernelGGL(k_bidder_epoch, dim3(rp.G), dim3(kDrThreads), 0, st, c->d_bkind, w.mode, w.init, d_bagent,
                         d_brank, d_nblk, w.counts + N, rp.ntot, rp.ntot + N, R, b_eu, S + (size_t)(k & 1) * N,
                         S + (size_t)((k + 1) & 1) * N, rp.totals + (size_t)((k + 1) & 1) * 32 * N,
                         rp.totals + (size_t)(k & 1) * 32 * N, rp.acc, rp.bar, d_baroff, rp.noise, rp.noise_n,
                         rp.noise_e0, rp.noise_epochs, c->fit_noise_seed, w.adam_tab, traces);
    AG_HIP(hipGetLastError());
    rp.k = k + 1;
  }
  if (launch_index) *launch_index = rp.k - 1;  // the last launch: its totals are at totals + 32 N (index & 1)
  return AG_OK;
}

int ag_bidder_rp_poll(ag_ctx *c, int32_t *fit, int32_t *epoch, int32_t *need_noise, void *stream) {
  if (!c || !c->dr.rp.active) return ag_set_error(AG_ERR_STATE, "ag_bidder_rp_poll: no ag_bidder_rp_begin");
  AgDeviceGuard g(c->device);
  const int N = c->shape.num_agents;
  ag_dr_rp &rp = c->dr.rp;
  std::vector<FitSt> h(N);
  hipStream_t st = (hipStream_t)stream;
  AG_HIP(hipMemcpyAsync(h.data(), (FitSt *)rp.st + (size_t)(rp.k & 1) * N, sizeof(FitSt) * N, hipMemcpyDeviceToHost,
                        st));
  AG_HIP(hipStreamSynchronize(st));
  for (int a = 0; a < N; ++a) {
    if (fit) fit[a] = h[a].fit == kFitDone ? -1 : h[a].fit;
    if (epoch) epoch[a] = h[a].epoch;
    if (need_noise) need_noise[a] = h[a].need_noise ? h[a].epoch : -1;
  }
  return AG_OK;
}

int ag_bidder_rp_end(ag_ctx *c, int32_t *epochs, int32_t *status, void *stream) {
  if (!c || !c->dr.rp.active) return ag_set_error(AG_ERR_STATE, "ag_bidder_rp_end: no ag_bidder_rp_begin");
  AgDeviceGuard g(c->device);
  const int N = c->shape.num_agents;
  ag_dr_ws &w = c->dr;
  ag_dr_rp &rp = w.rp;
  hipStream_t st = (hipStream_t)stream;
  std::vector<FitSt> h(N);
  std::vector<int32_t> mask(N), init(N), mode(N);
  std::vector<float> state(16 * (size_t)N);
  AG_HIP(hipMemcpyAsync(h.data(), (FitSt *)rp.st + (size_t)(rp.k & 1) * N, sizeof(FitSt) * N, hipMemcpyDeviceToHost,
                        st));
  AG_HIP(hipMemcpyAsync(mask.data(), rp.mask, sizeof(int32_t) * N, hipMemcpyDeviceToHost, st));
  AG_HIP(hipStreamSynchronize(st));
  rp.active = false;
  for (int a = 0; a < N; ++a)
    if (mask[a] && h[a].fit != kFitDone)
      return ag_set_error(AG_ERR_STATE, "ag_bidder_rp_end: agent %d is still training (fit %d, epoch %d)", a,
                          h[a].fit, h[a].epoch);
  AG_HIP(hipMemcpy(state.data(), w.state, sizeof(float) * 16 * N, hipMemcpyDeviceToHost));
  AG_HIP(hipMemcpy(init.data(), w.init, sizeof(int32_t) * N, hipMemcpyDeviceToHost));
  AG_HIP(hipMemcpy(mode.data(), w.mode, sizeof(int32_t) * N, hipMemcpyDeviceToHost));
  static const char *names[] = {"", "", "ValueLearningBidder", "PolicyLearningBidder", "DoublyRobustBidder"};
  int rc = AG_OK;
  for (int a = 0; a < N; ++a) {
    if (epochs) epochs[3 * a] = epochs[3 * a + 1] = epochs[3 * a + 2] = 0;
    if (status) status[a] = 0;
    if (!mask[a]) continue;
    if (epochs)
      for (int j = 0; j < 3; ++j) epochs[3 * a + j] = h[a].ep[j];
    if (status) status[a] = h[a].status;
    const int bk = c->h_bkind[a];
    if (h[a].status == -2 && rc == AG_OK)
      rc = ag_set_error(AG_ERR_INVALID, "agent %d: %s: NAN DETECTED! in losses (src/Bidder.py:%d)", a, names[bk],
                        bk == AG_BIDDER_DOUBLY_ROBUST ? 592 : 409);
    if (h[a].status != 1) {  // the fallback trains nothing (src/Bidder.py:206-211)
      for (int j = 0; j < 4; ++j) state[16 * (size_t)a + j] = h[a].wr[j];
      for (int j = 0; j < 12; ++j) state[16 * (size_t)a + 4 + j] = h[a].pol[j];
    }
    // from now on the agent bids from what it fitted (ag_bidder_update's rule)
    if (bk == AG_BIDDER_DOUBLY_ROBUST)
      init[a] = AG_LEARNER_POLICY;
    else
      init[a] = h[a].status == 1 ? AG_LEARNER_UNINITIALISED
                                 : (mode[a] == AG_VL_POLICY ? AG_LEARNER_POLICY : AG_LEARNER_SEARCH);
  }
  AG_HIP(hipMemcpy(w.state, state.data(), sizeof(float) * 16 * N, hipMemcpyHostToDevice));
  AG_HIP(hipMemcpy(w.init, init.data(), sizeof(int32_t) * N, hipMemcpyHostToDevice));
  learner_flags(c, init.data());
  return rc;
}

int ag_set_bidder_modes(ag_ctx *c, const int32_t *modes) {
  if (!c || !modes) return ag_set_error(AG_ERR_INVALID, "ag_set_bidder_modes: null argument");
  AgDeviceGuard g(c->device);
  if (int rc = dr_ws_ready(c)) return rc;
  const int N = c->shape.num_agents;
  for (int a = 0; a < N; ++a) {
    const int bk = c->h_bkind ? c->h_bkind[a] : -1;
    if (bk == AG_BIDDER_VALUE_LEARNING && modes[a] != AG_VL_SEARCH && modes[a] != AG_VL_POLICY)
      return ag_set_error(AG_ERR_INVALID, "agent %d: ValueLearningBidder inference must be 'search' or 'policy'", a);
    if (bk == AG_BIDDER_POLICY_LEARNING && (modes[a] < AG_PL_LOSS_REINFORCE || modes[a] > AG_PL_LOSS_PPO))
      return ag_set_error(AG_ERR_UNSUPPORTED,
                          "agent %d: PolicyLearningBidder loss %d (REINFORCE, REINFORCE_offpolicy, TRPO, PPO are built)",
                          a, modes[a]);
  }
  AG_HIP(hipMemcpy(c->dr.mode, modes, sizeof(int32_t) * N, hipMemcpyHostToDevice));
  return AG_OK;
}

}  // extern "C"
