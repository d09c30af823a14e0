// ag_sim.h -- the fused simulate kernel template (shared by the per-P translation units
// ag_sim_p.hip and the C-ABI in ag_kernels.hip). See ag_kernels.hip for the overview.
#pragma once
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>

#include "auctiongym.h"
#include "ag_exp.h"
#include "ag_exp_table.h"
#include "ag_log1p.h"
#include "ag_philox.h"

namespace ag {

// Build knobs (A/B variants, `make variant`): AG_PREFETCH software-pipelines the next
// tile's input loads; AG_MIN_WAVES caps VGPRs via launch bounds; AG_MAX_REPLICAS caps the
// per-lane counter replicas (LDS per block).
#ifndef AG_POLICY_COMPACT
#define AG_POLICY_COMPACT 1  // early path: fitted-policy bids compacted across the wave's slots
#endif
#ifndef AG_EARLY_COUNT
#define AG_EARLY_COUNT 1  // general kernel: per-slot stores and counter terms as slots resolve
#endif
#ifndef AG_STREAM_SYNC
#define AG_STREAM_SYNC 0  // streamed slots (P >= 3): workgroup barrier per tile (1) or per slot (2), A/B
#endif
#ifndef AG_XCD_MAP
#define AG_XCD_MAP 0  // general kernel: consecutive auction tiles to the workgroups of one XCD (A/B)
#endif
#ifndef AG_STREAM_PACK_AGENTS
#define AG_STREAM_PACK_AGENTS 0  // streamed slots (P >= 3): the counter pass's agents kept packed in registers
#endif
#ifndef AG_PREFETCH
#define AG_PREFETCH 0
#endif
#ifndef AG_GEN_MIN_WAVES
#define AG_GEN_MIN_WAVES 3  // the general kernel: <= 168 VGPRs
#endif
#ifndef AG_GEN_DOS_MIN_WAVES
#define AG_GEN_DOS_MIN_WAVES 4  // the full general build with the LR-TS width compile-time (DOS), P <= 2:
                                // 128 VGPRs (3 spilled) at 4 waves per SIMD instead of 140 at 3 --
                                // configs_2 0.212 -> 0.203 ms, configs_3 0.129 -> 0.121 ms in one
                                // process (profiles/r03s11_ab_w4.log)
#endif
#ifndef AG_TB_WIDE_MIN_WAVES
#define AG_TB_WIDE_MIN_WAVES 3  // ... at P >= 3 (streamed slots): 168 VGPRs, 2 spilled instead of 81;
                                // configs_1 at P = 8 0.658 -> 0.558 ms (profiles/r04o_ab_c1p8_tb3.log)
#endif
#ifndef AG_TB_MIN_WAVES
#define AG_TB_MIN_WAVES 4  // the general kernel for truthful bidders only: <= 128 VGPRs (115, none
                           // spilled; 5 waves: 96 VGPRs, 22 spilled, configs_1 0.160 -> 0.174 ms in
                           // one process, profiles/r04_ab_tb5.log)
#endif
#ifndef AG_TS_SCREEN
#define AG_TS_SCREEN 1  // screened Thompson item choice (ts_select)
#endif
#ifndef AG_MIN_WAVES
#define AG_MIN_WAVES 1
#endif
#ifndef AG_STREAM_GENALL
#define AG_STREAM_GENALL 0  // A/B: streamed slots for the full mix too (make variant)
#endif
#ifndef AG_STREAM_MIN_P
#define AG_STREAM_MIN_P 3  // general kernel: streamed slots (no per-slot result arrays) from this P on
#endif
#ifndef AG_MAX_REPLICAS
#define AG_MAX_REPLICAS 16
#endif
#ifndef AG_ABLATE
#define AG_ABLATE 0  // diagnostic ablations of the general kernel (see kAblate below)
#endif
#ifndef AG_TS_DMA
#define AG_TS_DMA 1  // replayed Thompson noise streamed into a per-wave LDS ring by LDS-DMA: the
                     // 256-lane shipped-shape builds (configs_1/2/3: 2-5 % in one process,
                     // profiles/r06i_ab_*.log); 0: the VGPR loads (A/B)
#endif
#ifndef AG_TS_DMA_MAXP
#define AG_TS_DMA_MAXP 8  // ... in the 256-lane builds of up to this many participants (P = 8,
                          // the streamed slots: configs_1_p8 -7 %, profiles/r06n_ab_dma8_c1p8.log)
#endif
#ifndef AG_TS_DMA_AHEAD
#define AG_TS_DMA_AHEAD 2  // ... items in flight ahead of the one being scored
#endif

constexpr int kThreads = 256;              // 4 waves of 64 lanes
#ifndef AG_LARGE_BT
#define AG_LARGE_BT 1024
#endif
constexpr int kLargeThreads = AG_LARGE_BT;  // the general kernel's workgroups for large LDS images
// ... and for the full mix at P >= 3 (streamed slots): 12 waves, <= 168 VGPRs, one workgroup
// per CU. The streamed full build at 1024 lanes (128 VGPRs) spilled; kept per-slot arrays
// spill more: configs_4 at P = 8 1.507 ms (1024, kept) / 1.624 (1024, streamed) / 1.592 (768,
// kept) / 1.387 (768, streamed), profiles/r04l_ab_c4p8.log
constexpr int kMidThreads = 768;
// k_simulate's GENERAL modes: Oracle + Truthful only; any population; allocators of any
// kind with TruthfulBidders only (no bid-shading code: fewer VGPRs, 4 waves per SIMD)
constexpr int kGenOracle = 0, kGenAll = 1, kGenTruthful = 2;
constexpr int kC = AG_NUM_COUNTERS;
// Auctions one block may resolve per launch: 1024 per counter replica keeps every replica's
// int64 sum exact (<= 1024 * P terms of magnitude < 2^50, to_fx).
constexpr int kAuctionsPerReplica = 1024;
constexpr int kMinGrid = 2048;             // 256 CUs x 8
constexpr int kMaxSimGrid = 2048;          // partial-sum workspace (>= resident blocks)
constexpr int kMaxP = 8;                   // per-lane slot registers (template range)
constexpr int kMaxD = 16;
constexpr double kFxScale = 0x1p36;        // 2^AG_FX_FRAC_BITS
constexpr double kMagic = 0x1.8p52;
constexpr int64_t kLimbMask = (int64_t(1) << AG_FX_LIMB_BITS) - 1;

// ------------------------------------------------------------------------------------
// reference arithmetic
// ------------------------------------------------------------------------------------

// numpy `items @ ctx` -> OpenBLAS dgemv_t (SURVEY §8 a5'; oracle/ag_oracle.c ora_dot):
// rows in blocks of 4 with one FMA accumulator per lane, lanes reduced (l0+l2)+(l1+l3),
// 1-3 tail rows added by contracted scalar code. `a` is in LDS, `x` in registers.
template <int D>
__device__ __forceinline__ double dot_ref(const double *__restrict__ a, const double (&x)[kMaxD]) {
  constexpr int m3 = D & 3, m1 = D - m3;
  double y = 0.0;
  if constexpr (m1 > 0) {
    double l0 = 0.0, l1 = 0.0, l2 = 0.0, l3 = 0.0;
#pragma unroll
    for (int i = 0; i < m1; i += 4) {
      l0 = fma(a[i + 0], x[i + 0], l0);
      l1 = fma(a[i + 1], x[i + 1], l1);
      l2 = fma(a[i + 2], x[i + 2], l2);
      l3 = fma(a[i + 3], x[i + 3], l3);
    }
    y = (l0 + l2) + (l1 + l3);
  }
  if constexpr (m3 == 1) y = fma(a[m1], x[m1], y);
  if constexpr (m3 == 2) y = y + fma(a[m1], x[m1], a[m1 + 1] * x[m1 + 1]);
  if constexpr (m3 == 3)
    y = y + fma(a[m1 + 2], x[m1 + 2], fma(a[m1], x[m1], a[m1 + 1] * x[m1 + 1]));
  return y;
}

// numpy Generator.binomial(1, p) from its single next_double U (src/Auction.py:65;
// numpy's inversion sampler for n = 1). The sampler compares U with exp(log(1 - p)); this
// uses 1 - p (resp. p), which differs from it by at most one ulp: the outcome can differ
// only when U lands on that ulp, probability <= 2^-53 per auction.
__device__ __forceinline__ int bernoulli(double p, double u) {
  if (p == 0.0) return 0;
  if (p <= 0.5) return u > (1.0 - p) ? 1 : 0;
  return u > p ? 0 : 1;
}

// Round x * 2^36 to the nearest integer (ties-to-even), exactly.
__device__ __forceinline__ unsigned long long to_fx(double x) {
  if (fabs(x) < 0x1p14) {
    double y = fma(x, kFxScale, kMagic);
    return (unsigned long long)(__double_as_longlong(y) - __double_as_longlong(kMagic));
  }
  if (!(fabs(x) < 0x1p26)) return 0ull;  // non-finite / absurd term: dropped
  return (unsigned long long)(long long)rint(x * kFxScale);
}

// LDS carve of k_simulate (all pieces 16-B aligned; offsets in bytes).
struct LdsLayout {
  int32_t tab, items, values, scr, scr_val, amax, akind, bkind, pg, gs, tsm, drs, dri, kag, cnt, total;
  int32_t tsr;             // generate mode: the LR-TS agents' 1 / sqrtf(q), laid out as tsm (0: none)
  int32_t items_stride;    // doubles between agents (odd: spreads agents over banks)
  int32_t values_stride;   // doubles
  int32_t scr_stride;      // floats between agents in the screening catalogue
  int32_t scr_val_stride;  // floats
  int32_t kpairs;          // item pairs in the screening catalogue (K rounded up to even)
  int32_t replicas;        // per-lane counter replicas (power of 2, <= 64)
  int32_t ncnt;            // counter slots held in LDS
  int32_t ts_do;           // LR-TS model width OE + 1 (general populations)
  int32_t tsm_stride;      // floats between agents' LR-TS means (K * ts_do, made odd)
  int32_t drs_stride;      // floats between agents' learner models (17: odd)
  int32_t pol;             // per-wave fitted-policy task slots [BT/64][64][32 B] (0: none)
};

__host__ inline int32_t align16(int64_t b) { return (int32_t)((b + 15) & ~(int64_t)15); }

// Counter slots accumulated in LDS (all exact fixed-point sums):
//   0 GROSS, 1 PAID, 2 OVERBID (FirstPrice only: price - second_price == 0 under SP),
//   3 UNDERBID, 4 BEST_EV, 5 packed counts (n_logs in bits 0-31, n_won in bits 32-63),
//   general populations only: 6 ALLOC_REGRET, 7 EST_REGRET, 8 CTR_SQERR, 9 CTR_BIAS.
// Derived at write-out: NET = GROSS - PAID. For OracleAllocator + TruthfulBidder
// populations the general slots are identically 0 (estimated CTR == true CTR and best_ev
// == true_ctr * value bit for bit) and CTR_BIAS == N_WON (est/true == 1): not accumulated.
constexpr int kOracleSlots = 6;
constexpr int kGeneralSlots = 10;
enum { kSlotGross = 0, kSlotPaid, kSlotOverbid, kSlotUnderbid, kSlotBestEv, kSlotCounts,
       kSlotAlloc, kSlotEst, kSlotSqerr, kSlotBias };

__host__ inline LdsLayout make_layout(int N, int K, int D, bool counters, bool general = false,
                                      int ts_do = 0, bool gen = false) {
  LdsLayout L;
  L.items_stride = (K * D) | 1;
  L.values_stride = K | 1;
  L.kpairs = (K + 1) / 2;
  // [pair][dim 0..7][2 items] floats; + 2 floats: the agent stride is 2 x odd dwords (mod 64),
  // so the lanes of a wave reading one (pair, dim) of up to 32 different agents hit 32
  // different 8-B bank pairs (+4 made it a multiple of 4: 16 pairs, 2-way conflicts beyond
  // 16 agents)
  L.scr_stride = L.kpairs * 16 + 2;
  L.scr_val_stride = L.kpairs * 2 + 2;
  L.ncnt = general ? kGeneralSlots : kOracleSlots;
  L.ts_do = general ? ts_do : 0;
  // agent strides odd in dwords: lanes reading the same coefficient of different agents'
  // LR-TS means / learner models hit different banks (K * 5 = 60 and 16 were multiples of 4:
  // 4- and 16-way conflicts in large populations)
  L.tsm_stride = general ? ((K * ts_do) | 1) : 0;
  L.drs_stride = 17;
  // counter replicas [slot][agent][R]: with R = 16 the 16 lanes of a 64-bit LDS atomic's lane
  // group hit 16 distinct 8-B bank pairs whatever their agents; fewer replicas put lanes l and
  // l + R on one pair. 16 kept up to 64 KB of replicas (32 agents x 10 slots = 40 KB)
  int R = AG_MAX_REPLICAS;
  while (R > 1 && (int64_t)R * N * L.ncnt * 8 > 65536) R >>= 1;
  L.replicas = R;
  int64_t b = 0;
  L.tab = 0;
  b += agexp::kExpTabLds * 8;  // ag_exp_tab + the expf table
  L.items = align16(b);
  b = L.items + (int64_t)N * L.items_stride * 8;
  L.values = align16(b);
  b = L.values + (int64_t)N * L.values_stride * 8;
  L.scr = align16(b);
  b = L.scr + (int64_t)N * L.scr_stride * 4;
  L.scr_val = align16(b);
  b = L.scr_val + (int64_t)N * L.scr_val_stride * 4;
  L.amax = align16(b);
  b = L.amax + (int64_t)N * 4;
  L.akind = align16(b);
  b = L.akind + (general ? (int64_t)N * 4 : 0);
  L.bkind = align16(b);
  b = L.bkind + (general ? (int64_t)N * 4 : 0);
  L.pg = align16(b);
  b = L.pg + (general ? (int64_t)N * 8 : 0);
  L.gs = align16(b);
  b = L.gs + (general ? (int64_t)N * 8 : 0);
  L.tsm = align16(b);
  b = L.tsm + (general ? (int64_t)N * L.tsm_stride * 4 : 0);
  L.drs = align16(b);
  b = L.drs + (general ? (int64_t)N * L.drs_stride * 4 : 0);
  L.dri = align16(b);
  b = L.dri + (general ? (int64_t)N * 4 : 0);
  L.kag = align16(b);
  b = L.kag + (general ? (int64_t)N * 4 : 0);
  L.cnt = align16(b);
  b = L.cnt + (counters ? (int64_t)R * N * L.ncnt * 8 : 0);
  L.tsr = 0;
  if (general && gen) {  // after the counters: the other offsets are those of the replay layout
    L.tsr = align16(b);
    b = L.tsr + (int64_t)N * L.tsm_stride * 4;
  }
  L.total = align16(b);
  L.pol = 0;
  return L;
}

// the per-wave task slots of the compacted fitted-policy pass (full general build, bt lanes)
__host__ inline void add_policy_tasks(LdsLayout &L, int bt) {
  L.pol = L.total;
  L.total = align16((int64_t)L.total + (int64_t)bt * 32);
}

struct SimParams {
  int32_t B;              // auctions in the batch = SoA leading dimension (B * P < 2^31)
  int32_t lo, hi;         // the auctions [lo, hi) this launch resolves
  int32_t N, K, mech;
  int32_t want_counters;
  int32_t ts_sample;      // general: LR-TS agents add ts_noise to m for the item choice
  LdsLayout lds;
  const double *items;    // global [N][K][D]
  const double *values;   // global [N][K]
  const int32_t *akind;   // general: [N] ag_allocator_kind
  const int32_t *bkind;   // general: [N] ag_bidder_kind
  const double *pg;       // general: [N] prev_gamma of shading bidders
  const double *gs;       // general: [N] gamma_sigma
  const float *tsm;       // general: [N][K][OE+1] LR-TS posterior means
  const float *drs;       // general: [N][16] DoublyRobustBidder models (NULL: none)
  const int32_t *dri;     // general: [N] fitted policy flags
  const int32_t *kag;     // general: [N] each agent's own item count (NULL: all K)
  ag_batch_in in;
  ag_batch_out out;
  int64_t *partials;      // [grid][N][AG_NUM_COUNTERS][2]
  int32_t P;              // participants per round (read by the runtime-P kernel, P = 0)
  // generate mode (k_simulate<..., GEN = true>): every input drawn in the kernel
  const float *tsq;       // [N][K][OE+1] LR-TS q (the Thompson noise's scale 1 / sqrtf(q))
  uint64_t seed, first;   // Philox key; global index of the batch's auction 0
  double scale;           // embedding_var (the contexts' scale)
};

// Screening margin. The screen ranks items by t_k = (1 + 2^(z'_k)) / v_k = 1 / (exact
// score) in f32, z'_k the f32 dot of the catalogue row pre-scaled by -log2(e), 1/v_k
// precomputed. With S = sum_d |a_d x_d| <= kPruneMaxS its relative error is
// eps <= S 2^-21 (inputs rounded to f32, D <= 8 FMAs) + |z| 2^-23 (exp2 argument) +
// 2^-22 (exp2, fma, 1/v) < 4e-5, so every item whose EXACT score is the maximum has
// t_k <= t_min (1 + eps)/(1 - eps) < t_min (1 + kPruneDelta), kPruneDelta = 2^-13 =
// 1.22e-4 > 2.01 eps: re-scoring every item under that threshold exactly keeps the exact
// argmax and all its exact ties. Lanes outside the bound (or with no finite t) re-score
// every item exactly.
constexpr float kPruneDelta = 0x1p-13f;
constexpr float kPruneMaxS = 64.0f;
constexpr int kMaxKPairs = 8;  // screened search for K <= 16
constexpr float kNegLog2e = -1.4426950408889634f;

typedef float f32x2 __attribute__((ext_vector_type(2)));

// Agent.select_item (src/Agent.py:29-42) for an OracleAllocator agent: the first k that
// maximises sigmoid(items_k . x) * value_k, with the reference's exact FP64 arithmetic.
// PRUNE: a packed-f32 pass scores all items two at a time; the f32 leader and any item
// within kPruneDelta of it are re-scored exactly, so the first-max rule and every bit of
// the chosen item's CTR / score are the reference's.
template <int D, bool PRUNE>
__device__ __forceinline__ int select_item(const double *__restrict__ itm, const double *__restrict__ vv,
                                           const float *__restrict__ scr, const float *__restrict__ sv,
                                           float amax, int K, int kpairs, const double (&x)[kMaxD],
                                           const float (&xf)[kMaxD], float xabs, const uint64_t *tab,
                                           double &ctr_best, double &score_best) {
  int best = -1;
  double best_s = 0.0, best_c = 0.0;
  auto exact = [&](int k) {
    const double c = agexp::sigmoid_fast(dot_ref<D>(itm + k * D, x), tab);
    const double sc = c * vv[k];
    if (best < 0 || sc > best_s || (sc == best_s && k < best)) {
      best = k;
      best_s = sc;
      best_c = c;
    }
  };
  if constexpr (PRUNE) {
    // f32 screen of one item pair: t = (1 + 2^z') / v of items 2p, 2p+1 (padding: +inf)
    auto screen = [&](int p) -> f32x2 {
      const float *row = scr + p * 16;
      f32x2 z = {0.0f, 0.0f};
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const f32x2 a = *reinterpret_cast<const f32x2 *>(row + 2 * d);
        const f32x2 xd = {xf[d], xf[d]};
        z = __builtin_elementwise_fma(a, xd, z);
      }
      const f32x2 e = {__builtin_amdgcn_exp2f(z.x), __builtin_amdgcn_exp2f(z.y)};
      const f32x2 iv = *reinterpret_cast<const f32x2 *>(sv + 2 * p);
      return __builtin_elementwise_fma(e, iv, iv);
    };
    // pass 1: f32 leader kf (smallest t), its t and the runner-up's
    float t1 = INFINITY, t2 = INFINITY;
    int kf = 0;
    for (int p = 0; p < kpairs; ++p) {
      const f32x2 t = screen(p);
      const float lo = fminf(t.x, t.y), hi = fmaxf(t.x, t.y);
      const int klo = t.y < t.x ? 2 * p + 1 : 2 * p;
      if (lo < t1) {
        t2 = fminf(t1, hi);
        t1 = lo;
        kf = klo;
      } else {
        t2 = fminf(t2, lo);
      }
    }
    const bool ok = (amax * xabs <= kPruneMaxS) && (t1 <= 1e30f);
    const float thr = ok ? t1 * (1.0f + kPruneDelta) : INFINITY;
    exact(kf);  // the f32 leader: every lane, no divergence
    if (!(t2 > thr)) {
      // near-tie (rare) or unscreenable lane: re-score every other item under thr
      for (int p = 0; p < kpairs; ++p) {
        const f32x2 t = screen(p);
        if (2 * p != kf && !(t.x > thr)) exact(2 * p);
        if (2 * p + 1 != kf && 2 * p + 1 < K && !(t.y > thr)) exact(2 * p + 1);
      }
    }
  } else {
    for (int k = 0; k < K; ++k) exact(k);
  }
  ctr_best = best_c;
  score_best = best_s;
  return best;
}

// ------------------------------------------------------------------------------------
// fused simulate kernel
// ------------------------------------------------------------------------------------

// W-wide SoA accesses (W = 2: one 16-B / 8-B / 2-B access per lane for two auctions).
// AG_NT_LOADS / AG_NT_STORES: non-temporal streaming of the batch inputs and outputs (each
// byte is touched once). Measured (tools/ab_libs.py, SP_Oracle shape, 2^24 auctions): 3 %
// faster back to back than cached accesses (0.501 vs 0.516 ms); on by default.
#ifndef AG_NT_LOADS
#define AG_NT_LOADS 1
#endif
#ifndef AG_NT_STORES
#define AG_NT_STORES 1
#endif
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef int i32x2 __attribute__((ext_vector_type(2)));
template <typename T>
__device__ __forceinline__ T ldg(const T *p) {
  if constexpr (AG_NT_LOADS) return __builtin_nontemporal_load(p);
  else return *p;
}
template <typename T>
__device__ __forceinline__ void stg(T *p, T v) {
  if constexpr (AG_NT_STORES) __builtin_nontemporal_store(v, p);
  else *p = v;
}
// ABI 17: winner and outcome as one word (ag_batch_out.winner_outcome)
__device__ __forceinline__ uint32_t pack_wo(int w, int oc) { return (uint32_t)w | ((uint32_t)(oc & 1) << 31); }

template <int W>
__device__ __forceinline__ void ld_f64(const double *p, double (&v)[W]) {
  if constexpr (W == 1) {
    v[0] = ldg(p);
  } else {
    const f64x2 t = ldg(reinterpret_cast<const f64x2 *>(p));
    v[0] = t.x;
    v[1] = t.y;
  }
}
template <int W>
__device__ __forceinline__ void ld_i32(const int32_t *p, int (&v)[W]) {
  if constexpr (W == 1) {
    v[0] = ldg(p);
  } else {
    const i32x2 t = ldg(reinterpret_cast<const i32x2 *>(p));
    v[0] = t.x;
    v[1] = t.y;
  }
}
template <int W>
__device__ __forceinline__ void st_f64(double *p, const double (&v)[W]) {
  if constexpr (W == 1) stg(p, v[0]);
  else stg(reinterpret_cast<f64x2 *>(p), f64x2{v[0], v[1]});
}
template <int W>
__device__ __forceinline__ void st_i32(int32_t *p, const int (&v)[W]) {
  if constexpr (W == 1) stg(p, (int32_t)v[0]);
  else stg(reinterpret_cast<i32x2 *>(p), i32x2{v[0], v[1]});
}
template <int W>
__device__ __forceinline__ void st_u8(uint8_t *p, const int (&v)[W]) {
  if constexpr (W == 1) stg(p, (uint8_t)v[0]);
  else stg(reinterpret_cast<uint16_t *>(p), (uint16_t)((v[0] & 1) | ((v[1] & 1) << 8)));
}

// LDS views of the catalogue + tables for one block
struct Lds {
  const uint64_t *tab;
  const double *items, *vals;
  const float *scr, *scr_val, *amax;
  int items_stride, values_stride, scr_stride, scr_val_stride, kpairs;
  // general populations
  const int32_t *akind, *bkind;
  const double *pg, *gs;
  const float *tsm;
  int ts_do, tsm_stride, drs_stride;
  const float *drs;
  const int32_t *dri;
  const int32_t *kag;  // general: each agent's own item count (src/main.py:61,66)
  const float *tsr;    // generate mode: the LR-TS agents' 1 / sqrtf(q) (stride tsm_stride)
  const float *ring;   // AG_TS_DMA: this wave's Thompson-noise ring (NULL: none)
  uint32_t ring_lds;   // ... its LDS byte address
};

// generate mode: one auction's Philox counter (its global index) and key
struct GenKey {
  uint32_t c0, c1, k0, k1;
};

// Where a slot's Thompson noise comes from: the HBM tiles (replay and HBM-resident synthetic
// batches) or, in generate mode, the draws ag_generate_noise would have stored there.
struct TsSrc {
  const float *nz;   // HBM: coefficient c at nz[c * 64] (NULL: no noise)
  const float *rsq;  // generate mode: the agent's 1 / sqrtf(q) [K][Do] (NULL: no noise)
  GenKey key;
  uint32_t stream;   // generate mode: 4 + slot
  // AG_TS_DMA: the wave's LDS ring of kTsDmaBufs item buffers (DOS rows of 64 floats each),
  // its LDS byte address, and the batch's item count K (wave-uniform: the DMA schedule)
  const float *ring;
  uint32_t ring_lds;
  int kg;
};

// ---- AG_TS_DMA: the replayed Thompson noise of a slot streamed into the wave's LDS ring by
// LDS-DMA (global_load_lds_dword: no VGPR held while in flight), kTsDmaAhead items ahead of
// the one being scored; the first items issued before the slot's exact true-CTR search. The
// loads are inline asm, outside the compiler's s_waitcnt bookkeeping: every wait is our own
// vmcnt(N), N = the DMA instructions issued after the item's (the compiler's own vector memory
// operations are made to complete before the first issue, so none sits between).
constexpr int kTsDmaAhead = AG_TS_DMA_AHEAD;
constexpr int kTsDmaBufs = kTsDmaAhead + 1;
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// the 5 noise rows of one item (the lane's element of row c at src + 64 c floats) into the LDS
// rows at lds + 256 c bytes (lds wave-uniform); the ring buffer it overwrites was read by the
// item before (lgkmcnt(0): those reads done)
__device__ __forceinline__ void ts_dma_item5(const float *src, uint32_t lds_any) {
  const uint32_t lds = (uint32_t)__builtin_amdgcn_readfirstlane((int)lds_any);
  uint32_t keep;
  asm volatile(
      "s_waitcnt lgkmcnt(0)\n\t"
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %6\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\t"
      "s_mov_b32 m0, %7\n\ts_nop 0\n\tglobal_load_lds_dword %2, off\n\t"
      "s_mov_b32 m0, %8\n\ts_nop 0\n\tglobal_load_lds_dword %3, off\n\t"
      "s_mov_b32 m0, %9\n\ts_nop 0\n\tglobal_load_lds_dword %4, off\n\t"
      "s_mov_b32 m0, %10\n\ts_nop 0\n\tglobal_load_lds_dword %5, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "v"(src + 64), "v"(src + 128), "v"(src + 192), "v"(src + 256), "s"(lds), "s"(lds + 256u),
        "s"(lds + 512u), "s"(lds + 768u), "s"(lds + 1024u)
      : "memory");
}

// One auction resolved (src/Auction.py:28-74 minus the draws).
template <int P>
struct Resolved {
  int ag[P], item[P];
  double val[P], bid[P], ctr[P], est[P], bev[P], gamma[P], prop[P];
  int w, oc;
  double price, second;
};

// torch's float32 exp on the CPU as torch.sigmoid's vectorised path computes it (SLEEF's
// expf_u10; oracle/ag_oracle_dr.c torch_expf bit for bit): q = round(x / ln 2), the reduced
// argument in two fused steps, a degree-5 fused Horner polynomial, times 2^q in two steps.
__device__ __forceinline__ float torch_expf(float d) {
  const float q = __builtin_rintf(d * 1.442695040888963407359924681001892137426645954152985934135449406931f);
  float s = __builtin_fmaf(q, -0.693145751953125f, d);
  s = __builtin_fmaf(q, -1.428606765330187045e-06f, s);
  float u = 0.000198527617612853646278381f;
  u = __builtin_fmaf(u, s, 0.00139304355252534151077271f);
  u = __builtin_fmaf(u, s, 0.00833336077630519866943359f);
  u = __builtin_fmaf(u, s, 0.0416664853692054748535156f);
  u = __builtin_fmaf(u, s, 0.166666671633720397949219f);
  u = __builtin_fmaf(u, s, 0.5f);
  u = 1.0f + __builtin_fmaf(s * s, u, s);
  const int e = (int)q, e1 = e >> 1;
  u = u * __builtin_ldexpf(1.0f, e1) * __builtin_ldexpf(1.0f, e - e1);
  if (d < -104.0f) u = 0.0f;
  if (d > 100.0f) u = INFINITY;
  return u;
}

// PyTorchLogisticRegression forward (src/Models.py:28-33) as torch runs it on the CPU for one
// context, oracle/ag_oracle.c ora_ts_logit / ora_ts_sigmoid bit for bit: F.linear(x[Do],
// W[K][Do]) is one MKL sgemv -- for Do = 5 (every shipped config) rows in whole blocks of 4
// sum (fma(w1, x1, w0 x0) + w3 x3) + (w4 x4 + w2 x2), the K % 4 remainder rows
// w0 x0 + ((w4 x4 + w2 x2) + (w3 x3 + w1 x1)); other Do in order -- then torch.sigmoid:
// elements of whole 32-lane chunks 1 / (1 + torch_expf(-z)), the rest its scalar path
// 1 / (1 + expf(-z)) with glibc's expf (agexp::expf_glibc). W = m (+ noise) in float32.
__device__ __forceinline__ float ts_logit_w(const float *wd, const float *x, int Do, int k, int K) {
  if (Do == 5) {
    const float p0 = wd[0] * x[0], p2 = wd[2] * x[2], p3 = wd[3] * x[3], p4 = wd[4] * x[4];
    if (k < (K & ~3)) return (__builtin_fmaf(wd[1], x[1], p0) + p3) + (p4 + p2);
    const float p1 = wd[1] * x[1];
    return p0 + ((p4 + p2) + (p3 + p1));
  }
  float z = wd[0] * x[0];
  for (int d = 1; d < Do; ++d) z = z + wd[d] * x[d];
  return z;
}
__device__ __forceinline__ float ts_ctr_of(float z, int k, int K, const uint64_t *tab) {
  const float e = k < (K & ~31) ? torch_expf(-z) : agexp::expf_glibc(-z, tab + 256);
  return 1.0f / (1.0f + e);
}
// K < 32: every element on the scalar path. `tab`: the kExpTabLds-entry LDS table.
__device__ __forceinline__ float ts_ctr_scalar(float z, const uint64_t *tab) {
  return 1.0f / (1.0f + agexp::expf_glibc(-z, tab + 256));
}
__device__ __forceinline__ float ts_ctr(const float *w, const float *x, int Do, const float *nz, uint32_t nz_stride,
                                        int k, int K, const uint64_t *tab) {
  float wd[AG_LRTS_MAX_DO];
  for (int d = 0; d < Do; ++d) wd[d] = nz ? w[d] + nz[(uint32_t)d * nz_stride] : w[d];
  return ts_ctr_of(ts_logit_w(wd, x, Do, k, K), k, K, tab);
}

// the same logit over a compile-time register width DW >= Do (the runtime model width).
// nzv: the coefficients' noise, already in registers (noisy = false: the MAP CTR).
template <int DW>
__device__ __forceinline__ float ts_logit(const float *w, const float (&x)[DW], const float (&nzv)[DW], bool noisy,
                                          int Do, int k, int K) {
  float wd[DW];
#pragma unroll
  for (int d = 0; d < DW; ++d) wd[d] = d < Do ? (noisy ? w[d] + nzv[d] : w[d]) : 0.0f;
  float z = 0.0f;
#pragma unroll
  for (int d = 0; d < DW; ++d) {
    if (d < Do) {
      const float t = wd[d] * x[d];
      z = d == 0 ? t : z + t;
    }
  }
  if constexpr (DW >= 5) {  // Do = 5: the sgemv kernel's order (branch-free: selects)
    const float p0 = wd[0] * x[0], p1 = wd[1] * x[1], p2 = wd[2] * x[2], p3 = wd[3] * x[3], p4 = wd[4] * x[4];
    const float blk = (__builtin_fmaf(wd[1], x[1], p0) + p3) + (p4 + p2);
    const float rem = p0 + ((p4 + p2) + (p3 + p1));
    z = Do == 5 ? (k < (K & ~3) ? blk : rem) : z;
  }
  return z;
}
template <int DW>
__device__ __forceinline__ float ts_ctr_k(const float *w, const float (&x)[DW], const float (&nzv)[DW],
                                          bool noisy, int Do, int k, int K, const uint64_t *tab) {
  return ts_ctr_of(ts_logit<DW>(w, x, nzv, noisy, Do, k, K), k, K, tab);
}

// Thompson-sampling item choice of an LR-TS agent (src/Agent.py:29-42): first argmax of
// sampled CTR * value. The noise of kTsGroup items is loaded together (one memory latency
// per group instead of one per item), then the group is scored.
//
// Screened (K <= kTsScreenK): every item's logit is exact (float32, ts_logit's), its score
// first estimated with the hardware exp2 / reciprocal -- relative error < 2^-16 for |z| <
// 64 and value > 0 (argument rounding |z| log2 e 2^-23 <= 2^-16.5, v_exp_f32 / v_rcp_f32
// 1 ulp each, float value and product 2^-24 each) -- then only the items within 2^-13 of
// the best estimate (and any item outside those bounds) are scored exactly, in increasing
// k: the exact first argmax is always among them (its estimate is >= best * (1 - 2^-15)),
// so the choice is the plain loop's bit for bit.
#ifndef AG_TS_GROUP
#define AG_TS_GROUP 4  // items whose noise is loaded together (divides kTsScreenK)
#endif
constexpr int kTsGroup = AG_TS_GROUP;
constexpr int kTsScreenK = 12;
constexpr int kShipDo = 5;   // the shipped configs' LR-TS model width (OE = 4)
constexpr int kGenShip = 8;  // pick_kernel_for: OR-ed into `general` for that width (D = 6)
constexpr int kGenGen = 16;  // pick_kernel_for: OR-ed into `general` for the generate-mode build
// the noise of items k0 .. k0 + kTsGroup - 1 (coefficient stride 64: the tile layout). (Tried:
// non-temporal loads of the dense layout, and loading the first group before the true-CTR
// search: no gain / scratch spills, profiles/r05m_ab_pre.log, r05n_ab_nt.log.)
template <int DW>
__device__ __forceinline__ void ts_load_group(const TsSrc &src, int k0, int K, int Do, float (&nzv)[kTsGroup][DW]) {
  if constexpr ((AG_ABLATE & 64) != 0) {  // ablation: the noise not read (a lane-dependent constant)
#pragma unroll
    for (int g = 0; g < kTsGroup; ++g)
#pragma unroll
      for (int d = 0; d < DW; ++d) nzv[g][d] = src.nz ? 1e-3f * (float)((threadIdx.x + g * 7 + d) & 15) : 0.0f;
    return;
  }
  const float *nz = src.nz;
#pragma unroll
  for (int g = 0; g < kTsGroup; ++g)
#pragma unroll
    for (int d = 0; d < DW; ++d)
      nzv[g][d] = (nz && k0 + g < K && d < Do) ? nz[(size_t)((k0 + g) * Do + d) * 64] : 0.0f;
}
// Generate mode (compile-time model width DOS): the noise of item k0 + g, drawn as
// ag_generate_noise draws it -- coefficient c = k Do + d is normal c % 4 of Philox block c / 4
// (ag_philox.h gen_normals4) times the coefficient's 1 / sqrtf(q). A group's kTsGroup items are
// kTsGroup DOS / 4 whole blocks (k0 % 4 == 0); the items are drawn in order (g compile-time
// after unrolling), each block when its first coefficient comes, the block's normals carried
// in z4 -- at most 4 + DOS noise values live instead of a group's kTsGroup DOS.
template <int DW, int DOS>
__device__ __forceinline__ void ts_gen_item(const TsSrc &src, int k0, int g, float (&z4)[4], float (&nzg)[DW]) {
  static_assert(DOS > 0 && DOS <= DW && kTsGroup % 4 == 0, "generate mode: compile-time width, whole blocks");
#pragma unroll
  for (int d = 0; d < DW; ++d) nzg[d] = 0.0f;
  if (!src.rsq) return;
  const uint32_t b0 = (uint32_t)(k0 * DOS) >> 2;
#pragma unroll
  for (int d = 0; d < DOS; ++d) {
    const int c = g * DOS + d;
    if ((c & 3) == 0)
      gen_normals4(src.key.c0, src.key.c1, b0 + (uint32_t)(c >> 2), src.stream, src.key.k0, src.key.k1, z4);
    nzg[d] = z4[c & 3] * src.rsq[(k0 + g) * DOS + d];
  }
}
template <int DW, bool GEN = false, int DOS = 0>
__device__ __forceinline__ int ts_select(const float *m, const float (&xo)[DW], const TsSrc &src, int K, int Do,
                                         const double *vals, const uint64_t *tab) {
  const bool noisy = GEN ? src.rsq != nullptr : src.nz != nullptr;
  if (AG_TS_SCREEN && K <= kTsScreenK) {
    float zk[kTsScreenK], ek[kTsScreenK];  // logits; score estimates (-1: score exactly)
    float best_est = 0.0f;
    if (AG_TS_DMA && !GEN && DOS == 5 && src.ring) {
      // the noise from the wave's LDS ring: items 0 .. kTsDmaAhead - 1 were issued before the
      // slot's true-CTR search; item k issues item k + kTsDmaAhead, then waits for its own.
      // The batch's K is kTsScreenK (resolve_slot's condition), whatever the lane's own count:
      // the schedule and every vmcnt are compile-time constants
      constexpr int KG = kTsScreenK;
      const int lane = (int)(threadIdx.x & 63);
#pragma unroll
      for (int k = 0; k < KG; ++k) {
        zk[k] = 0.0f;
        ek[k] = -1.0f;
        {
          if (k + kTsDmaAhead < KG)
            ts_dma_item5(src.nz + (size_t)(k + kTsDmaAhead) * 5 * 64,
                         src.ring_lds + (uint32_t)(((k + kTsDmaAhead) % kTsDmaBufs) * 5 * 256));
          constexpr int kLast = KG - 1;
          const int later = (k + kTsDmaAhead < kLast ? k + kTsDmaAhead : kLast) - k;  // items issued after k
          static_assert(kTsDmaAhead <= 8, "vmcnt counts up to 63: at most 8 items of 5 DMAs ahead");
          switch (later) {  // a constant after unrolling
            case 1: wait_vm<5>(); break;
            case 2: wait_vm<10>(); break;
            case 3: wait_vm<15>(); break;
            case 4: wait_vm<20>(); break;
            case 5: wait_vm<25>(); break;
            case 6: wait_vm<30>(); break;
            case 7: wait_vm<35>(); break;
            case 8: wait_vm<40>(); break;
            default: wait_vm<0>(); break;
          }
          const float *row = src.ring + (k % kTsDmaBufs) * 5 * 64 + lane;
          float nzg[DW];
#pragma unroll
          for (int d = 0; d < DW; ++d) nzg[d] = d < 5 ? row[d * 64] : 0.0f;
          if (k < K) {
            const float z = ts_logit<DW>(m + k * Do, xo, nzg, noisy, Do, k, K);
            const float v = (float)vals[k];
            const bool ok = __builtin_fabsf(z) < 64.0f && v > 0.0f;
            const float e = __builtin_amdgcn_exp2f(-z * 1.44269504f);
            const float est = ok ? __builtin_amdgcn_rcpf(1.0f + e) * v : -1.0f;
            zk[k] = z;
            ek[k] = est;
            best_est = est > best_est ? est : best_est;
          }
        }
      }
    } else
#pragma unroll
    for (int k0 = 0; k0 < kTsScreenK; k0 += kTsGroup) {
      if (k0 < K) {
        float nzv[GEN ? 1 : kTsGroup][DW], z4[4];
        if constexpr (!GEN) ts_load_group<DW>(src, k0, K, Do, nzv);
#pragma unroll
        for (int g = 0; g < kTsGroup; ++g) {
          const int k = k0 + g;
          zk[k] = 0.0f;
          ek[k] = -1.0f;
          if (k < K) {
            if constexpr (GEN) ts_gen_item<DW, DOS>(src, k0, g, z4, nzv[0]);
            const float z = ts_logit<DW>(m + k * Do, xo, nzv[GEN ? 0 : g], noisy, Do, k, K);
            const float v = (float)vals[k];
            const bool ok = __builtin_fabsf(z) < 64.0f && v > 0.0f;
            const float e = __builtin_amdgcn_exp2f(-z * 1.44269504f);
            const float est = ok ? __builtin_amdgcn_rcpf(1.0f + e) * v : -1.0f;
            zk[k] = z;
            ek[k] = est;
            best_est = est > best_est ? est : best_est;
          }
        }
      } else {
#pragma unroll
        for (int g = 0; g < kTsGroup; ++g) {
          zk[k0 + g] = 0.0f;
          ek[k0 + g] = -1.0f;
        }
      }
    }
    const float thr = best_est * (1.0f - 0x1p-13f);
    uint32_t cand = 0;
#pragma unroll
    for (int k = 0; k < kTsScreenK; ++k)
      if (k < K && (ek[k] < 0.0f || ek[k] >= thr)) cand |= 1u << k;
    // exact scores of the candidates in increasing k (one exp in the code: a loop over the
    // mask, the logit picked out of the register row by selects)
    double best_sc = 0.0;
    int best = -1;
    while (cand) {
      const int k = __builtin_ctz(cand);
      cand &= cand - 1;
      float z = zk[0];
#pragma unroll
      for (int kk = 1; kk < kTsScreenK; ++kk) z = k == kk ? zk[kk] : z;
      const double sc = (double)ts_ctr_scalar(z, tab) * vals[k];  // K <= kTsScreenK < 32
      if (best < 0 || sc > best_sc) {
        best_sc = sc;
        best = k;
      }
    }
    return best;
  }
  double best_sc = 0.0;
  int best = 0;
  for (int k0 = 0; k0 < K; k0 += kTsGroup) {
    float nzv[GEN ? 1 : kTsGroup][DW], z4[4];
    if constexpr (!GEN) ts_load_group<DW>(src, k0, K, Do, nzv);
#pragma unroll
    for (int g = 0; g < kTsGroup; ++g) {
      const int k = k0 + g;
      if (k < K) {
        if constexpr (GEN) ts_gen_item<DW, DOS>(src, k0, g, z4, nzv[0]);
        const float ck = ts_ctr_k<DW>(m + k * Do, xo, nzv[GEN ? 0 : g], noisy, Do, k, K, tab);
        const double sc = (double)ck * vals[k];
        if (k == 0 || sc > best_sc) {
          best_sc = sc;
          best = k;
        }
      }
    }
  }
  return best;
}

// A learning bidder's bid from its fitted policy (src/Bidder.py:198-203 ValueLearningBidder
// 'policy', :358-362 PolicyLearningBidder, :466-470 DoublyRobustBidder; src/Models.py:82-90
// and :155-164 -- the same forward):
// ora_policy_bid (oracle/ag_oracle_dr.c) bit for bit -- the policy forward in double
// (softplus = log1p(exp), the restated log1p), mu / sigma rounded to float32, the rsample
// mu + sigma * eps in float32, exp(log_prob) rounded to float32, gamma = clip(sample, 0, 1).
__device__ __forceinline__ double policy_softplus(double u, const uint64_t *tab) {
  const double e = agexp::exp_fast(u, tab);
  bool lok;
  const double l = aglog1p::log1p_main(e, lok);
  return u > 20.0 ? u : (__builtin_expect(lok, 1) ? l : aglog1p::log1p(e));
}
__device__ __forceinline__ void policy_bid(const float *p, double ctr, double value, float eps,
                                           const uint64_t *tab, double &gamma, double &prop) {
  const double c = (double)(float)ctr, v = (double)(float)value;
  double sft[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
    sft[j] = policy_softplus(c * (double)p[2 * j] + v * (double)p[2 * j + 1] + (double)p[4 + j], tab);
  const double am = sft[0] * (double)p[6] + sft[1] * (double)p[7] + (double)p[8];
  const double as = sft[0] * (double)p[9] + sft[1] * (double)p[10] + (double)p[11];
  const float mu = (float)policy_softplus(am, tab), sg = (float)(policy_softplus(as, tab) + 0.01);
  const float raw = mu + sg * eps;
  const double z = ((double)raw - (double)mu) / (double)sg;
  const double logp = -(z * z) / 2.0 - aglog1p::log1p((double)sg - 1.0) - 0.91893853320467274178;
  prop = (double)(float)agexp::exp_fast(logp, tab);
  gamma = raw < 0.0f ? 0.0 : (raw > 1.0f ? 1.0 : (double)raw);
}

// ValueLearningBidder 'search' bid (src/Bidder.py:180-196): the shading factor maximising
// the win-rate model's predicted utility W(ctr, value, g) (ev - ev g), ev = value * ctr,
// over the agent's 128 grid draws (dev [128] with stride B). W in float32 as torch runs the
// reference's model on the CPU: Linear(3, 1) summed as its BLAS kernel does,
// z = (fma(v, w1, c w0) + g w2) + b, then torch.sigmoid's vectorised 1 / (1 + exp(-z))
// (torch_expf). The first maximum in sorted-grid order = the smallest gamma among tied
// maxima, so the grid may arrive unsorted. oracle/ag_oracle_dr.c ora_search_gamma is this,
// bit for bit; it picks the reference's gamma in all 24000 bids of search_bid_kat.npz.
__device__ __forceinline__ double search_gamma(const float *wr, double ctr, double value, const double *grid,
                                               uint32_t stride, const uint64_t *tab) {
  (void)tab;
  const float c = (float)ctr, v = (float)value;
  const float cv = __builtin_fmaf(v, wr[1], c * wr[0]);
  const double ev = value * ctr;
  double best_u = -INFINITY, best_g = 0.0;
  for (int j = 0; j < 128; ++j) {
    const double g = grid[(size_t)j * stride];
    const float z = (cv + (float)g * wr[2]) + wr[3];
    const float pw = 1.0f / (1.0f + torch_expf(-z));
    const double ut = (double)pw * (ev - ev * g);
    if (ut > best_u || (ut == best_u && g < best_g)) {
      best_u = ut;
      best_g = g;
    }
  }
  return best_g;
}

// Gaussian density of a shading factor (src/Bidder.py:178, :355, :462).
__device__ __forceinline__ double shading_propensity(double pg, double sigma, double g,
                                                     const uint64_t *tab) {
  const double t = (pg - g) / sigma;
  return agexp::exp_fast(-(t * t) / 2.0, tab) / (sigma * 2.5066282746310002);  // sqrt(2 pi)
}

// One participant (slot s, agent a) of a round: its item, bid and the values its log
// record and counters need (src/Auction.py:44-53, src/Agent.py:29-68).
constexpr int kTsjLoad = -2;  // resolve_slot: no prefetched ts_noise_index entry

struct SlotResult {
  int item;
  double val, bid, ctr, est, bev, gamma, prop;
  bool pol;  // DEFER: a fitted-policy bid left to the caller (bid = value * est, gamma / prop NaN)
};

// Diagnostic ablations of the general kernel (WRONG results; make variant-p VFLAGS=-DAG_ABLATE=..):
// 1 no fitted-policy forward (gamma 1), 2 no Thompson item choice (the true-CTR leader),
// 4 no exact true-CTR item search (item 0, CTR 0.5), 16 no MAP estimate (0.5), 32 no re-scored
// true CTR of the Thompson choice (the leader's), 64 the Thompson choice computed but its noise not read
#ifndef AG_ABLATE
#define AG_ABLATE 0
#endif
constexpr int kAblate = AG_ABLATE;

// GEN: generate mode -- the slot's draws (Thompson noise, rsample, shading) made here from the
// auction's Philox counter `gk`, the bits ag_generate_noise stores (ag_philox.h); `in` unread.
template <int D, bool PRUNE, int GENERAL, bool DEFER = false, bool GEN = false, int DOS = 0>
__device__ __forceinline__ SlotResult resolve_slot(const Lds &T, int K, const double (&x)[kMaxD],
                                                   const float (&xf)[kMaxD], float xabs, int a, int s,
                                                   const ag_batch_in &in, uint32_t B, uint32_t i, bool ts_sample,
                                                   int tsj = kTsjLoad, GenKey gk = GenKey{0, 0, 0, 0}) {
  // true CTRs (src/Auction.py:52-53): exact search on the true context; for an Oracle
  // agent this IS Agent.select_item (src/BidderAllocation.py:81-82)
  double c = 0.5, bs = 0.5;
  const double *itm = T.items + a * T.items_stride;
  const bool lrts = GENERAL && T.akind[a] == AG_ALLOCATOR_LRTS;
  // LR-TS: where the slot's Thompson noise comes from (tiled noise: coefficient c of auction i
  // at ((s*T + i/64)*K*Do + c)*64 + i%64; the compact layout tiles the batch's LR-TS pairs
  // only, pair j = ts_noise_index[s*B + i] in place of s*T*64 + i -- mixed populations: no
  // noise stored or fetched for the slots of other agents)
  TsSrc nz{nullptr, nullptr, gk, 4u + (uint32_t)s};
  if constexpr (GENERAL) {
    const int Do = DOS > 0 ? DOS : T.ts_do;
    if constexpr (GEN) {
      if (lrts && ts_sample) nz.rsq = T.tsr + (size_t)a * T.tsm_stride;
    } else if (lrts && ts_sample && in.ts_noise) {
      if (in.ts_noise_index) {
        // prefetched with the tile's inputs (tsj), or loaded here
        const uint32_t j = (uint32_t)(tsj != kTsjLoad ? tsj : ldg(in.ts_noise_index + (size_t)s * B + i));
        nz.nz = in.ts_noise + ((size_t)(j >> 6) * K * Do) * 64 + (j & 63);
      } else {
        nz.nz = in.ts_noise + ((size_t)(s * ((B + 63) >> 6) + (i >> 6)) * K * Do) * 64 + (i & 63);
      }
      if (AG_TS_DMA && DOS == 5 && T.ring && K == kTsScreenK) {
        // the first kTsDmaAhead items' rows into the wave's ring now: they land while the exact
        // true-CTR search below runs (k_simulate has made the compiler wait for all of the
        // tile's own loads already, so no compiler-counted load sits behind these DMAs)
        nz.ring = T.ring;
        nz.ring_lds = T.ring_lds;
        nz.kg = kTsScreenK;
#pragma unroll
        for (int k = 0; k < kTsDmaAhead; ++k) ts_dma_item5(nz.nz + (size_t)k * 5 * 64, T.ring_lds + (uint32_t)(k * 5 * 256));
      }
    }
  }
  const int best_t = (kAblate & 4) ? 0
                                   : select_item<D, PRUNE>(itm, T.vals + a * T.values_stride,
                                                           T.scr + a * T.scr_stride, T.scr_val + a * T.scr_val_stride,
                                                           PRUNE ? T.amax[a] : 0.0f, K, T.kpairs, x, xf, xabs, T.tab,
                                                           c, bs);
  int best = best_t;
  double est = c, tru = c;
  double g = NAN, prop = NAN;
  if constexpr (GENERAL) {
    if (lrts) {
      // LR-TS (src/Agent.py:29-42): the sampled CTRs on the observed context pick the
      // item by first argmax of CTR * value (float32 CTR widened to double), the MAP CTR
      // of that item is the estimate
      const int Do = DOS > 0 ? DOS : T.ts_do;
      const float *m = T.tsm + (size_t)a * T.tsm_stride;
      // observed context (src/Auction.py:36) in a register row of width D >= Do
      float xo[D];
#pragma unroll
      for (int d = 0; d < D; ++d) xo[d] = d < Do - 1 ? (float)x[d] : (d == Do - 1 ? 1.0f : 0.0f);
      // the agent's own Ka items: its torch model's rows (the sgemv block / remainder rows and
      // the sigmoid's chunks follow Ka); the catalogue rows beyond are padding (value 0)
      // (per-agent Ka even when every agent has K: the uniform-K form, scalar item loops, ran
      // 2-4 % slower on every population line, profiles/r04s_ab_c*_kag.log)
      const int Ka = T.kag[a];
      best = (kAblate & 2) ? best_t
                           : ts_select<D, GEN, DOS>(m, xo, nz, Ka, Do, T.vals + a * T.values_stride, T.tab);
      est = (kAblate & 16) ? 0.5 : (double)ts_ctr_k<D>(m + best * Do, xo, xo, false, Do, best, Ka, T.tab);
      tru = (best == best_t || (kAblate & 32)) ? c : agexp::sigmoid_fast(dot_ref<D>(itm + best * D, x), T.tab);
    }
  }
  const double v = T.vals[a * T.values_stride + best];
  double b = v * est;  // Bidder.bid: value * estimated CTR (src/Bidder.py:35, :49, :173, ...)
  bool pol = false;
  if constexpr (GENERAL == kGenAll) {  // kGenTruthful: every bidder is a TruthfulBidder
    const int bk = T.bkind[a];
    if (bk >= AG_BIDDER_VALUE_LEARNING && T.drs && T.dri[a] == AG_LEARNER_POLICY) {  // the fitted policy
      if constexpr (DEFER) {
        pol = true;
      } else if constexpr (kAblate & 1) {
        g = 1.0;
        prop = 1.0;
      } else {
        const float eps = GEN ? gen_normal1(gk.c0, gk.c1, 0, 16u + (uint32_t)s, gk.k0, gk.k1)
                              : in.policy_eps[(size_t)s * B + i];
        policy_bid(T.drs + a * T.drs_stride + 4, est, v, eps, T.tab, g, prop);
        b = b * g;
      }
    } else if (!GEN && bk == AG_BIDDER_VALUE_LEARNING && T.drs && T.dri[a] == AG_LEARNER_SEARCH) {
      // (generate mode has no search grids: the host refuses such populations)
      g = search_gamma(T.drs + a * T.drs_stride, est, v, in.gamma_grid + (size_t)s * 128 * B + i, B, T.tab);
      prop = 1.0;  // src/Bidder.py:196
      b = b * g;
    } else if (bk != AG_BIDDER_TRUTHFUL) {
      g = GEN ? gen_shading_raw(gk.c0, gk.c1, s, gk.k0, gk.k1, T.pg[a], T.gs[a]) : in.gamma_raw[(size_t)s * B + i];
      if (bk == AG_BIDDER_EMPIRICAL_SHADED) {  // clipped to [0, 1] (src/Bidder.py:52-55)
        if (g < 0.0) g = 0.0;
        if (g > 1.0) g = 1.0;
      } else {
        prop = shading_propensity(T.pg[a], T.gs[a], g, T.tab);
      }
      b = b * g;  // bid *= gamma
    }
  }
  return SlotResult{best, v, b, tru, est, bs, g, prop, pol};  // bev: max_k true_CTR_k * value_k (src/Auction.py:53)
}

// streaming top-2 of the bids in slot order, ties -> lowest slot (src/AuctionAllocation.py:19-34)
__device__ __forceinline__ void top2_step(int s, double b, double &m1, double &m2, int &w) {
  if (s == 0) {
    m1 = b;
  } else if (b > m1) {
    m2 = m1;
    m1 = b;
    w = s;
  } else if (b > m2) {
    m2 = b;
  }
}

template <int P, int D, bool PRUNE, int GENERAL, bool GEN = false, int DOS = 0>
__device__ __forceinline__ void resolve(const Lds &T, int K, int mech, const double (&x)[kMaxD],
                                        const float (&xf)[kMaxD], float xabs, const int (&ag)[P], double u,
                                        const ag_batch_in &in, uint32_t B, uint32_t i, bool ts_sample,
                                        const int (&tsj)[P], Resolved<P> &r, GenKey gk) {
  double m1 = 0.0, m2 = -INFINITY;
  int w = 0;
#pragma unroll
  for (int s = 0; s < P; ++s) {
    const int a = ag[s];
    r.ag[s] = a;
    const SlotResult q =
        resolve_slot<D, PRUNE, GENERAL, false, GEN, DOS>(T, K, x, xf, xabs, a, s, in, B, i, ts_sample, tsj[s], gk);
    r.item[s] = q.item;
    r.val[s] = q.val;
    r.bid[s] = q.bid;
    r.ctr[s] = q.ctr;
    r.est[s] = q.est;
    r.bev[s] = q.bev;
    r.gamma[s] = q.gamma;
    r.prop[s] = q.prop;
    top2_step(s, q.bid, m1, m2, w);
  }
  r.w = w;
  r.price = mech == AG_FIRST_PRICE ? m1 : m2;
  r.second = m2;
  double ctr_w = r.ctr[0];
#pragma unroll
  for (int s = 1; s < P; ++s)
    if (s == w) ctr_w = r.ctr[s];
  r.oc = bernoulli(ctr_w, u);  // src/Auction.py:65 (true CTR of the winner's item)
}

// DOS: 0, or the LR-TS model width Do = OE + 1 as a compile-time constant (the host picks
// DOS = 5, the shipped configs' OE = 4, when the layout's ts_do is 5): the width masks of the
// observed-context row, the generic-width logit chain and the sgemv order's Do == 5 test fold
// away, and fewer values stay live (P = 2, 256 lanes, TruthfulBidders: 128 -> 115 VGPRs,
// 441 -> 155 SGPRs spilled to VGPR lanes; the full build at 1024 lanes: 112 -> 52 B of
// scratch per lane). K stays a runtime value: with it compile-time the item loops unroll
// fully and spill (200 VGPRs at P = 2), measured.
// GEN: generate mode (ag_simulate_generated) -- every input drawn in the kernel from the
// auction's global index, the bits ag_generate + ag_generate_noise store (contexts,
// participants, uniform: gen_auction; Thompson noise, rsample and shading draws: resolve_slot);
// only the outputs touch HBM. Shipped-shape builds (DOS > 0) only.
template <int P, int D, bool PRUNE, int W, int GENERAL, int BT = kThreads, int DOS = 0, bool GEN = false>
__global__ __launch_bounds__(BT, GENERAL == kGenTruthful ? (P >= 3 ? AG_TB_WIDE_MIN_WAVES : AG_TB_MIN_WAVES)
                                 : (GENERAL ? ((DOS && P > 0 && P <= 2) ? AG_GEN_DOS_MIN_WAVES : AG_GEN_MIN_WAVES)
                                            : AG_MIN_WAVES)) void k_simulate(SimParams prm) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int N = prm.N, K = prm.K;
  const uint32_t B = (uint32_t)prm.B;  // SoA leading dimension (auctions in the batch)
  const uint32_t lo = (uint32_t)prm.lo, hi = (uint32_t)prm.hi;  // this launch's auctions
  LdsLayout L = prm.lds;
  if constexpr (DOS > 0) L.ts_do = DOS;
  uint64_t *s_tab = reinterpret_cast<uint64_t *>(smem + L.tab);
  double *s_items = reinterpret_cast<double *>(smem + L.items);
  double *s_vals = reinterpret_cast<double *>(smem + L.values);
  float *s_scr = reinterpret_cast<float *>(smem + L.scr);
  float *s_scr_val = reinterpret_cast<float *>(smem + L.scr_val);
  float *s_amax = reinterpret_cast<float *>(smem + L.amax);
  int32_t *s_akind = reinterpret_cast<int32_t *>(smem + L.akind);
  int32_t *s_bkind = reinterpret_cast<int32_t *>(smem + L.bkind);
  double *s_pg = reinterpret_cast<double *>(smem + L.pg);
  double *s_gs = reinterpret_cast<double *>(smem + L.gs);
  float *s_tsm = reinterpret_cast<float *>(smem + L.tsm);
  float *s_drs = reinterpret_cast<float *>(smem + L.drs);
  int32_t *s_dri = reinterpret_cast<int32_t *>(smem + L.dri);
  int32_t *s_kag = reinterpret_cast<int32_t *>(smem + L.kag);
  float *s_tsr = reinterpret_cast<float *>(smem + L.tsr);
  // AG_TS_DMA: every wave's Thompson-noise ring (kTsDmaBufs items of 5 rows x 64 floats)
  constexpr bool kDma = AG_TS_DMA && GENERAL && DOS == 5 && !GEN && BT == kThreads && P >= 1 && P <= AG_TS_DMA_MAXP;
  __shared__ __attribute__((aligned(16))) float s_ring[kDma ? (BT / 64) * kTsDmaBufs * 5 * 64 : 1];
  static_assert(!GEN || (DOS > 0 && P > 0 && W == 1 && GENERAL), "generate mode: shipped-shape general builds");
  unsigned long long *s_cnt = reinterpret_cast<unsigned long long *>(smem + L.cnt);

  const int tid = threadIdx.x;
  if constexpr (GENERAL) {
    for (int a = tid; a < N; a += BT) {
      s_akind[a] = prm.akind[a];
      s_bkind[a] = prm.bkind[a];
      s_pg[a] = prm.pg[a];
      s_gs[a] = prm.gs[a];
      s_kag[a] = prm.kag ? prm.kag[a] : K;
    }
    for (int j = tid; j < N * K * L.ts_do; j += BT) {
      const int a = j / (K * L.ts_do);
      s_tsm[a * L.tsm_stride + (j - a * K * L.ts_do)] = prm.tsm[j];
      // generate mode: the noise scale as k_generate_noise computes it
      if constexpr (GEN) s_tsr[a * L.tsm_stride + (j - a * K * L.ts_do)] = 1.0f / sqrtf(prm.tsq[j]);
    }
    if (prm.drs) {
      for (int j = tid; j < N * 16; j += BT) s_drs[(j >> 4) * L.drs_stride + (j & 15)] = prm.drs[j];
      for (int a = tid; a < N; a += BT) s_dri[a] = prm.dri[a];
    }
  }
  for (int i = tid; i < 256; i += BT) s_tab[i] = ag_exp_tab[i];
  for (int j = tid; j < 32; j += BT) s_tab[256 + j] = agexp::expf_tab_entry(ag_exp_tab, j);
  for (int i = tid; i < N * K * D; i += BT) {
    const int a = i / (K * D), r = i - a * (K * D);
    s_items[a * L.items_stride + r] = prm.items[i];
  }
  for (int i = tid; i < N * K; i += BT) {
    const int a = i / K, r = i - a * K;
    s_vals[a * L.values_stride + r] = prm.values[i];
  }
  if (PRUNE) {
    // screening rows: [pair p][dim d][item 2p, 2p+1], coefficients * -log2(e); padded
    // dims and the odd item's partner are 0
    for (int i = tid; i < N * L.kpairs * 16; i += BT) {
      const int a = i / (L.kpairs * 16), r = i - a * (L.kpairs * 16);
      const int p = r >> 4, d = (r >> 1) & 7, k = 2 * p + (r & 1);
      const float c = (d < D && k < K) ? (float)prm.items[((size_t)a * K + k) * D + d] : 0.0f;
      s_scr[a * L.scr_stride + r] = c * kNegLog2e;
    }
    for (int i = tid; i < N * L.kpairs * 2; i += BT) {  // 1/v (padding items: +inf)
      const int a = i / (L.kpairs * 2), k = i - a * (L.kpairs * 2);
      s_scr_val[a * L.scr_val_stride + k] = k < K ? 1.0f / (float)prm.values[(size_t)a * K + k] : INFINITY;
    }
    for (int a = tid; a < N; a += BT) {
      float m = 0.0f;
      for (int r = 0; r < K * D; ++r) m = fmaxf(m, (float)fabs(prm.items[(size_t)a * K * D + r]));
      s_amax[a] = m * 1.001f;
    }
  }
  const int R = L.replicas;
  if (prm.want_counters)
    for (int i = tid; i < R * N * L.ncnt; i += BT) s_cnt[i] = 0ull;
  __syncthreads();

  Lds T{s_tab, s_items, s_vals, s_scr, s_scr_val, s_amax, L.items_stride, L.values_stride,
              L.scr_stride, L.scr_val_stride, L.kpairs, s_akind, s_bkind, s_pg, s_gs, s_tsm, L.ts_do,
              L.tsm_stride, L.drs_stride, (GENERAL && prm.drs) ? s_drs : nullptr, s_dri,
              GENERAL ? s_kag : nullptr, GEN ? s_tsr : nullptr, nullptr, 0u};
  if constexpr (kDma) {
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    T.ring = s_ring + wv * kTsDmaBufs * 5 * 64;
    T.ring_lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float *)s_ring +
                 (uint32_t)(wv * kTsDmaBufs * 5 * 256);
    T.ring_lds = (uint32_t)__builtin_amdgcn_readfirstlane((int)T.ring_lds);
  }
  const int rep = tid & (R - 1);
  const ag_batch_in in = prm.in;
  const ag_batch_out out = prm.out;
  // P == 0: the runtime-P kernel (more than kMaxP participants; slot results are not kept
  // in registers -- see the wide path in the loop)
  constexpr int PA = P > 0 ? P : 1;  // register array extent
  static_assert(P > 0 || !AG_PREFETCH, "the runtime-P path has no software-pipelined loads");
  const bool charged = P == 0 ? prm.P >= 2 : P >= 2;  // P == 1: nobody charged (Auction.py:68)

  // inputs of one tile: the context, participants and uniform of W consecutive auctions
  double xv[kMaxD][W];
  int pv[PA][W];
  double uv[W];
  int jv[PA][W];  // compact ts_noise_index entries (GENERAL with ts_noise_index; else kTsjLoad)
  const bool pre_tsj = !GEN && GENERAL && !AG_PREFETCH && in.ts_noise_index && in.ts_noise && prm.ts_sample;
  static_assert(!GEN || !AG_PREFETCH, "generate mode has no input loads to pipeline");
  const uint32_t gk0 = (uint32_t)prm.seed, gk1 = (uint32_t)(prm.seed >> 32);
  // generate mode: the tile's inputs drawn (ag_generate's bits) instead of loaded
  auto gen_tile = [&](uint32_t i) {
    double x[kMaxD], u;
    int pk[PA];
    gen_auction<PA, kMaxD>(gk0, gk1, prm.first + i, N, PA, D - 1, prm.scale, x, pk, u);
#pragma unroll
    for (int e = 0; e < D - 1; ++e) xv[e][0] = x[e];
#pragma unroll
    for (int s = 0; s < PA; ++s) {
      pv[s][0] = pk[s];
      jv[s][0] = kTsjLoad;
    }
    uv[0] = u;
  };
  // streamed slots (below): each slot's participant / noise index loaded with the slot
  // streamed slots for TruthfulBidder-only populations (configs_1 at P = 8: 0.665 vs 0.730 ms
  // kept per-slot arrays, profiles/r04k_ab_c1p8.log) and for the full mix in its 768-lane build
  // (kMidThreads)
  constexpr bool kStream =
      (GENERAL == kGenTruthful || (GENERAL == kGenAll && (BT == kMidThreads || AG_STREAM_GENALL))) && W == 1 &&
      P >= AG_STREAM_MIN_P;
  auto load_tile = [&](uint32_t i) {
#pragma unroll
    for (int e = 0; e < D - 1; ++e) ld_f64<W>(in.ctx + e * B + i, xv[e]);
    if constexpr (kStream) {
      ld_f64<W>(in.u + i, uv);
      return;
    }
#pragma unroll
    for (int s = 0; s < P; ++s) ld_i32<W>(in.part + s * B + i, pv[s]);
    ld_f64<W>(in.u + i, uv);
#pragma unroll
    for (int s = 0; s < P; ++s) {
      if (pre_tsj) {
        ld_i32<W>(in.ts_noise_index + s * B + i, jv[s]);
      } else {
#pragma unroll
        for (int q = 0; q < W; ++q) jv[s][q] = kTsjLoad;
      }
    }
  };
  const uint32_t stride = gridDim.x * (BT * W);
  // the workgroup's tile in each grid stride: blockIdx, or with AG_XCD_MAP the workgroups of one
  // XCD (dispatched round-robin over the 8) on consecutive tiles, so the lines two neighbouring
  // tiles share (the compact Thompson noise's runs) meet in one L2
  const uint32_t wg_tile = (AG_XCD_MAP && gridDim.x % 8 == 0) ? (blockIdx.x % 8) * (gridDim.x / 8) + blockIdx.x / 8
                                                               : blockIdx.x;
  // Participation / win counts: a lane resolves at most kAuctionsPerReplica * R / BT
  // (<= 255) auctions per launch, so for N <= 8 agents its counts fit 8-bit fields of one
  // register each; flushed to the LDS counters once, after the loop.
  const bool packed = P > 0 && N <= 8 && kAuctionsPerReplica * R / BT <= 255;
  uint64_t n_logs_packed = 0, n_won_packed = 0;
  // the counter terms of one participant (src/Agent.py:96-118, via the exact LDS replicas)
  auto count_slot = [&](int a, bool won, double lp, double price, double second, double bid, double ctr,
                        double val, double est, double bev, int oc) {
    // [slot j][agent a][replica]: lane-private replicas, conflict-free 8-B atomics
    auto add_raw = [&](int j, unsigned long long v) { atomicAdd(s_cnt + ((size_t)(j * N + a) * R + rep), v); };
    // zero terms are skipped (a wave whose lanes all hold 0 issues no atomic): no clicks
    // for GROSS, and under SecondPrice with P == 2 the loser's underbid term
    // (price - bid) * [...] is exactly 0 because the price is its bid
    auto add_nz = [&](int j, unsigned long long v) {
      if (v != 0ull) add_raw(j, v);
    };
    const double tv = ctr * val;
    if (won) {
      add_nz(kSlotGross, to_fx(val * (double)oc));
      add_raw(kSlotPaid, to_fx(price));
      if (prm.mech == AG_FIRST_PRICE) add_nz(kSlotOverbid, to_fx(lp - second));
    } else {
      add_nz(kSlotUnderbid, to_fx((lp - bid) * (double)(lp < tv)));
    }
    add_raw(kSlotBestEv, to_fx(bev));
    if (packed) {  // 8-bit per-agent fields in registers, flushed once per block
      const uint64_t bit = 1ull << (8 * a);
      n_logs_packed += bit;
      if (won) n_won_packed += bit;
    } else {
      add_raw(kSlotCounts, won ? 0x100000001ull : 1ull);
    }
    if constexpr (GENERAL) {  // src/Agent.py:96-118 terms that vanish for Oracle agents
      add_nz(kSlotAlloc, to_fx(bev - tv));
      add_nz(kSlotEst, to_fx(est * val - tv));
      const double dd = ctr - est;
      add_nz(kSlotSqerr, to_fx(dd * dd));
      if (won) add_raw(kSlotBias, to_fx(est / ctr));
    }
  };
  // count_slot in two parts (the same exact integer terms, added in another order): the
  // terms that do not depend on the auction's winner as soon as a slot is resolved, so the
  // slot's CTRs / best EV need not stay live while the other slots are resolved ...
  auto count_pre = [&](int a, double ctr, double val, double est, double bev) {
    auto add_raw = [&](int j, unsigned long long v) { atomicAdd(s_cnt + ((size_t)(j * N + a) * R + rep), v); };
    auto add_nz = [&](int j, unsigned long long v) {
      if (v != 0ull) add_raw(j, v);
    };
    const double tv = ctr * val;
    add_raw(kSlotBestEv, to_fx(bev));
    add_nz(kSlotAlloc, to_fx(bev - tv));
    add_nz(kSlotEst, to_fx(est * val - tv));
    const double dd = ctr - est;
    add_nz(kSlotSqerr, to_fx(dd * dd));
  };
  // ... and the rest once the winner and price are known (tv = ctr * val, ratio = est / ctr)
  auto count_post = [&](int a, bool won, double lp, double price, double second, double bid, double tv,
                        double val, double ratio, int oc) {
    auto add_raw = [&](int j, unsigned long long v) { atomicAdd(s_cnt + ((size_t)(j * N + a) * R + rep), v); };
    auto add_nz = [&](int j, unsigned long long v) {
      if (v != 0ull) add_raw(j, v);
    };
    if (won) {
      add_nz(kSlotGross, to_fx(val * (double)oc));
      add_raw(kSlotPaid, to_fx(price));
      if (prm.mech == AG_FIRST_PRICE) add_nz(kSlotOverbid, to_fx(lp - second));
      add_raw(kSlotBias, to_fx(ratio));
    } else {
      add_nz(kSlotUnderbid, to_fx((lp - bid) * (double)(lp < tv)));
    }
    if (packed) {
      const uint64_t bit = 1ull << (8 * a);
      n_logs_packed += bit;
      if (won) n_won_packed += bit;
    } else {
      add_raw(kSlotCounts, won ? 0x100000001ull : 1ull);
    }
  };
#if AG_PREFETCH
  // software pipelining: the next tile's loads are in flight while this tile computes
  double xn[kMaxD][W];
  int pn[PA][W];
  double un[W];
  if (lo + wg_tile * (BT * W) + tid * W < hi) load_tile(lo + wg_tile * (BT * W) + tid * W);
#endif
  for (uint32_t base = lo + wg_tile * (BT * W); base < hi; base += stride) {
    const uint32_t i = base + tid * W;  // W consecutive auctions (even chunk bounds when W = 2)
    // generate mode: the auction's Philox counter (its global index) for the slots' draws
    const GenKey gk{(uint32_t)(prm.first + i), (uint32_t)((prm.first + i) >> 32), gk0, gk1};
    if constexpr (kStream && AG_STREAM_SYNC == 1) __syncthreads();
    [[maybe_unused]] const bool wg_full = base + BT * W <= hi;  // uniform over the workgroup
#if AG_PREFETCH
    if (i >= hi) continue;
#pragma unroll
    for (int e = 0; e < D - 1; ++e)
#pragma unroll
      for (int q = 0; q < W; ++q) xn[e][q] = xv[e][q];
#pragma unroll
    for (int s = 0; s < P; ++s)
#pragma unroll
      for (int q = 0; q < W; ++q) pn[s][q] = pv[s][q];
#pragma unroll
    for (int q = 0; q < W; ++q) un[q] = uv[q];
    if (i + stride < hi) load_tile(i + stride);
#define XV xn
#define PV pn
#define UV un
#else
    if (i >= hi) continue;
    if constexpr (P == 0) {
      // more than kMaxP participants (runtime P): the slots are resolved in a loop, their
      // outputs written as they come; the counter terms need the winner and price, so the
      // slots are resolved once more (the same arithmetic: the same values) afterwards
      const int Pn = prm.P;
      double x[kMaxD];
      float xf[kMaxD];
      float xabs = 1.0f;
#pragma unroll
      for (int e = 0; e < D - 1; ++e) {
        x[e] = ldg(in.ctx + e * B + i);
        xf[e] = (float)x[e];
        xabs += fabsf(xf[e]);
      }
      x[D - 1] = 1.0;  // intercept (src/Auction.py:33)
      xf[D - 1] = 1.0f;
      xabs *= 1.001f;
      const double u = ldg(in.u + i);
      double m1 = 0.0, m2 = -INFINITY, ctr_w = 0.0;
      int w = 0;
      for (int s = 0; s < Pn; ++s) {
        const uint32_t o = (uint32_t)s * B + i;
        const int a = ldg(in.part + o);
        const SlotResult q = resolve_slot<D, PRUNE, GENERAL>(T, K, x, xf, xabs, a, s, in, B, i, prm.ts_sample != 0);
        if (out.item) stg(out.item + o, (int32_t)q.item);
        if (out.bid) stg(out.bid + o, q.bid);
        if (out.est_ctr) stg(out.est_ctr + o, q.est);
        if (out.true_ctr) stg(out.true_ctr + o, q.ctr);
        if (out.best_ev) stg(out.best_ev + o, q.bev);
        if (out.gamma) stg(out.gamma + o, q.gamma);
        if (out.propensity) stg(out.propensity + o, q.prop);
        top2_step(s, q.bid, m1, m2, w);
        if (w == s) ctr_w = q.ctr;  // the current leader's true CTR
      }
      const double price = prm.mech == AG_FIRST_PRICE ? m1 : m2;
      const int oc = bernoulli(ctr_w, u);  // src/Auction.py:65
      if (out.winner) stg(out.winner + i, (int32_t)w);
      if (out.price) stg(out.price + i, charged ? price : (double)NAN);
      if (out.second_price) stg(out.second_price + i, charged ? m2 : (double)NAN);
      if (out.outcome) stg(out.outcome + i, (uint8_t)oc);
      if (out.winner_outcome) stg(out.winner_outcome + i, pack_wo(w, oc));
      if (prm.want_counters) {
        for (int s = 0; s < Pn; ++s) {
          const int a = ldg(in.part + (uint32_t)s * B + i);
          const SlotResult q =
              resolve_slot<D, PRUNE, GENERAL>(T, K, x, xf, xabs, a, s, in, B, i, prm.ts_sample != 0);
          count_slot(a, charged && s == w, charged ? price : 0.0, price, m2, q.bid, q.ctr, q.val, q.est, q.bev, oc);
        }
      }
      continue;
    }
    if constexpr (GEN)
      gen_tile(i);
    else
      load_tile(i);
    if constexpr (kDma) {
      // AG_TS_DMA: every input of the tile used here, so the compiler waits for all of its own
      // loads now -- none is left for it to wait for (with a count that cannot see the noise
      // DMAs) once the slots' DMAs are in flight
#pragma unroll
      for (int e = 0; e < D - 1; ++e) asm volatile("" ::"v"(xv[e][0]));
      asm volatile("" ::"v"(uv[0]));
      if constexpr (!kStream) {
#pragma unroll
        for (int s = 0; s < PA; ++s) asm volatile("" ::"v"(pv[s][0]), "v"(jv[s][0]));
      }
    }
#define XV xv
#define PV pv
#define UV uv
#endif

    if constexpr (kStream) {
      // Streamed slots (wide auctions): each slot resolved with its bid made in place (a fitted
      // policy's forward included), its outputs stored and its winner-independent counter terms
      // added at once, the top-2 carried along in slot order together with the leader's true
      // CTR, value and est / true ratio. Only each slot's bid and true EV stay live, for the
      // losers' underbid terms: 4 VGPRs per slot instead of the 16+ the deferred paths keep
      // (at P = 8 those spilled 880 B per lane to scratch in the 1024-lane build, more than
      // doubling its HBM traffic). The same values, the same exact integer counter terms.
      double x[kMaxD];
      float xf[kMaxD];
      float xabs = 1.0f;
#pragma unroll
      for (int e = 0; e < D - 1; ++e) {
        x[e] = XV[e][0];
        xf[e] = (float)x[e];
        xabs += fabsf(xf[e]);
      }
      x[D - 1] = 1.0;  // intercept (src/Auction.py:33)
      xf[D - 1] = 1.0f;
      xabs *= 1.001f;
      double m1 = 0.0, m2 = -INFINITY, ctr_w = 0.0, val_w = 0.0, rat_w = 0.0;
      int w = 0;
      double bidv[PA], tvv[PA];
#if AG_STREAM_PACK_AGENTS
      uint32_t apk[(PA + 1) / 2];  // the slots' agents, 16 bits each (N <= 65536), for the counter pass
#endif
#pragma unroll
      for (int s = 0; s < P; ++s) {
        if constexpr (AG_STREAM_SYNC == 2) {
          if (wg_full) __syncthreads();
        }
        const uint32_t o = s * B + i;
        const int a = GEN ? PV[s][0] : ldg(in.part + o);
#if AG_STREAM_PACK_AGENTS
        if (s & 1)
          apk[s >> 1] |= (uint32_t)a << 16;
        else
          apk[s >> 1] = (uint32_t)a;
#endif
        const SlotResult q = resolve_slot<D, PRUNE, GENERAL, false, GEN, DOS>(T, K, x, xf, xabs, a, s, in, B, i,
                                                                              prm.ts_sample != 0, kTsjLoad, gk);
        if (out.item) stg(out.item + o, (int32_t)q.item);
        if (out.bid) stg(out.bid + o, q.bid);
        if (out.est_ctr) stg(out.est_ctr + o, q.est);
        if (out.true_ctr) stg(out.true_ctr + o, q.ctr);
        if (out.best_ev) stg(out.best_ev + o, q.bev);
        if (out.gamma) stg(out.gamma + o, q.gamma);
        if (out.propensity) stg(out.propensity + o, q.prop);
        if (prm.want_counters) count_pre(a, q.ctr, q.val, q.est, q.bev);
        bidv[s] = q.bid;
        tvv[s] = q.ctr * q.val;
        // top2_step, with the leader's values captured as it changes (ties -> lowest slot)
        if (s == 0 || q.bid > m1) {
          if (s != 0) m2 = m1;
          m1 = q.bid;
          w = s;
          ctr_w = q.ctr;
          val_w = q.val;
          rat_w = q.est / q.ctr;
        } else if (q.bid > m2) {
          m2 = q.bid;
        }
      }
      const double price = prm.mech == AG_FIRST_PRICE ? m1 : m2;
      const int oc = bernoulli(ctr_w, UV[0]);  // src/Auction.py:65
      if (out.winner) stg(out.winner + i, (int32_t)w);
      if (out.price) stg(out.price + i, charged ? price : (double)NAN);
      if (out.second_price) stg(out.second_price + i, charged ? m2 : (double)NAN);
      if (out.outcome) stg(out.outcome + i, (uint8_t)oc);
      if (out.winner_outcome) stg(out.winner_outcome + i, pack_wo(w, oc));
      if (prm.want_counters) {
#pragma unroll
        for (int s = 0; s < P; ++s) {
#if AG_STREAM_PACK_AGENTS
          const int a = (int)((apk[s >> 1] >> (16 * (s & 1))) & 0xffffu);
#else
          const int a = GEN ? PV[s][0] : ldg(in.part + s * B + i);
#endif
          count_post(a, charged && s == w, charged ? price : 0.0, price, m2, bidv[s], tvv[s], val_w, rat_w, oc);
        }
      }
      continue;
    }
#if AG_EARLY_COUNT
    if constexpr (GENERAL == kGenAll && W == 1 && P > 0) {  // A/B: +2 % on kGenTruthful (configs_1), -4 % on the mix
      // each slot's outputs stored and its winner-independent counter terms added as soon
      // as it is resolved; only bid, value, true EV and est / true CTR stay live per slot
      double x[kMaxD];
      float xf[kMaxD];
      float xabs = 1.0f;
#pragma unroll
      for (int e = 0; e < D - 1; ++e) {
        x[e] = XV[e][0];
        xf[e] = (float)x[e];
        xabs += fabsf(xf[e]);
      }
      x[D - 1] = 1.0;  // intercept (src/Auction.py:33)
      xf[D - 1] = 1.0f;
      xabs *= 1.001f;
      // compacted policy bids in the 1024-lane build (large mixed populations); A/B: the
      // 256-lane build (FP_DM_TS / FP_DR_TS, every slot a policy bidder) is 3 % faster without
      constexpr bool kCompactPolicy = AG_POLICY_COMPACT != 0 && BT == kLargeThreads;
      double m1 = 0.0, m2 = -INFINITY, ctr_w = 0.0;
      int w = 0;
      double bidv[PA], valv[PA], tvv[PA], ratv[PA], ctrv[PA], estv[PA], gmv[PA], prv[PA];
      int polx[PA];  // the slot's place among the wave's fitted-policy tasks (-1: none)
      const int lane = (int)(threadIdx.x & 63);
      const uint64_t below = (1ull << lane) - 1ull;
      int ntask = 0, nslot = 0;
#pragma unroll
      for (int s = 0; s < P; ++s) {
        const uint32_t o = s * B + i;
        const int a = PV[s][0];
        const SlotResult q = resolve_slot<D, PRUNE, GENERAL, kCompactPolicy, GEN, DOS>(
            T, K, x, xf, xabs, a, s, in, B, i, prm.ts_sample != 0, AG_PREFETCH ? kTsjLoad : jv[s][0], gk);
        if (out.item) stg(out.item + o, (int32_t)q.item);
        if (out.est_ctr) stg(out.est_ctr + o, q.est);
        if (out.true_ctr) stg(out.true_ctr + o, q.ctr);
        if (out.best_ev) stg(out.best_ev + o, q.bev);
        if (prm.want_counters) count_pre(a, q.ctr, q.val, q.est, q.bev);
        bidv[s] = q.bid;
        valv[s] = q.val;
        tvv[s] = q.ctr * q.val;
        ratv[s] = q.est / q.ctr;
        ctrv[s] = q.ctr;
        estv[s] = q.est;
        gmv[s] = q.gamma;
        prv[s] = q.prop;
        const uint64_t m = __ballot(q.pol);
        polx[s] = q.pol ? ntask + __popcll(m & below) : -1;
        ntask += __popcll(m);
        nslot += m != 0ull;
      }
      // Fitted-policy bids (src/Bidder.py:466-470) of the wave's slots, compacted: the
      // tasks of all P slots go through this wave's LDS task slots, 64 per pass, so a wave
      // whose slots hold t policy bidders runs ceil(t / 64) policy forwards instead of one
      // per slot holding any. Same function, same inputs: the same bits.
      // workers: the wave's active lanes (a ragged last tile leaves the top lanes idle),
      // nact tasks per pass, worker k takes task slot k. Compacted only when that takes
      // fewer passes than the slots holding tasks (a population of policy bidders only,
      // FP_DM_TS / FP_DR_TS, has a task in every slot of every lane: each slot in place)
      const uint64_t act = __ballot(1);
      const int nact = __popcll(act), wrk = __popcll(act & below);
      if (!kCompactPolicy) {
        // policy bids were made in resolve_slot
      } else if (ntask > 0 && (ntask + nact - 1) / nact >= nslot) {
#pragma unroll
        for (int s = 0; s < P; ++s) {
          if (polx[s] >= 0) {
            double g, pr;
            const float eps = GEN ? gen_normal1(gk.c0, gk.c1, 0, 16u + (uint32_t)s, gk.k0, gk.k1)
                                  : ldg(in.policy_eps + (size_t)s * B + i);
            policy_bid(T.drs + PV[s][0] * T.drs_stride + 4, estv[s], valv[s], eps, T.tab, g, pr);
            gmv[s] = g;
            prv[s] = pr;
            bidv[s] = bidv[s] * g;
          }
        }
      } else if (kCompactPolicy && ntask > 0) {
        unsigned char *slots = smem + L.pol + (size_t)(threadIdx.x >> 6) * 64 * 32;
        for (int base = 0; base < ntask; base += nact) {  // wave-uniform
#pragma unroll
          for (int s = 0; s < P; ++s) {
            const int t = polx[s] - base;
            if (polx[s] >= 0 && t >= 0 && t < nact) {
              // the wave's task slots as structure of arrays (est, value [64] doubles, agent,
              // eps [64] words): a wave's lanes touch consecutive words, no bank conflict
              reinterpret_cast<double *>(slots)[t] = estv[s];
              reinterpret_cast<double *>(slots)[64 + t] = valv[s];
              reinterpret_cast<int32_t *>(slots + 1024)[t] = PV[s][0];
              reinterpret_cast<float *>(slots + 1280)[t] =
                  GEN ? gen_normal1(gk.c0, gk.c1, 0, 16u + (uint32_t)s, gk.k0, gk.k1)
                      : ldg(in.policy_eps + (size_t)s * B + i);
            }
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          if (wrk < ntask - base) {
            double *e0 = reinterpret_cast<double *>(slots) + wrk, *e1 = e0 + 64;
            const int a = reinterpret_cast<const int32_t *>(slots + 1024)[wrk];
            const float eps = reinterpret_cast<const float *>(slots + 1280)[wrk];
            double g, pr;
            policy_bid(T.drs + a * T.drs_stride + 4, *e0, *e1, eps, T.tab, g, pr);
            *e0 = g;
            *e1 = pr;
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
          for (int s = 0; s < P; ++s) {
            const int t = polx[s] - base;
            if (polx[s] >= 0 && t >= 0 && t < nact) {
              const double g = reinterpret_cast<const double *>(slots)[t];
              gmv[s] = g;
              prv[s] = reinterpret_cast<const double *>(slots)[64 + t];
              bidv[s] = bidv[s] * g;  // bid *= gamma, as resolve_slot does
            }
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
      }
#pragma unroll
      for (int s = 0; s < P; ++s) {
        const uint32_t o = s * B + i;
        if (out.bid) stg(out.bid + o, bidv[s]);
        if (out.gamma) stg(out.gamma + o, gmv[s]);
        if (out.propensity) stg(out.propensity + o, prv[s]);
        top2_step(s, bidv[s], m1, m2, w);
        if (w == s) ctr_w = ctrv[s];  // the current leader's true CTR
      }
      const double price = prm.mech == AG_FIRST_PRICE ? m1 : m2;
      const int oc = bernoulli(ctr_w, UV[0]);  // src/Auction.py:65
      if (out.winner) stg(out.winner + i, (int32_t)w);
      if (out.price) stg(out.price + i, charged ? price : (double)NAN);
      if (out.second_price) stg(out.second_price + i, charged ? m2 : (double)NAN);
      if (out.outcome) stg(out.outcome + i, (uint8_t)oc);
      if (out.winner_outcome) stg(out.winner_outcome + i, pack_wo(w, oc));
      if (prm.want_counters) {
#pragma unroll
        for (int s = 0; s < P; ++s)
          count_post(PV[s][0], charged && s == w, charged ? price : 0.0, price, m2, bidv[s], tvv[s], valv[s],
                     ratv[s], oc);
      }
      continue;
    }
#endif
    Resolved<PA> r[W];
#pragma unroll
    for (int q = 0; q < W; ++q) {
      double x[kMaxD];
      float xf[kMaxD];
      float xabs = 1.0f;
#pragma unroll
      for (int e = 0; e < D - 1; ++e) {
        x[e] = XV[e][q];
        xf[e] = (float)x[e];
        xabs += fabsf(xf[e]);
      }
      x[D - 1] = 1.0;  // intercept (src/Auction.py:33)
      xf[D - 1] = 1.0f;
      xabs *= 1.001f;
      int ag[PA], tj[PA];
#pragma unroll
      for (int s = 0; s < P; ++s) {
        ag[s] = PV[s][q];
        tj[s] = AG_PREFETCH ? kTsjLoad : jv[s][q];
      }
      resolve<PA, D, PRUNE, GENERAL, GEN, DOS>(T, K, prm.mech, x, xf, xabs, ag, UV[q], in, B, i + q,
                                              prm.ts_sample != 0, tj, r[q], gk);
    }

    // SoA stores, W auctions per access
#pragma unroll
    for (int s = 0; s < P; ++s) {
      const uint32_t o = s * B + i;
      int iv[W];
      double bv[W], cv[W], sv[W], ev[W], gv[W], pv2[W];
#pragma unroll
      for (int q = 0; q < W; ++q) {
        iv[q] = r[q].item[s];
        bv[q] = r[q].bid[s];
        cv[q] = r[q].ctr[s];
        sv[q] = r[q].est[s];
        ev[q] = r[q].bev[s];
        gv[q] = r[q].gamma[s];
        pv2[q] = r[q].prop[s];
      }
      if (out.item) st_i32<W>(out.item + o, iv);
      if (out.bid) st_f64<W>(out.bid + o, bv);
      if (out.est_ctr) st_f64<W>(out.est_ctr + o, sv);
      if (out.true_ctr) st_f64<W>(out.true_ctr + o, cv);
      if (out.best_ev) st_f64<W>(out.best_ev + o, ev);
      if (out.gamma) st_f64<W>(out.gamma + o, gv);
      if (out.propensity) st_f64<W>(out.propensity + o, pv2);
    }
    {
      int wv[W], ov[W];
      double pr[W], sp[W];
#pragma unroll
      for (int q = 0; q < W; ++q) {
        wv[q] = r[q].w;
        ov[q] = r[q].oc;
        pr[q] = charged ? r[q].price : NAN;
        sp[q] = charged ? r[q].second : NAN;
      }
      if (out.winner) st_i32<W>(out.winner + i, wv);
      if (out.price) st_f64<W>(out.price + i, pr);
      if (out.second_price) st_f64<W>(out.second_price + i, sp);
      if (out.outcome) st_u8<W>(out.outcome + i, ov);
      if (out.winner_outcome) {
#pragma unroll
        for (int q = 0; q < W; ++q) stg(out.winner_outcome + i + q, pack_wo(wv[q], ov[q]));
      }
    }

    if (prm.want_counters) {
#pragma unroll
      for (int q = 0; q < W; ++q) {
        const Resolved<PA> &rr = r[q];
#pragma unroll
        for (int s = 0; s < P; ++s)
          count_slot(rr.ag[s], charged && s == rr.w, charged ? rr.price : 0.0, rr.price, rr.second, rr.bid[s],
                     rr.ctr[s], rr.val[s], rr.est[s], rr.bev[s], rr.oc);
      }
    }
  }

#undef XV
#undef PV
#undef UV
  if (prm.want_counters) {
    if (packed) {
      for (int a = 0; a < N; ++a) {
        const uint64_t v = ((n_logs_packed >> (8 * a)) & 255ull) | (((n_won_packed >> (8 * a)) & 255ull) << 32);
        if (v) atomicAdd(s_cnt + ((size_t)(kSlotCounts * N + a) * R + rep), (unsigned long long)v);
      }
    }
    __syncthreads();
    // replica sums of every (slot, agent) pair in parallel, written over the pair's first two
    // replicas (two limbs, value = lo + hi * 2^42; counts: logs in lo, wins in hi)
    auto split = [&](int pair, unsigned long long c, long long &lo, long long &hi) {
      if (pair / N == kSlotCounts) {
        lo = (long long)(c & 0xffffffffull);
        hi = (long long)(c >> 32);
      } else {
        lo = (long long)c & kLimbMask;
        hi = (long long)c >> AG_FX_LIMB_BITS;
      }
    };
    const int pairs = L.ncnt * N;
    if (R >= 2) {
      for (int pr = tid; pr < pairs; pr += BT) {
        long long slo = 0, shi = 0;
        for (int r = 0; r < R; ++r) {
          long long l, h;
          split(pr, s_cnt[(size_t)pr * R + r], l, h);
          slo += l;
          shi += h;
        }
        s_cnt[(size_t)pr * R] = (unsigned long long)slo;
        s_cnt[(size_t)pr * R + 1] = (unsigned long long)shi;
      }
      __syncthreads();
    }
    for (int a = tid; a < N; a += BT) {
      long long lo[kGeneralSlots], hi[kGeneralSlots];
      unsigned long long nlogs = 0, nwon = 0;
      for (int j = 0; j < kGeneralSlots; ++j) {
        lo[j] = 0;
        hi[j] = 0;
        if (j >= L.ncnt) continue;
        const int pr = j * N + a;
        if (R >= 2) {
          lo[j] = (long long)s_cnt[(size_t)pr * R];
          hi[j] = (long long)s_cnt[(size_t)pr * R + 1];
        } else {
          split(pr, s_cnt[pr], lo[j], hi[j]);
        }
        if (j == kSlotCounts) {
          nlogs = (unsigned long long)lo[j];
          nwon = (unsigned long long)hi[j];
        }
      }
      // two limbs per counter (value = lo + hi * 2^42): no block total can overflow
      int64_t *dst = prm.partials + ((size_t)blockIdx.x * N + a) * kC * 2;
      auto put = [&](int c, long long lo, long long hi) {
        dst[2 * c] = lo;
        dst[2 * c + 1] = hi;
      };
      auto put_count = [&](int c, unsigned long long n) {
        put(c, (long long)((n & 63ull) << AG_FX_FRAC_BITS), (long long)(n >> 6));
      };
      put(AG_C_NET, lo[kSlotGross] - lo[kSlotPaid], hi[kSlotGross] - hi[kSlotPaid]);
      put(AG_C_GROSS, lo[kSlotGross], hi[kSlotGross]);
      put(AG_C_ALLOC_REGRET, lo[kSlotAlloc], hi[kSlotAlloc]);
      put(AG_C_EST_REGRET, lo[kSlotEst], hi[kSlotEst]);
      put(AG_C_OVERBID, lo[kSlotOverbid], hi[kSlotOverbid]);
      put(AG_C_UNDERBID, lo[kSlotUnderbid], hi[kSlotUnderbid]);
      put(AG_C_CTR_SQERR, lo[kSlotSqerr], hi[kSlotSqerr]);
      if (GENERAL)
        put(AG_C_CTR_BIAS, lo[kSlotBias], hi[kSlotBias]);
      else
        put_count(AG_C_CTR_BIAS, nwon);
      put(AG_C_BEST_EV, lo[kSlotBestEv], hi[kSlotBestEv]);
      put_count(AG_C_N_LOGS, nlogs);
      put_count(AG_C_N_WON, nwon);
      put(AG_C_PAID, lo[kSlotPaid], hi[kSlotPaid]);
    }
  }
}


typedef void (*SimKernel)(SimParams);

// Defined per participant count P in ag_sim_p.hip (one translation unit per P, compiled
// in parallel): the k_simulate instantiation for (D, screened search, auctions per lane).
template <int P>
SimKernel pick_kernel_for(int D, bool prune, int W, int general, int bt);
template <> SimKernel pick_kernel_for<0>(int, bool, int, int, int);
template <> SimKernel pick_kernel_for<1>(int, bool, int, int, int);
template <> SimKernel pick_kernel_for<2>(int, bool, int, int, int);
template <> SimKernel pick_kernel_for<3>(int, bool, int, int, int);
template <> SimKernel pick_kernel_for<4>(int, bool, int, int, int);
template <> SimKernel pick_kernel_for<5>(int, bool, int, int, int);
template <> SimKernel pick_kernel_for<6>(int, bool, int, int, int);
template <> SimKernel pick_kernel_for<7>(int, bool, int, int, int);
template <> SimKernel pick_kernel_for<8>(int, bool, int, int, int);

}  // namespace ag
