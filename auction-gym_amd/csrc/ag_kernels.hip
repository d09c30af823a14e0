// ag_kernels.hip -- MI355X (gfx950) kernels + C-ABI for the AuctionGym hot path.
//
//   Auction.simulate_opportunity (src/Auction.py:28-74)
//     -> Agent.bid / select_item (src/Agent.py:29-68) -> OracleAllocator.estimate_CTR
//        (src/BidderAllocation.py:81-82) -> TruthfulBidder.bid (src/Bidder.py:34-35)
//     -> {First,Second}Price.allocate (src/AuctionAllocation.py:19-34)
//     -> Agent.charge / set_price (src/Agent.py:70-77) and the metric getters
//        (src/Agent.py:96-118) as per-agent counters.
//
// One lane per auction; B auctions laid out structure-of-arrays in HBM so every load and
// store of a wave is 64 consecutive elements. The item catalogue, the exp table and the
// counter accumulators live in LDS. Counters are exact fixed-point sums (include/
// auctiongym.h AG_FX_*), so totals do not depend on grid, block order or GPU count.
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off (see ../Makefile). The FP64
// arithmetic must not be contracted: every FMA the reference's BLAS / libm performs is
// written explicitly with fma().
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <string>

#include "auctiongym.h"
#include "ag_exp.h"
#include "ag_exp_table.h"

// ------------------------------------------------------------------------------------
// error plumbing
// ------------------------------------------------------------------------------------
static thread_local std::string g_last_error;

static int set_error(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
static int set_error(int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

#define AG_HIP(call)                                                                    \
  do {                                                                                  \
    hipError_t e_ = (call);                                                             \
    if (e_ != hipSuccess)                                                               \
      return set_error(AG_ERR_HIP, "%s: %s (%s:%d)", #call, hipGetErrorString(e_),      \
                       __FILE__, __LINE__);                                             \
  } while (0)

namespace {

constexpr int kThreads = 256;              // 4 waves of 64 lanes
constexpr int kC = AG_NUM_COUNTERS;
constexpr int kMaxAuctionsPerBlock = 65536; // per launch: keeps a replica's int64 sum exact
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
  int32_t tab, items, values, scr, scr_val, amax, cnt, total;
  int32_t items_stride;    // doubles between agents (odd: spreads agents over banks)
  int32_t values_stride;   // doubles
  int32_t scr_stride;      // floats between agents in the screening catalogue
  int32_t scr_val_stride;  // floats
  int32_t kpairs;          // item pairs in the screening catalogue (K rounded up to even)
  int32_t replicas;        // per-lane counter replicas (power of 2, <= 64)
  int32_t ncnt;            // counter slots held in LDS
};

__host__ inline int32_t align16(int64_t b) { return (int32_t)((b + 15) & ~(int64_t)15); }

// Counter slots accumulated in LDS for OracleAllocator + TruthfulBidder populations:
//   0 GROSS, 1 PAID, 2 OVERBID (FirstPrice only: price - second_price == 0 under SP),
//   3 UNDERBID, 4 BEST_EV, 5 packed counts (n_logs in bits 0-31, n_won in bits 32-63).
// Derived at write-out: NET = GROSS - PAID (both exact fixed-point sums), CTR_BIAS =
// N_WON (est/true == 1 for Oracle agents); ALLOC / EST regrets and CTR_SQERR are
// identically zero for them (estimated CTR == true CTR, best_ev == true_ctr * value).
constexpr int kOracleSlots = 6;
enum { kSlotGross = 0, kSlotPaid, kSlotOverbid, kSlotUnderbid, kSlotBestEv, kSlotCounts };

__host__ inline LdsLayout make_layout(int N, int K, int D, bool counters) {
  LdsLayout L;
  L.items_stride = (K * D) | 1;
  L.values_stride = K | 1;
  L.kpairs = (K + 1) / 2;
  // [pair][dim 0..7][2 items] floats; + 4 floats so agents start on different 16-B slots
  L.scr_stride = L.kpairs * 16 + 4;
  L.scr_val_stride = L.kpairs * 2 + 2;
  L.ncnt = kOracleSlots;
  int R = 64;
  while (R > 1 && (int64_t)R * N * L.ncnt * 8 > 32768) R >>= 1;
  L.replicas = R;
  int64_t b = 0;
  L.tab = 0;
  b += 256 * 8;
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
  L.cnt = align16(b);
  b = L.cnt + (counters ? (int64_t)R * N * L.ncnt * 8 : 0);
  L.total = align16(b);
  return L;
}

struct SimParams {
  int32_t B;              // auctions in this launch (< 2^28: 32-bit SoA indexing)
  int32_t N, K, mech;
  int32_t want_counters;
  LdsLayout lds;
  const double *items;    // global [N][K][D]
  const double *values;   // global [N][K]
  ag_batch_in in;
  ag_batch_out out;
  int64_t *partials;      // [grid][N][AG_NUM_COUNTERS]
};

// Screening margin. The f32 score of item k is v_k / (1 + 2^(z'_k)) with z'_k the f32 dot
// of the catalogue row pre-scaled by -log2(e). With S = sum_d |a_d x_d| <= kPruneMaxS its
// relative error is eps <= S 2^-21 (inputs rounded to f32, D <= 8 FMAs) + |z| 2^-23 (exp2
// argument) + 2^-21 (exp2, add, rcp, mul) < 4.2e-5, so every item whose EXACT score is the
// maximum has f32 score >= max_f32 (1 - eps)/(1 + eps) > max_f32 (1 - kPruneDelta) with
// kPruneDelta = 2^-13 = 1.22e-4 > 2 eps: re-scoring every item above that threshold
// exactly keeps the exact argmax and all its exact ties. Lanes outside the bound (or with
// a vanishing f32 maximum) re-score every item exactly.
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
    const double c = agexp::sigmoid(dot_ref<D>(itm + k * D, x), tab);
    const double sc = c * vv[k];
    if (best < 0 || sc > best_s || (sc == best_s && k < best)) {
      best = k;
      best_s = sc;
      best_c = c;
    }
  };
  if constexpr (PRUNE) {
    // f32 screen of one item pair: scores of items 2p, 2p+1 (padding items score 0)
    auto screen = [&](int p) -> f32x2 {
      const float *row = scr + p * 16;
      f32x2 z = {0.0f, 0.0f};
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const f32x2 a = *reinterpret_cast<const f32x2 *>(row + 2 * d);
        const f32x2 xd = {xf[d], xf[d]};
        z = __builtin_elementwise_fma(a, xd, z);
      }
      const f32x2 one = {1.0f, 1.0f};
      const f32x2 t = f32x2{__builtin_amdgcn_exp2f(z.x), __builtin_amdgcn_exp2f(z.y)} + one;
      const f32x2 r = {__builtin_amdgcn_rcpf(t.x), __builtin_amdgcn_rcpf(t.y)};
      return *reinterpret_cast<const f32x2 *>(sv + 2 * p) * r;
    };
    // pass 1: f32 leader kf, its score and the runner-up score
    float mx = 0.0f, m2 = 0.0f;
    int kf = 0;
    for (int p = 0; p < kpairs; ++p) {
      const f32x2 sc = screen(p);
      const float lo = fminf(sc.x, sc.y), hi = fmaxf(sc.x, sc.y);
      const int khi = sc.y > sc.x ? 2 * p + 1 : 2 * p;
      if (hi > mx) {
        m2 = fmaxf(mx, lo);
        mx = hi;
        kf = khi;
      } else {
        m2 = fmaxf(m2, hi);
      }
    }
    const bool ok = (amax * xabs <= kPruneMaxS) && (mx >= 1e-30f);
    const float thr = ok ? mx * (1.0f - kPruneDelta) : -1.0f;
    exact(kf);  // the f32 leader: every lane, no divergence
    if (m2 >= thr) {
      // near-tie (rare) or unscreenable lane: re-score every other item above thr
      for (int p = 0; p < kpairs; ++p) {
        const f32x2 sc = screen(p);
        if (2 * p != kf && sc.x >= thr) exact(2 * p);
        if (2 * p + 1 != kf && 2 * p + 1 < K && sc.y >= thr) exact(2 * p + 1);
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
template <int P, int D, bool PRUNE>
__global__ __launch_bounds__(kThreads) void k_simulate(SimParams prm) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int N = prm.N, K = prm.K;
  const uint32_t B = (uint32_t)prm.B;
  const LdsLayout L = prm.lds;
  uint64_t *s_tab = reinterpret_cast<uint64_t *>(smem + L.tab);
  double *s_items = reinterpret_cast<double *>(smem + L.items);
  double *s_vals = reinterpret_cast<double *>(smem + L.values);
  float *s_scr = reinterpret_cast<float *>(smem + L.scr);
  float *s_scr_val = reinterpret_cast<float *>(smem + L.scr_val);
  float *s_amax = reinterpret_cast<float *>(smem + L.amax);
  unsigned long long *s_cnt = reinterpret_cast<unsigned long long *>(smem + L.cnt);

  const int tid = threadIdx.x;
  for (int i = tid; i < 256; i += kThreads) s_tab[i] = ag_exp_tab[i];
  for (int i = tid; i < N * K * D; i += kThreads) {
    const int a = i / (K * D), r = i - a * (K * D);
    s_items[a * L.items_stride + r] = prm.items[i];
  }
  for (int i = tid; i < N * K; i += kThreads) {
    const int a = i / K, r = i - a * K;
    s_vals[a * L.values_stride + r] = prm.values[i];
  }
  if (PRUNE) {
    // screening rows: [pair p][dim d][item 2p, 2p+1], coefficients * -log2(e); padded
    // dims and the odd item's partner are 0 (value 0 -> score 0, never the leader)
    for (int i = tid; i < N * L.kpairs * 16; i += kThreads) {
      const int a = i / (L.kpairs * 16), r = i - a * (L.kpairs * 16);
      const int p = r >> 4, d = (r >> 1) & 7, k = 2 * p + (r & 1);
      const float c = (d < D && k < K) ? (float)prm.items[((size_t)a * K + k) * D + d] : 0.0f;
      s_scr[a * L.scr_stride + r] = c * kNegLog2e;
    }
    for (int i = tid; i < N * L.kpairs * 2; i += kThreads) {
      const int a = i / (L.kpairs * 2), k = i - a * (L.kpairs * 2);
      s_scr_val[a * L.scr_val_stride + k] = k < K ? (float)prm.values[(size_t)a * K + k] : 0.0f;
    }
    for (int a = tid; a < N; a += kThreads) {
      float m = 0.0f;
      for (int r = 0; r < K * D; ++r) m = fmaxf(m, (float)fabs(prm.items[(size_t)a * K * D + r]));
      s_amax[a] = m * 1.001f;
    }
  }
  const int R = L.replicas;
  if (prm.want_counters)
    for (int i = tid; i < R * N * L.ncnt; i += kThreads) s_cnt[i] = 0ull;
  __syncthreads();

  const int rep = tid & (R - 1);
  const ag_batch_in in = prm.in;
  const ag_batch_out out = prm.out;

  for (uint32_t base = blockIdx.x * kThreads; base < B; base += gridDim.x * kThreads) {
    const uint32_t i = base + tid;
    if (i >= B) continue;

    double x[kMaxD];
    float xf[kMaxD];
    float xabs = 1.0f;
#pragma unroll
    for (int e = 0; e < D - 1; ++e) {
      x[e] = in.ctx[e * B + i];
      xf[e] = (float)x[e];
      xabs += fabsf(xf[e]);
    }
    x[D - 1] = 1.0;  // intercept (src/Auction.py:33)
    xf[D - 1] = 1.0f;
    xabs *= 1.001f;
    const double u = in.u[i];

    int ag[P];
    double val[P], bid[P], ctr[P], bev[P];
    int w = 0;
    double m1 = 0.0, m2 = -INFINITY;

#pragma unroll
    for (int s = 0; s < P; ++s) {
      const int a = in.part[s * B + i];
      ag[s] = a;
      double c, bs;
      const int best = select_item<D, PRUNE>(s_items + a * L.items_stride, s_vals + a * L.values_stride,
                                             s_scr + a * L.scr_stride, s_scr_val + a * L.scr_val_stride,
                                             PRUNE ? s_amax[a] : 0.0f, K, L.kpairs, x, xf, xabs, s_tab,
                                             c, bs);
      const double v = s_vals[a * L.values_stride + best];
      const double b = v * c;  // TruthfulBidder.bid
      val[s] = v;
      bid[s] = b;
      ctr[s] = c;   // Oracle: estimated CTR == true CTR, bit for bit
      bev[s] = bs;  // max_k true_CTR_k * value_k
      const uint32_t o = s * B + i;
      if (out.item) out.item[o] = best;
      if (out.bid) out.bid[o] = b;
      if (out.est_ctr) out.est_ctr[o] = c;
      if (out.true_ctr) out.true_ctr[o] = c;
      if (out.best_ev) out.best_ev[o] = bs;
      // streaming top-2, ties -> lowest slot
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

    const bool charged = P >= 2;  // P == 1: empty price arrays, nobody charged
    const double price = prm.mech == AG_FIRST_PRICE ? m1 : m2;
    const double second = m2;
    double ctr_w = ctr[0];
#pragma unroll
    for (int s = 1; s < P; ++s)
      if (s == w) ctr_w = ctr[s];
    const int oc = bernoulli(ctr_w, u);
    if (out.winner) out.winner[i] = w;
    if (out.price) out.price[i] = charged ? price : NAN;
    if (out.second_price) out.second_price[i] = charged ? second : NAN;
    if (out.outcome) out.outcome[i] = (uint8_t)oc;

    if (prm.want_counters) {
      // [slot j][agent a][replica]: lane-private replicas, conflict-free 8-B atomics
      auto add_raw = [&](int j, int a, unsigned long long v) {
        atomicAdd(s_cnt + ((size_t)(j * N + a) * R + rep), v);
      };
#pragma unroll
      for (int s = 0; s < P; ++s) {
        const bool won = charged && s == w;
        const double lp = charged ? price : 0.0;
        const double tv = ctr[s] * val[s];
        if (won) {
          add_raw(kSlotGross, ag[s], to_fx(val[s] * (double)oc));
          add_raw(kSlotPaid, ag[s], to_fx(price));
          if (prm.mech == AG_FIRST_PRICE) add_raw(kSlotOverbid, ag[s], to_fx(lp - second));
        } else {
          add_raw(kSlotUnderbid, ag[s], to_fx((lp - bid[s]) * (double)(lp < tv)));
        }
        add_raw(kSlotBestEv, ag[s], to_fx(bev[s]));
        add_raw(kSlotCounts, ag[s], won ? 0x100000001ull : 1ull);
      }
    }
  }

  if (prm.want_counters) {
    __syncthreads();
    for (int a = tid; a < N; a += kThreads) {
      long long lo[kOracleSlots], hi[kOracleSlots];
      unsigned long long nlogs = 0, nwon = 0;
      for (int j = 0; j < kOracleSlots; ++j) {
        lo[j] = 0;
        hi[j] = 0;
        for (int r = 0; r < R; ++r) {
          const unsigned long long c = s_cnt[(size_t)(j * N + a) * R + r];
          if (j == kSlotCounts) {
            nlogs += c & 0xffffffffull;
            nwon += c >> 32;
          } else {
            lo[j] += (long long)c & kLimbMask;
            hi[j] += (long long)c >> AG_FX_LIMB_BITS;
          }
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
      put(AG_C_ALLOC_REGRET, 0, 0);
      put(AG_C_EST_REGRET, 0, 0);
      put(AG_C_OVERBID, lo[kSlotOverbid], hi[kSlotOverbid]);
      put(AG_C_UNDERBID, lo[kSlotUnderbid], hi[kSlotUnderbid]);
      put(AG_C_CTR_SQERR, 0, 0);
      put_count(AG_C_CTR_BIAS, nwon);
      put(AG_C_BEST_EV, lo[kSlotBestEv], hi[kSlotBestEv]);
      put_count(AG_C_N_LOGS, nlogs);
      put_count(AG_C_N_WON, nwon);
      put(AG_C_PAID, lo[kSlotPaid], hi[kSlotPaid]);
    }
  }
}

// Sum the per-block partials (two limbs each) of one counter exactly into its limbs
// (one block per (agent, counter)). Integer sums: any order gives the same bits.
__global__ __launch_bounds__(kThreads) void k_reduce_counters(const int64_t *__restrict__ partials,
                                                              int nblocks, int ncounters,
                                                              int64_t *__restrict__ limbs) {
  __shared__ long long s0[kThreads], s1[kThreads];
  const int j = blockIdx.x;
  long long a0 = 0, a1 = 0;
  for (int b = threadIdx.x; b < nblocks; b += kThreads) {
    a0 += partials[((size_t)b * ncounters + j) * 2];
    a1 += partials[((size_t)b * ncounters + j) * 2 + 1];
  }
  s0[threadIdx.x] = a0;
  s1[threadIdx.x] = a1;
  __syncthreads();
  for (int st = kThreads / 2; st > 0; st >>= 1) {
    if (threadIdx.x < st) {
      s0[threadIdx.x] += s0[threadIdx.x + st];
      s1[threadIdx.x] += s1[threadIdx.x + st];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    int64_t *L = limbs + (size_t)j * AG_FX_LIMBS;
    long long l0 = L[0] + s0[0], l1 = L[1] + s1[0], l2 = L[2];
    long long c = l0 >> AG_FX_LIMB_BITS;
    l0 &= kLimbMask;
    l1 += c;
    c = l1 >> AG_FX_LIMB_BITS;
    l1 &= kLimbMask;
    l2 += c;
    L[0] = l0;
    L[1] = l1;
    L[2] = l2;
  }
}

// ------------------------------------------------------------------------------------
// allocate kernels (src/AuctionAllocation.py)
// ------------------------------------------------------------------------------------
__device__ __forceinline__ void write_alloc(int mech, int P, int64_t i, int w, double m1, double m2,
                                            int32_t *winner, double *price, double *second) {
  if (winner) winner[i] = w;
  if (P < 2) {
    if (price) price[i] = mech == AG_FIRST_PRICE ? m1 : NAN;
    if (second) second[i] = NAN;
  } else {
    if (price) price[i] = mech == AG_FIRST_PRICE ? m1 : m2;
    if (second) second[i] = m2;
  }
}

// Small P: one lane per auction, streaming top-2 over the coalesced [P][B] rows.
__global__ __launch_bounds__(kThreads) void k_allocate_lane(const double *__restrict__ bids, int64_t B,
                                                           int P, int mech, int32_t *winner,
                                                           double *price, double *second) {
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < B;
       i += (int64_t)gridDim.x * kThreads) {
    double m1 = bids[i], m2 = -INFINITY;
    int w = 0;
    for (int s = 1; s < P; ++s) {
      const double b = bids[(int64_t)s * B + i];
      if (b > m1) {
        m2 = m1;
        m1 = b;
        w = s;
      } else if (b > m2) {
        m2 = b;
      }
    }
    write_alloc(mech, P, i, w, m1, m2, winner, price, second);
  }
}

// Large P: a tile of T auctions is staged through LDS with coalesced row reads, then one
// wave resolves each auction: lanes take slots lane, lane+64, ..., keep a local top-2 and
// the wave merges them with DPP/shuffles on the key (bid desc, slot asc).
__device__ __forceinline__ void merge_top2(double &m1, int &i1, double &m2, double n1, int j1, double n2) {
  const bool other = (n1 > m1) || (n1 == m1 && j1 < i1);
  if (other) {
    m2 = fmax(m1, n2);
    m1 = n1;
    i1 = j1;
  } else {
    m2 = fmax(m2, n1);
  }
}

__global__ __launch_bounds__(kThreads) void k_allocate_wave(const double *__restrict__ bids, int64_t B,
                                                           int P, int T, int mech, int32_t *winner,
                                                           double *price, double *second) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double *tile = reinterpret_cast<double *>(smem);  // [P][T]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int64_t base = (int64_t)blockIdx.x * T; base < B; base += (int64_t)gridDim.x * T) {
    const int nt = (int)min((int64_t)T, B - base);
    for (int e = threadIdx.x; e < P * T; e += kThreads) {
      const int s = e / T, j = e - s * T;
      tile[e] = j < nt ? bids[(int64_t)s * B + base + j] : 0.0;
    }
    __syncthreads();
    for (int j = wv; j < nt; j += kThreads / 64) {
      double m1 = -INFINITY, m2 = -INFINITY;
      int i1 = 0x7fffffff;
      for (int s = lane; s < P; s += 64) merge_top2(m1, i1, m2, tile[s * T + j], s, -INFINITY);
      for (int d = 32; d > 0; d >>= 1) {
        const double n1 = __shfl_xor(m1, d), n2 = __shfl_xor(m2, d);
        const int j1 = __shfl_xor(i1, d);
        merge_top2(m1, i1, m2, n1, j1, n2);
      }
      if (lane == 0) write_alloc(mech, P, base + j, i1, m1, m2, winner, price, second);
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------
// synthetic batch generator (Philox4x32-10; oracle/ag_oracle.c restates the integer part)
// ------------------------------------------------------------------------------------
__device__ __forceinline__ void philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                       uint32_t k0, uint32_t k1, uint32_t (&o)[4]) {
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

__global__ __launch_bounds__(kThreads) void k_generate(uint64_t seed, uint64_t first, int64_t B, int N, int P,
                                                      int E, double scale, double *ctx, int32_t *part,
                                                      double *u) {
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < B;
       i += (int64_t)gridDim.x * kThreads) {
    const uint64_t idx = first + (uint64_t)i;
    const uint32_t c0 = (uint32_t)idx, c1 = (uint32_t)(idx >> 32);
    uint32_t w[4];
    philox(c0, c1, 0, 0, k0, k1, w);
    u[i] = (double)((((uint64_t)w[0] << 32) | w[1]) >> 11) * 0x1p-53;
    // participants: Floyd's algorithm, slot order = insertion order (stream 1)
    int picked[64];
    int n = 0;
    for (int j = N - P; j < N; ++j) {
      const int step = j - (N - P);
      if ((step & 3) == 0) philox(c0, c1, (uint32_t)(step >> 2), 1, k0, k1, w);
      int pick = (int)(((uint64_t)w[step & 3] * (uint64_t)(j + 1)) >> 32);
      for (int q = 0; q < n; ++q)
        if (picked[q] == pick) {
          pick = j;
          break;
        }
      picked[n++] = pick;
      part[(int64_t)step * B + i] = pick;
    }
    // context: Box-Muller pairs (stream 2), ctx = 0 + scale * z (numpy normal(0, scale))
    for (int m = 0; 2 * m < E; ++m) {
      philox(c0, c1, (uint32_t)m, 2, k0, k1, w);
      const double u1 = (double)(((((uint64_t)w[0] << 32) | w[1]) >> 11) + 1) * 0x1p-53;
      const double u2 = (double)((((uint64_t)w[2] << 32) | w[3]) >> 11) * 0x1p-53;
      const double r = sqrt(-2.0 * log(u1));
      double sn, cs;
      sincospi(2.0 * u2, &sn, &cs);
      ctx[(int64_t)(2 * m) * B + i] = 0.0 + scale * (r * cs);
      if (2 * m + 1 < E) ctx[(int64_t)(2 * m + 1) * B + i] = 0.0 + scale * (r * sn);
    }
  }
}

// ------------------------------------------------------------------------------------
// known-answer kernels
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void k_exp_kat(const double *x, double *y, int64_t n, int sig) {
  __shared__ uint64_t s_tab[256];
  for (int i = threadIdx.x; i < 256; i += kThreads) s_tab[i] = ag_exp_tab[i];
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads)
    y[i] = sig ? agexp::sigmoid(x[i], s_tab) : agexp::exp(x[i], s_tab);
}

// ------------------------------------------------------------------------------------
// dispatch
// ------------------------------------------------------------------------------------
typedef void (*SimKernel)(SimParams);

template <int P, bool PRUNE>
SimKernel pick_d(int D) {
  switch (D) {
    case 2: return k_simulate<P, 2, PRUNE>;
    case 3: return k_simulate<P, 3, PRUNE>;
    case 4: return k_simulate<P, 4, PRUNE>;
    case 5: return k_simulate<P, 5, PRUNE>;
    case 6: return k_simulate<P, 6, PRUNE>;
    case 7: return k_simulate<P, 7, PRUNE>;
    case 8: return k_simulate<P, 8, PRUNE>;
    default: return nullptr;
  }
}

template <int P>
SimKernel pick_prune(int D, bool prune) {
  if (prune) return pick_d<P, true>(D);
  if (D <= 8) return pick_d<P, false>(D);
  switch (D) {
    case 9: return k_simulate<P, 9, false>;
    case 11: return k_simulate<P, 11, false>;
    case 13: return k_simulate<P, 13, false>;
    case 16: return k_simulate<P, 16, false>;
    default: return nullptr;
  }
}

// prune: the f32-screened item search (D <= 8, K <= kPruneMaxK); otherwise exact scan.
SimKernel pick_kernel(int P, int D, bool prune) {
  switch (P) {
    case 1: return pick_prune<1>(D, prune);
    case 2: return pick_prune<2>(D, prune);
    case 3: return pick_prune<3>(D, prune);
    case 4: return pick_prune<4>(D, prune);
    case 5: return pick_prune<5>(D, prune);
    case 6: return pick_prune<6>(D, prune);
    case 7: return pick_prune<7>(D, prune);
    case 8: return pick_prune<8>(D, prune);
    default: return nullptr;
  }
}

int grid_for(int64_t B, int64_t per_block_cap) {
  int64_t tiles = (B + kThreads - 1) / kThreads;
  int64_t need = (B + per_block_cap - 1) / per_block_cap;
  int64_t g = tiles < kMinGrid ? tiles : (need > kMinGrid ? need : kMinGrid);
  return (int)(g < 1 ? 1 : g);
}

}  // namespace

// ------------------------------------------------------------------------------------
// C-ABI
// ------------------------------------------------------------------------------------
struct ag_ctx {
  int32_t device;
  ag_shape shape;
  int32_t D;
  int32_t item_search = AG_ITEM_SEARCH_AUTO;
  bool can_simulate = false;
  double *d_items = nullptr;
  double *d_values = nullptr;
  int64_t *d_partials = nullptr;
  int32_t partial_blocks = 0;
  int32_t resident[4] = {0, 0, 0, 0};  // resident k_simulate blocks [screened][counters]
  bool catalog = false;
};

namespace {
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) == hipSuccess && prev != dev) hipSetDevice(dev);
    else prev = -1;
  }
  ~DeviceGuard() {
    if (prev >= 0) hipSetDevice(prev);
  }
};
}  // namespace

extern "C" {

const char *ag_last_error(void) { return g_last_error.c_str(); }
int32_t ag_abi_version(void) { return AG_ABI_VERSION; }

int ag_create(int32_t device, const ag_shape *s, ag_ctx **out) {
  if (!s || !out) return set_error(AG_ERR_INVALID, "ag_create: null argument");
  *out = nullptr;
  if (s->num_agents < 1 || s->num_items < 1 || s->embedding_size < 1)
    return set_error(AG_ERR_INVALID, "ag_create: N, K, E must be >= 1 (N=%d K=%d E=%d)",
                     s->num_agents, s->num_items, s->embedding_size);
  if (s->num_participants < 1 || s->num_participants > s->num_agents)
    return set_error(AG_ERR_INVALID,
                     "ag_create: Cannot take a larger sample than population when replace is "
                     "False (P=%d, N=%d; src/Auction.py:42)",
                     s->num_participants, s->num_agents);
  if (s->mechanism != AG_FIRST_PRICE && s->mechanism != AG_SECOND_PRICE)
    return set_error(AG_ERR_INVALID, "ag_create: unknown mechanism %d", s->mechanism);
  if (s->num_slots != 1)
    return set_error(AG_ERR_UNSUPPORTED, "ag_create: num_slots must be 1 (src/main.py:37)");
  const int D = s->embedding_size + 1;
  if (s->num_participants > 4096)
    return set_error(AG_ERR_UNSUPPORTED, "ag_create: P=%d > 4096", s->num_participants);
  if (s->obs_embedding_size < 0 || s->obs_embedding_size > s->embedding_size)
    return set_error(AG_ERR_INVALID, "ag_create: obs_embedding_size out of range");
  ag_ctx *c = new ag_ctx();
  c->device = device;
  c->shape = *s;
  c->D = D;
  const int nc = s->num_agents * kC;
  // simulate needs a kernel for (P, D) and the catalogue in LDS; allocate-only contexts
  // (any P) do not.
  const LdsLayout lay = make_layout(s->num_agents, s->num_items, D, true);
  c->can_simulate = s->num_participants <= kMaxP && pick_kernel(s->num_participants, D, false) &&
                    lay.total <= 160 * 1024;
  DeviceGuard g(device);
  hipError_t e = hipMalloc(&c->d_items, sizeof(double) * s->num_agents * s->num_items * D);
  if (e == hipSuccess) e = hipMalloc(&c->d_values, sizeof(double) * s->num_agents * s->num_items);
  // partials for the largest grid a call can use: grids grow past kMinGrid only to keep
  // <= kMaxAuctionsPerBlock auctions per block; allocate lazily beyond the default.
  c->partial_blocks = kMaxSimGrid;
  if (e == hipSuccess) e = hipMalloc(&c->d_partials, sizeof(int64_t) * 2 * (size_t)kMaxSimGrid * nc);
  if (e != hipSuccess) {
    (void)hipFree(c->d_items);
    (void)hipFree(c->d_values);
    (void)hipFree(c->d_partials);
    delete c;
    return set_error(AG_ERR_HIP, "ag_create: hipMalloc: %s", hipGetErrorString(e));
  }
  *out = c;
  return AG_OK;
}

int ag_destroy(ag_ctx *c) {
  if (!c) return AG_OK;
  DeviceGuard g(c->device);
  (void)hipFree(c->d_items);
  (void)hipFree(c->d_values);
  (void)hipFree(c->d_partials);
  delete c;
  return AG_OK;
}

int ag_set_agent_kinds(ag_ctx *c, const int32_t *alloc_kind, const int32_t *bid_kind) {
  if (!c) return set_error(AG_ERR_INVALID, "ag_set_agent_kinds: null ctx");
  for (int a = 0; a < c->shape.num_agents; ++a) {
    if (alloc_kind && alloc_kind[a] != AG_ALLOCATOR_ORACLE)
      return set_error(AG_ERR_UNSUPPORTED, "agent %d: allocator kind %d not implemented", a, alloc_kind[a]);
    if (bid_kind && bid_kind[a] != AG_BIDDER_TRUTHFUL)
      return set_error(AG_ERR_UNSUPPORTED, "agent %d: bidder kind %d not implemented", a, bid_kind[a]);
  }
  return AG_OK;
}

int ag_set_option(ag_ctx *c, int32_t option, int64_t value) {
  if (!c) return set_error(AG_ERR_INVALID, "ag_set_option: null ctx");
  switch (option) {
    case AG_OPT_ITEM_SEARCH:
      if (value != AG_ITEM_SEARCH_AUTO && value != AG_ITEM_SEARCH_EXACT)
        return set_error(AG_ERR_INVALID, "ag_set_option: bad item search mode %lld", (long long)value);
      c->item_search = (int32_t)value;
      return AG_OK;
    default:
      return set_error(AG_ERR_INVALID, "ag_set_option: unknown option %d", option);
  }
}

int ag_load_catalog(ag_ctx *c, const double *item_emb, const double *item_val) {
  if (!c || !item_emb || !item_val) return set_error(AG_ERR_INVALID, "ag_load_catalog: null argument");
  DeviceGuard g(c->device);
  const size_t n = (size_t)c->shape.num_agents * c->shape.num_items;
  AG_HIP(hipMemcpy(c->d_items, item_emb, n * c->D * sizeof(double), hipMemcpyHostToDevice));
  AG_HIP(hipMemcpy(c->d_values, item_val, n * sizeof(double), hipMemcpyHostToDevice));
  c->catalog = true;
  return AG_OK;
}

int ag_allocate(ag_ctx *c, const double *bids, int64_t B, int32_t *winner, double *price,
                double *second_price, void *stream) {
  if (!c || (!bids && B > 0)) return set_error(AG_ERR_INVALID, "ag_allocate: null argument");
  if (B < 0) return set_error(AG_ERR_INVALID, "ag_allocate: B < 0");
  if (B == 0) return AG_OK;
  DeviceGuard g(c->device);
  const int P = c->shape.num_participants, mech = c->shape.mechanism;
  hipStream_t st = (hipStream_t)stream;
  if (P <= 16) {
    const int grid = grid_for(B, (int64_t)1 << 40);
    hipLaunchKernelGGL(k_allocate_lane, dim3(grid), dim3(kThreads), 0, st, bids, B, P, mech, winner,
                       price, second_price);
  } else {
    int T = 4096 / P;
    T = T < 1 ? 1 : (T > 64 ? 64 : T);
    const int64_t tiles = (B + T - 1) / T;
    const int grid = (int)(tiles < 4096 ? tiles : 4096);
    hipLaunchKernelGGL(k_allocate_wave, dim3(grid), dim3(kThreads), (size_t)P * T * 8, st, bids, B, P, T,
                       mech, winner, price, second_price);
  }
  AG_HIP(hipGetLastError());
  return AG_OK;
}

int ag_simulate(ag_ctx *c, int64_t B, const ag_batch_in *in, ag_batch_out *out, int64_t *counters_fx,
                void *stream) {
  if (!c || !in || !out) return set_error(AG_ERR_INVALID, "ag_simulate: null argument");
  if (!c->can_simulate)
    return set_error(AG_ERR_UNSUPPORTED,
                     "ag_simulate: supports P in [1,%d], E+1 in {2..9,11,13,16} and a catalogue "
                     "that fits LDS (P=%d, D=%d, N=%d, K=%d)",
                     kMaxP, c->shape.num_participants, c->D, c->shape.num_agents, c->shape.num_items);
  if (!c->catalog) return set_error(AG_ERR_STATE, "ag_simulate: ag_load_catalog not called");
  if (B < 0) return set_error(AG_ERR_INVALID, "ag_simulate: B < 0");
  if (B == 0) return AG_OK;
  if (!in->ctx || !in->part || !in->u) return set_error(AG_ERR_INVALID, "ag_simulate: null input array");
  if (B * c->shape.num_participants > INT32_MAX)
    return set_error(AG_ERR_UNSUPPORTED, "ag_simulate: B * P must be < 2^31 (32-bit SoA indexing); "
                     "split the batch");
  DeviceGuard g(c->device);
  const ag_shape &s = c->shape;
  const int nc = s.num_agents * kC;
  const int D = c->D;
  const bool prune = c->item_search == AG_ITEM_SEARCH_AUTO && D <= 8 && s.num_items <= 2 * kMaxKPairs;
  SimParams prm;
  prm.B = B;
  prm.N = s.num_agents;
  prm.K = s.num_items;
  prm.mech = s.mechanism;
  prm.want_counters = counters_fx != nullptr;
  prm.lds = make_layout(s.num_agents, s.num_items, D, prm.want_counters);
  prm.items = c->d_items;
  prm.values = c->d_values;
  prm.in = *in;
  prm.out = *out;
  prm.partials = c->d_partials;
  SimKernel k = pick_kernel(s.num_participants, D, prune);
  const size_t lds = (size_t)prm.lds.total;
  hipStream_t st = (hipStream_t)stream;
  if (lds > 64 * 1024)
    AG_HIP(hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  // Persistent grid: exactly the blocks the device keeps resident (no partial last round),
  // each striding over 256-auction tiles.
  int &res = c->resident[(prune ? 2 : 0) + (prm.want_counters ? 1 : 0)];
  if (res == 0) {
    int per_cu = 0, cus = 0;
    AG_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)k, kThreads, lds));
    AG_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device));
    res = per_cu * cus;
    if (res < 1) res = 1;
    if (res > c->partial_blocks) res = c->partial_blocks;
  }
  const int64_t tiles = (B + kThreads - 1) / kThreads;
  const int grid = (int)(tiles < res ? tiles : res);
  if (B > (int64_t)grid * kMaxAuctionsPerBlock)
    return set_error(AG_ERR_UNSUPPORTED, "ag_simulate: B=%lld > %lld auctions per call; split the batch",
                     (long long)B, (long long)grid * kMaxAuctionsPerBlock);
  hipLaunchKernelGGL(k, dim3(grid), dim3(kThreads), lds, st, prm);
  AG_HIP(hipGetLastError());
  if (counters_fx) {
    hipLaunchKernelGGL(k_reduce_counters, dim3(nc), dim3(kThreads), 0, st, c->d_partials, grid, nc,
                       counters_fx);
    AG_HIP(hipGetLastError());
  }
  return AG_OK;
}

int ag_generate(ag_ctx *c, uint64_t seed, uint64_t first, int64_t B, double *ctx_out, int32_t *part_out,
                double *u_out, void *stream) {
  if (!c || !ctx_out || !part_out || !u_out) return set_error(AG_ERR_INVALID, "ag_generate: null argument");
  if (B < 0) return set_error(AG_ERR_INVALID, "ag_generate: B < 0");
  if (B == 0) return AG_OK;
  if (c->shape.num_participants > 64) return set_error(AG_ERR_UNSUPPORTED, "ag_generate: P > 64");
  DeviceGuard g(c->device);
  const int grid = grid_for(B, (int64_t)1 << 40);
  hipLaunchKernelGGL(k_generate, dim3(grid), dim3(kThreads), 0, (hipStream_t)stream, seed, first, B,
                     c->shape.num_agents, c->shape.num_participants, c->shape.embedding_size,
                     c->shape.embedding_var, ctx_out, part_out, u_out);
  AG_HIP(hipGetLastError());
  return AG_OK;
}

int ag_counters_to_double(const int64_t *fx, int64_t n, double *out) {
  if ((!fx || !out) && n > 0) return set_error(AG_ERR_INVALID, "ag_counters_to_double: null argument");
  for (int64_t j = 0; j < n; ++j) {
    const int64_t *L = fx + j * AG_FX_LIMBS;
    __int128 t = (__int128)L[2];
    t = t * ((__int128)1 << AG_FX_LIMB_BITS) + L[1];
    t = t * ((__int128)1 << AG_FX_LIMB_BITS) + L[0];
    out[j] = ldexp((double)t, -AG_FX_FRAC_BITS);
  }
  return AG_OK;
}

int ag_sigmoid(const double *z, double *o, int64_t n, void *stream) {
  if (n <= 0) return AG_OK;
  const int grid = grid_for(n, (int64_t)1 << 40);
  hipLaunchKernelGGL(k_exp_kat, dim3(grid), dim3(kThreads), 0, (hipStream_t)stream, z, o, n, 1);
  AG_HIP(hipGetLastError());
  return AG_OK;
}

int ag_exp(const double *x, double *o, int64_t n, void *stream) {
  if (n <= 0) return AG_OK;
  const int grid = grid_for(n, (int64_t)1 << 40);
  hipLaunchKernelGGL(k_exp_kat, dim3(grid), dim3(kThreads), 0, (hipStream_t)stream, x, o, n, 0);
  AG_HIP(hipGetLastError());
  return AG_OK;
}

}  // extern "C"
