// ag_sim_pop.h -- k_pop: the simulate kernel for general populations (LR-TS allocators,
// shading and learning bidders, Oracle agents among them) of a compile-time catalogue shape,
// written for issue economy the way k_oracle is for the Oracle-only headline.
//
// Same results as k_simulate<P, D, PRUNE=true, 1, GENERAL> bit for bit (items, CTRs, bids,
// gammas, propensities, winners, prices, outcomes and the exact counter limbs;
// tests/test_gpu_parity.py runs both on every general-population case), and the same
// reference lines: src/Auction.py:28-74 per lane; the item choice of src/Agent.py:29-42 with
// OracleAllocator (src/BidderAllocation.py:81-82) or PyTorchLogisticRegressionAllocator's
// Thompson forward (src/BidderAllocation.py:67-68, src/Models.py:28-33); the bids of
// src/Bidder.py (Truthful :34-35, EmpiricalShaded :43-58, the learning bidders :171-208,
// :348-367, :455-475); {First,Second}Price.allocate (src/AuctionAllocation.py:19-34);
// Agent.charge / set_price and the metric terms (src/Agent.py:70-122).
//
// What is different from k_simulate (which stays for every other shape):
//  - K (items), D (true context + intercept) and DO (observed context + intercept) are
//    template constants (the shipped configs are all K = 12, E = 5, OE = 4: D = 6, DO = 5):
//    every catalogue / noise / table offset is an immediate, no loop-invariant offset lives
//    in a scalar register (k_simulate's runtime K / Do kept ~450 of them live and spilled
//    them into vector-register lanes: v_readlane / v_writelane in the loop);
//  - one agent's whole LDS record (catalogue, screen rows, 1/v, LR-TS means, learner model,
//    kinds, shading parameters) at one base address a * kStride, so a slot's LDS reads are
//    immediate offsets from ONE register, 16-B vector reads where rows are 16-B aligned; the
//    stride is 16 B times an odd number, so lanes reading different agents spread over banks;
//  - the Thompson screen keeps a running minimum and second minimum of t_k = (1 + 2^(-z_k
//    log2 e)) / v_k as integers carrying the item index in 4 low mantissa bits (v_min /
//    v_med3), like k_oracle's true-CTR screen; items are scored exactly only when the two
//    smallest are within the screen's margin (or a logit is out of its range): the exact
//    first argmax is then the plain loop's (ts_select's bound, ag_sim.h);
//  - per-record counter terms go to lane-private LDS replicas laid out [agent][replica][slot]
//    with an odd qword stride (every slot an immediate offset from one address), the
//    winner-independent terms as soon as a slot resolves.
#pragma once
#include "ag_sim.h"

namespace ag {

constexpr int align16c(int b) { return (b + 15) & ~15; }

// An agent's LDS record, byte offsets from its base (all 16-B aligned where read as vectors).
template <int K, int D, int DO>
struct PopRec {
  static constexpr int kPairs = (K + 1) / 2;
  static constexpr int items = 0;                              // f64 [K][D]
  static constexpr int values = items + K * D * 8;             // f64 [K]
  static constexpr int scr = align16c(values + K * 8);         // f32 [kPairs][8][2], * -log2(e)
  static constexpr int inv = scr + kPairs * 64;                // f32 [2 kPairs] 1 / v (padding +inf)
  static constexpr int tsm = align16c(inv + kPairs * 8);       // f32 [K][DO] LR-TS means
  static constexpr int drs = align16c(tsm + K * DO * 4);       // f32 [16] learner model
  static constexpr int pg = drs + 64;                          // f64 prev_gamma
  static constexpr int gs = pg + 8;                            // f64 gamma_sigma
  static constexpr int amax = gs + 8;                          // f32 max |item coefficient| * 1.001
  static constexpr int akind = amax + 4;                       // i32 allocator kind
  static constexpr int bkind = akind + 4;                      // i32 bidder kind
  static constexpr int dri = bkind + 4;                        // i32 learner state
  static constexpr int used = align16c(dri + 4);
  static constexpr int stride = (used / 16) % 2 ? used : used + 16;  // 16 B x odd
};

constexpr int kPopSlots = 10;     // counter slots (kSlotGross .. kSlotBias, ag_sim.h)
constexpr int kPopCntStride = 11;  // qwords per (agent, replica): odd
constexpr int kPopTabBytes = agexp::kExpTabLds * 8;
constexpr int kPopFlush = 255;  // auctions between flushes of the 8-bit count fields
// build knobs (A/B variants: make variant NAME=... VFLAGS=-D...)
#ifndef AG_POP_PREFETCH
#define AG_POP_PREFETCH 0  // k_pop: the next tile's inputs requested before this tile resolves
#endif
#ifndef AG_POP_LDS_BUDGET
#define AG_POP_LDS_BUDGET 40960  // LDS per 256-lane workgroup: 4 resident per CU
#endif
#ifndef AG_POP_TB_WAVES
#define AG_POP_TB_WAVES 4  // truthful-bidder populations: <= 128 VGPRs
#endif
#ifndef AG_POP_ALL_WAVES
#define AG_POP_ALL_WAVES 3  // any bidders: <= 168 VGPRs (256-lane workgroups)
#endif
#ifndef AG_POP_SLOW
#define AG_POP_SLOW 3  // 0..3: the near-tie paths (bit 0 true CTRs, bit 1 Thompson); 3 = exact
#endif
#ifndef AG_POP_SLOW_INLINE
#define AG_POP_SLOW_INLINE __forceinline__
#endif
#ifndef AG_POP_SCHED_BARRIER
#define AG_POP_SCHED_BARRIER 1
#endif
#ifndef AG_POP_NZ_PREFETCH
#define AG_POP_NZ_PREFETCH 1
#endif
#ifndef AG_POP_NZ_GROUP
#define AG_POP_NZ_GROUP 4
#endif
constexpr int kPopNzGroup = AG_POP_NZ_GROUP;  // items whose Thompson noise is loaded together

struct PopLayout {
  int32_t agents;    // byte offset of agent 0's record
  int32_t cnt;       // counter replicas [N][R][kPopCntStride] u64
  int32_t replicas;  // R (power of 2, <= 64)
  int32_t total;
};

// lds_budget: bytes of LDS per workgroup that keep the wanted workgroups resident per CU
template <int K, int D, int DO>
__host__ inline PopLayout make_pop_layout(int N, bool counters, int64_t lds_budget) {
  using R = PopRec<K, D, DO>;
  PopLayout L;
  L.agents = align16(kPopTabBytes);
  L.cnt = align16((int64_t)L.agents + (int64_t)N * R::stride);
  int rep = 64;  // one replica per wave lane while the LDS budget allows
  while (rep > 1 && (int64_t)L.cnt + (int64_t)N * rep * kPopCntStride * 8 > lds_budget) rep >>= 1;
  L.replicas = rep;
  // the counter region also holds the last workgroup's [N][AG_NUM_COUNTERS][2] sums
  int64_t cnt_bytes = (int64_t)N * rep * kPopCntStride * 8;
  if (cnt_bytes < (int64_t)N * AG_NUM_COUNTERS * 16) cnt_bytes = (int64_t)N * AG_NUM_COUNTERS * 16;
  L.total = align16((int64_t)L.cnt + (counters ? cnt_bytes : 0));
  return L;
}

struct PopParams {
  int32_t B;       // SoA leading dimension (B * P < 2^31)
  int32_t lo, hi;  // auctions [lo, hi) of this launch
  int32_t N, mech, want_counters, ts_sample;
  PopLayout L;
  const unsigned char *image;    // the LDS image of the tables and agent records (k_pop_image)
  const float *nz_zero;          // [K*DO][64] zeros (the noise of lanes that draw none)
  const uint8_t *ts_item;        // [P][B] the LR-TS choices of k_ts_choice (TSX kernels)
  ag_batch_in in;
  ag_batch_out out;
  int64_t *partials;  // [grid][N][AG_NUM_COUNTERS][2]
  int64_t *limbs;     // the caller's exact counters [N][AG_NUM_COUNTERS][3] (NULL: k_reduce_counters)
  unsigned *ticket;   // [1] zero between launches (the last workgroup resets it)
};

// ---- the LDS images of k_pop and k_ts_choice, built in global memory by k_pop_image once
// per ag_simulate (from the catalogue, kinds, shading parameters, LR-TS means and learner
// models as they are at that point of the stream) so that every workgroup's prologue is one
// 16-B copy of the bytes it needs, all loads in flight at once, instead of several passes
// over the source arrays with index arithmetic (measured: ~15 us of fixed cost per k_pop
// launch, profiles/r03e_*). Layout: [exp tables][N x PopRec] (k_pop's LDS from byte 0) then
// [exp tables][N x TsChoiceRec] (k_ts_choice's), each 16-B aligned.
template <int K, int D, int DO>
struct PopImage {
  __host__ __device__ static int64_t pop_bytes(int N) { return (int64_t)kPopTabBytes + (int64_t)N * PopRec<K, D, DO>::stride; }
  __host__ __device__ static int64_t tsc_bytes(int N);
  __host__ __device__ static int64_t total(int N) { return pop_bytes(N) + tsc_bytes(N); }
};

struct PopImageParams {
  int32_t N;
  const double *items, *values;  // [N][K][D], [N][K]
  const int32_t *akind, *bkind;  // [N]
  const double *pg, *gs;         // [N]
  const float *tsm;              // [N][K][DO] (NULL: zeros)
  const float *drs;              // [N][16] (NULL: zeros)
  const int32_t *dri;            // [N]
  unsigned char *image;          // PopImage::total(N) bytes
};

// Copy `bytes` (a multiple of 16) from global to LDS with every load of a pass in flight.
template <int BT>
__device__ __forceinline__ void lds_copy16(unsigned char *dst, const unsigned char *src, int bytes) {
  typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
  const u32x4v *g = reinterpret_cast<const u32x4v *>(src);
  u32x4v *l = reinterpret_cast<u32x4v *>(dst);
  const int n = bytes >> 4;
  constexpr int kU = 8;
  for (int base = 0; base < n; base += BT * kU) {
    u32x4v v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int j = base + u * BT + (int)threadIdx.x;
      if (j < n) v[u] = g[j];
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int j = base + u * BT + (int)threadIdx.x;
      if (j < n) l[j] = v[u];
    }
  }
}

// the logit of src/Models.py:28-33 for one item of width DO (w = m [+ noise]) in torch's CPU
// order (ts_logit_w, ag_sim.h: MKL sgemv blocks of 4 rows for DO = 5, else in order)
template <int DO>
__device__ __forceinline__ float pop_logit(const float (&w)[DO], const float (&x)[DO], int k, int K) {
  if constexpr (DO == 5) {
    const float p0 = w[0] * x[0], p2 = w[2] * x[2], p3 = w[3] * x[3], p4 = w[4] * x[4];
    if (k < (K & ~3)) return (__builtin_fmaf(w[1], x[1], p0) + p3) + (p4 + p2);
    const float p1 = w[1] * x[1];
    return p0 + ((p4 + p2) + (p3 + p1));
  } else {
    float z = w[0] * x[0];
#pragma unroll
    for (int d = 1; d < DO; ++d) z = z + w[d] * x[d];
    return z;
  }
}

// The Thompson item choice's near-tie path (rare; out of line so the hot path's registers
// are not sized for it): the exact scores of every candidate (all items when a logit is
// out of the screen's range, `bad`) in increasing k -- float32 CTR widened times the
// float64 value, first max (ts_select, ag_sim.h); logits recomputed from the means and
// the re-read noise.
template <int K, int DO>
__device__ AG_POP_SLOW_INLINE int pop_ts_slow(const float *m, const float *nz, const float (&xo)[DO],
                                                     const float *iv, const double *vv, float uthr, bool bad,
                                                     const uint64_t *tab) {
  double best_sc = 0.0;
  int tb = -1;
#pragma unroll 1
  for (int k = 0; k < K; ++k) {
    float wk[DO];
#pragma unroll
    for (int d = 0; d < DO; ++d) wk[d] = m[k * DO + d] + ldg(nz + (k * DO + d) * 64);
    const float z = pop_logit<DO>(wk, xo, k, K);
    if (!bad) {
      const float t = fmaf(__builtin_amdgcn_exp2f(z * -1.44269504f), iv[k], iv[k]);
      if (!(__uint_as_float((__float_as_uint(t) & ~15u) | (uint32_t)k) <= uthr)) continue;
    }
    const double sc = (double)ts_ctr_scalar(z, tab) * vv[k];  // K < 32: the scalar path
    if (tb < 0 || sc > best_sc) {
      best_sc = sc;
      tb = k;
    }
  }
  return tb;
}

// The Thompson item choice of one LR-TS participant (src/Agent.py:29-42, src/Models.py:28-33):
// first argmax over k of float32 sigmoid(logit_k(m + noise)) * value_k. Screened: t_k = (1 +
// 2^(-z_k log2 e)) / v_k estimates 1 / score with relative error < 2^-16 for |z| < 64
// (ts_select's bound, ag_sim.h; the 4 index bits add < 2^-19), so the exact first argmax has
// t <= t_min (1 + 2^-13); only when the two smallest t are that close (or a logit is out of
// range) are the candidates scored exactly (pop_ts_slow). m: the agent's means in LDS; nz:
// its noise rows (stride 64 floats); nzv: the noise, already in registers.
template <int K, int DO>
__device__ __forceinline__ int pop_ts_choose(const float *m, const float (&nzv)[K * DO], const float *nz,
                                             const float (&xo)[DO], const float *iv, const double *vv,
                                             const uint64_t *tab) {
  uint32_t u1 = 0xffffffffu, u2 = 0xffffffffu;
  bool bad = false;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    float wk[DO];
#pragma unroll
    for (int d = 0; d < DO; ++d) wk[d] = m[k * DO + d] + nzv[k * DO + d];
    const float z = pop_logit<DO>(wk, xo, k, K);
    bad |= !(__builtin_fabsf(z) < 64.0f);
    const float t = fmaf(__builtin_amdgcn_exp2f(z * -1.44269504f), iv[k], iv[k]);
    const uint32_t tt = (__float_as_uint(t) & ~15u) | (uint32_t)k;
    u2 = max(u1, min(u2, tt));  // the median of (u1 <= u2, tt): v_med3_u32
    u1 = min(u1, tt);
  }
  const float uthr = __uint_as_float(u1 & ~15u) * (1.0f + 0x1p-13f);
  int tb = (int)(u1 & 15u);
  if ((AG_POP_SLOW & 2) && (bad || !(__uint_as_float(u2 & ~15u) > uthr)))
    tb = pop_ts_slow<K, DO>(m, nz, xo, iv, vv, uthr, bad, tab);  // rare
  return tb;
}

// k_ts_choice: the Thompson item choice of every LR-TS participant of a batch, written as
// one byte per (slot, auction) for k_pop<..., TSX = true> (255: not an LR-TS participant).
// Split out of the simulate kernel because it is where the bytes are (the K (OE + 1) float32
// noise draws of every LR-TS participant, 480 B per SP_Truthful_TS auction) and it needs few
// registers: at high occupancy its noise loads keep HBM busy, while k_pop -- the FP64 true
// CTRs, bids, allocation and counters on 2 B of choices per auction -- keeps its registers.
template <int K, int DO>
struct TsChoiceRec {
  static constexpr int tsm = 0;                                // f32 [K][DO]
  static constexpr int inv = align16c(K * DO * 4);              // f32 [K] 1 / v
  static constexpr int values = align16c(inv + K * 4);          // f64 [K]
  static constexpr int akind = values + K * 8;                  // i32
  static constexpr int used = align16c(akind + 4);
  static constexpr int stride = (used / 16) % 2 ? used : used + 16;
};

template <int K, int D, int DO>
__host__ __device__ int64_t PopImage<K, D, DO>::tsc_bytes(int N) { return (int64_t)kPopTabBytes + (int64_t)N * TsChoiceRec<K, DO>::stride; }

// one workgroup per agent (+ the tables): the agent's PopRec and TsChoiceRec
template <int K, int D, int DO>
__global__ __launch_bounds__(256) void k_pop_image(PopImageParams prm) {
  using R = PopRec<K, D, DO>;
  using T = TsChoiceRec<K, DO>;
  constexpr int kP = R::kPairs;
  const int N = prm.N, a = blockIdx.x, tid = threadIdx.x;
  unsigned char *pop = prm.image;
  unsigned char *tsc = prm.image + PopImage<K, D, DO>::pop_bytes(N);
  if (a == N) {  // the exp tables, at the head of both images
    for (int i = tid; i < 256 + 32; i += 256) {
      const uint64_t v = i < 256 ? ag_exp_tab[i] : agexp::expf_tab_entry(ag_exp_tab, i - 256);
      reinterpret_cast<uint64_t *>(pop)[i] = v;
      reinterpret_cast<uint64_t *>(tsc)[i] = v;
    }
    return;
  }
  unsigned char *rec = pop + kPopTabBytes + (size_t)a * R::stride;
  unsigned char *trec = tsc + kPopTabBytes + (size_t)a * T::stride;
  for (int i = tid; i < R::stride / 4; i += 256) reinterpret_cast<uint32_t *>(rec)[i] = 0u;  // padding
  for (int i = tid; i < T::stride / 4; i += 256) reinterpret_cast<uint32_t *>(trec)[i] = 0u;
  __syncthreads();
  const double *itm = prm.items + (size_t)a * K * D;
  const double *val = prm.values + (size_t)a * K;
  for (int r = tid; r < K * D; r += 256) reinterpret_cast<double *>(rec + R::items)[r] = itm[r];
  for (int k = tid; k < K; k += 256) {
    reinterpret_cast<double *>(rec + R::values)[k] = val[k];
    reinterpret_cast<double *>(trec + T::values)[k] = val[k];
    reinterpret_cast<float *>(trec + T::inv)[k] = 1.0f / (float)val[k];
  }
  for (int r = tid; r < kP * 16; r += 256) {  // [pair][dim][2 items] * -log2(e)
    const int p = r >> 4, d = (r >> 1) & 7, k = 2 * p + (r & 1);
    const float c = (d < D && k < K) ? (float)itm[k * D + d] : 0.0f;
    reinterpret_cast<float *>(rec + R::scr)[r] = c * kNegLog2e;
  }
  for (int k = tid; k < kP * 2; k += 256)  // 1/v (padding items: +inf)
    reinterpret_cast<float *>(rec + R::inv)[k] = k < K ? 1.0f / (float)val[k] : INFINITY;
  for (int r = tid; r < K * DO; r += 256) {
    const float m = prm.tsm ? prm.tsm[(size_t)a * K * DO + r] : 0.0f;
    reinterpret_cast<float *>(rec + R::tsm)[r] = m;
    reinterpret_cast<float *>(trec + T::tsm)[r] = m;
  }
  for (int r = tid; r < 16; r += 256)
    reinterpret_cast<float *>(rec + R::drs)[r] = prm.drs ? prm.drs[(size_t)a * 16 + r] : 0.0f;
  if (tid == 0) {
    float m = 0.0f;
    for (int r = 0; r < K * D; ++r) m = fmaxf(m, (float)fabs(itm[r]));
    *reinterpret_cast<float *>(rec + R::amax) = m * 1.001f;
    *reinterpret_cast<double *>(rec + R::pg) = prm.pg[a];
    *reinterpret_cast<double *>(rec + R::gs) = prm.gs[a];
    *reinterpret_cast<int32_t *>(rec + R::akind) = prm.akind[a];
    *reinterpret_cast<int32_t *>(trec + T::akind) = prm.akind[a];
    *reinterpret_cast<int32_t *>(rec + R::bkind) = prm.bkind[a];
    *reinterpret_cast<int32_t *>(rec + R::dri) = prm.drs ? prm.dri[a] : AG_LEARNER_UNINITIALISED;
  }
}

struct TsChoiceParams {
  int32_t B, lo, hi, N;
  const unsigned char *image;  // its LDS image (k_pop_image: tables + N x TsChoiceRec)
  const double *ctx;      // [E][B]
  const int32_t *part;    // [P][B]
  const float *ts_noise;  // dense tiles or the compact layout (ts_noise_index)
  const int32_t *ts_noise_index;
  const float *nz_zero;   // [K*DO][64] zeros (no Thompson sampling)
  uint8_t *ts_item;       // [P][B] out
};

#ifndef AG_TSC_WAVES
#define AG_TSC_WAVES 5  // k_ts_choice: <= 96 VGPRs
#endif

template <int P, int K, int DO, int BT>
__global__ __launch_bounds__(BT, AG_TSC_WAVES) void k_ts_choice(TsChoiceParams prm) {
  using R = TsChoiceRec<K, DO>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int N = prm.N;
  const uint32_t B = (uint32_t)prm.B, lo = (uint32_t)prm.lo, hi = (uint32_t)prm.hi;
  const int tid = threadIdx.x;
  const uint64_t *tab = reinterpret_cast<const uint64_t *>(smem);
  const unsigned char *s_ag = smem + kPopTabBytes;
  lds_copy16<BT>(smem, prm.image, kPopTabBytes + N * R::stride);
  __syncthreads();
  const uint32_t T64 = (B + 63u) >> 6;
  for (uint32_t i = lo + blockIdx.x * BT + tid; i < hi; i += gridDim.x * BT) {
    float xo[DO];
#pragma unroll
    for (int d = 0; d < DO - 1; ++d) xo[d] = (float)ldg(prm.ctx + d * B + i);
    xo[DO - 1] = 1.0f;
#pragma unroll 1
    for (int s = 0; s < P; ++s) {  // one slot's noise live at a time
      const int a = ldg(prm.part + s * B + i);
      const unsigned char *rec = s_ag + a * R::stride;
      int tb = 255;
      if (*reinterpret_cast<const int32_t *>(rec + R::akind) == AG_ALLOCATOR_LRTS) {
        const float *nz = prm.nz_zero + (i & 63);
        if (prm.ts_noise) {
          if (prm.ts_noise_index) {
            const uint32_t j = (uint32_t)ldg(prm.ts_noise_index + (size_t)s * B + i);
            nz = prm.ts_noise + ((size_t)(j >> 6) * (K * DO)) * 64 + (j & 63);
          } else {
            nz = prm.ts_noise + ((size_t)(s * T64 + (i >> 6)) * (K * DO)) * 64 + (i & 63);
          }
        }
        float nzv[K * DO];
#pragma unroll
        for (int c = 0; c < K * DO; ++c) nzv[c] = ldg(nz + c * 64);
        tb = pop_ts_choose<K, DO>(reinterpret_cast<const float *>(rec + R::tsm), nzv, nz, xo,
                                  reinterpret_cast<const float *>(rec + R::inv),
                                  reinterpret_cast<const double *>(rec + R::values), tab);
      }
      stg(prm.ts_item + (size_t)s * B + i, (uint8_t)tb);
    }
  }
}

// TSX: the LR-TS participants' item choices come from k_ts_choice (prm.ts_item) instead of
// being made here from the Thompson noise.
template <int P, int D, int K, int DO, int MODE, int BT, bool TSX>
__global__ __launch_bounds__(BT, MODE == kGenTruthful ? AG_POP_TB_WAVES : AG_POP_ALL_WAVES) void k_pop(PopParams prm) {
  static_assert(D <= 8 && K <= 2 * kMaxKPairs && K <= 16 && DO <= D, "k_pop: shape out of range");
  using R = PopRec<K, D, DO>;
  constexpr int kP = R::kPairs;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int N = prm.N;
  const uint32_t B = (uint32_t)prm.B, lo = (uint32_t)prm.lo, hi = (uint32_t)prm.hi;
  const PopLayout L = prm.L;
  const uint64_t *s_tab = reinterpret_cast<const uint64_t *>(smem);
  unsigned char *s_ag = smem + L.agents;
  unsigned char *s_cnt = smem + L.cnt;
  const int tid = threadIdx.x;

  // ---- prologue: the tables and agent records (one copy of k_pop_image's bytes), counters
  lds_copy16<BT>(smem, prm.image, kPopTabBytes + N * R::stride);
  if (prm.want_counters)
    for (int i = tid; i < N * L.replicas * kPopCntStride; i += BT) reinterpret_cast<unsigned long long *>(s_cnt)[i] = 0ull;
  __syncthreads();

  const int Rn = L.replicas;
  const uint32_t cnt_agent = (uint32_t)Rn * kPopCntStride * 8;
  const uint32_t cnt_lane = (uint32_t)(tid & (Rn - 1)) * kPopCntStride * 8;
  const bool charged = P >= 2;  // P == 1: nobody charged (src/Auction.py:68)
  const bool fp = prm.mech == AG_FIRST_PRICE;
  const bool sample = prm.ts_sample != 0;
  const bool packed = N <= 8;  // participation counts in 8-bit register fields
  uint64_t n_logs_packed = 0, n_won_packed = 0;
  int since_flush = 0;
  auto cadd = [&](uint32_t addr, int slot, unsigned long long v) {
    atomicAdd(reinterpret_cast<unsigned long long *>(s_cnt + addr + slot * 8), v);
  };
  auto cadd_nz = [&](uint32_t addr, int slot, unsigned long long v) {
    if (v != 0ull) cadd(addr, slot, v);
  };
  auto flush_counts = [&]() {
    for (int a = 0; a < N; ++a) {
      const uint64_t v = ((n_logs_packed >> (8 * a)) & 255ull) | (((n_won_packed >> (8 * a)) & 255ull) << 32);
      if (v) cadd((uint32_t)a * cnt_agent + cnt_lane, kSlotCounts, (unsigned long long)v);
    }
    n_logs_packed = 0;
    n_won_packed = 0;
    since_flush = 0;
  };
  const ag_batch_in &in = prm.in;
  const ag_batch_out &out = prm.out;
  const uint32_t T64 = (B + 63u) >> 6;
  const uint32_t stride = gridDim.x * BT;

  // the next tile's inputs are in flight while this tile resolves (AG_POP_PREFETCH; a lane
  // resolves only a few tiles per launch at the populations' batch sizes, so the first load's
  // latency is every tile's unless the next one is requested early)
  double xn[D - 1], un = 0.0;
  int an[P], tn[P];
  auto load_in = [&](uint32_t j) {
#pragma unroll
    for (int e = 0; e < D - 1; ++e) xn[e] = ldg(in.ctx + e * B + j);
#pragma unroll
    for (int s = 0; s < P; ++s) an[s] = ldg(in.part + s * B + j);
    un = ldg(in.u + j);
#pragma unroll
    for (int s = 0; s < P; ++s) tn[s] = TSX ? (int)ldg(prm.ts_item + (size_t)s * B + j) : 0;
  };
  constexpr bool kPre = AG_POP_PREFETCH && TSX;  // the fused kernels have no registers to spare
  if (kPre && lo + blockIdx.x * BT + tid < hi) load_in(lo + blockIdx.x * BT + tid);
#pragma unroll 1
  for (uint32_t i = lo + blockIdx.x * BT + tid; i < hi; i += stride) {
    double x[kMaxD];
    float xf[kMaxD];
    float xabs = 1.0f;
    int ag[P], tsi[P];
    if (!kPre) load_in(i);
#pragma unroll
    for (int e = 0; e < D - 1; ++e) x[e] = xn[e];
#pragma unroll
    for (int s = 0; s < P; ++s) {
      ag[s] = an[s];
      tsi[s] = tn[s];
    }
    const double u = un;
    if (kPre) load_in(i + stride < hi ? i + stride : i);  // branch-free: the last tile re-reads its own
#pragma unroll
    for (int e = 0; e < D - 1; ++e) {
      xf[e] = (float)x[e];
      xabs += fabsf(xf[e]);
    }
    x[D - 1] = 1.0;  // intercept (src/Auction.py:33)
    xf[D - 1] = 1.0f;
    xabs *= 1.001f;
    float xo[DO];  // observed context + intercept (src/Auction.py:36) as torch.Tensor rounds it
#pragma unroll
    for (int d = 0; d < DO; ++d) xo[d] = d < DO - 1 ? xf[d] : 1.0f;

    double m1 = 0.0, m2 = -INFINITY, ctr_w = 0.0;
    int w = 0;
    double bidv[P], valv[P], tvv[P], ratv[P];
#pragma unroll
    for (int s = 0; s < P; ++s) {
      const int a = ag[s];
      const unsigned char *rec = s_ag + a * R::stride;
      const double *itm = reinterpret_cast<const double *>(rec + R::items);
      const double *vv = reinterpret_cast<const double *>(rec + R::values);
      const float *scr = reinterpret_cast<const float *>(rec + R::scr);
      const float *iv = reinterpret_cast<const float *>(rec + R::inv);
      const int akind = *reinterpret_cast<const int32_t *>(rec + R::akind);
      const bool lrts = akind == AG_ALLOCATOR_LRTS;
      // Thompson noise of this participant (src/Models.py:31), tiled by 64 auctions
      // (nz_zero: K*DO rows of 64 zeros, L2-resident, for lanes without noise -- the loads and
      // adds run unconditionally; m + 0.0f == m up to the sign of a zero, which no logit's
      // sigmoid sees)
      constexpr int kG = kPopNzGroup;
      const float *nz = prm.nz_zero + (i & 63);
      float nzv[2][kG * DO];
      if constexpr (!TSX) {
        if (lrts && sample) {
          if (in.ts_noise_index) {
            const uint32_t j = (uint32_t)ldg(in.ts_noise_index + (size_t)s * B + i);
            nz = in.ts_noise + ((size_t)(j >> 6) * (K * DO)) * 64 + (j & 63);
          } else {
            nz = in.ts_noise + ((size_t)(s * T64 + (i >> 6)) * (K * DO)) * 64 + (i & 63);
          }
        }
        // the noise of the first kG items is in flight during the true-CTR search
#pragma unroll
        for (int c = 0; c < kG * DO; ++c) nzv[0][c] = ldg(nz + c * 64);
      }

      // ---- true CTRs (src/Auction.py:52-53): max_k CTR_k * value_k exactly; for an
      // Oracle agent this IS its item choice (f32 screen + exact FP64 leader, k_oracle's)
      uint32_t t1 = 0xffffffffu, t2 = 0xffffffffu;
#pragma unroll
      for (int p = 0; p < kP; ++p) {
        const float *r = scr + p * 16;
        f32x2 z = *reinterpret_cast<const f32x2 *>(r + 2 * (D - 1));  // intercept: x_{D-1} == 1
#pragma unroll
        for (int d = 0; d < D - 1; ++d) {
          const f32x2 c = *reinterpret_cast<const f32x2 *>(r + 2 * d);
          const f32x2 xd = {xf[d], xf[d]};
          z = __builtin_elementwise_fma(c, xd, z);
        }
        const f32x2 e = {__builtin_amdgcn_exp2f(z.x), __builtin_amdgcn_exp2f(z.y)};
        const f32x2 ivp = *reinterpret_cast<const f32x2 *>(iv + 2 * p);
        const f32x2 t = __builtin_elementwise_fma(e, ivp, ivp);
        const uint32_t ta = (__float_as_uint(t.x) & ~15u) | (uint32_t)(2 * p);
        const uint32_t tb = (__float_as_uint(t.y) & ~15u) | (uint32_t)(2 * p + 1);
        const uint32_t l = min(ta, tb), h = max(ta, tb);
        t2 = min(min(max(t1, l), t2), h);
        t1 = min(t1, l);
      }
      const float amax = *reinterpret_cast<const float *>(rec + R::amax);
      const bool ok = (amax * xabs <= kPruneMaxS) && (__uint_as_float(t1 & ~15u) <= 1e30f);
      const float thr = __uint_as_float(t1 & ~15u) * (1.0f + kPruneDelta);
      int lead = (int)(t1 & 15u);
      double c = agexp::sigmoid_fast(dot_ref<D>(itm + lead * D, x), s_tab);
      double bev = c * vv[lead];
      if ((AG_POP_SLOW & 1) && (!ok || !(__uint_as_float(t2 & ~15u) > thr))) {
        // near-tie (rare) or unscreenable lane: every item under the threshold, exactly, in
        // increasing k (first maximum, src/Agent.py:35)
        const int kf = lead;
        const double c_kf = c;
        lead = -1;
        for (int k = 0; k < K; ++k) {
          if (ok && k != kf) {
            const float *r = scr + (k >> 1) * 16 + (k & 1);
            float z = r[2 * (D - 1)];
#pragma unroll
            for (int d = 0; d < D - 1; ++d) z = fmaf(r[2 * d], xf[d], z);
            const float t = fmaf(__builtin_amdgcn_exp2f(z), iv[k], iv[k]);
            if (!(__uint_as_float((__float_as_uint(t) & ~15u) | (uint32_t)k) <= thr)) continue;
          }
          const double ck = k == kf ? c_kf : agexp::sigmoid_fast(dot_ref<D>(itm + k * D, x), s_tab);
          const double sk = ck * vv[k];
          if (lead < 0 || sk > bev) {
            lead = k;
            bev = sk;
            c = ck;
          }
        }
      }
      int item = lead;
      double est = c, tru = c;

      if (lrts) {
        // ---- LR-TS (src/Agent.py:29-42): the sampled CTRs on the observed context pick the
        // item (first argmax of float32 CTR * value), the MAP CTR of that item is the estimate
        const float *m = reinterpret_cast<const float *>(rec + R::tsm);
        int tb;
        if constexpr (TSX) {
          tb = tsi[s];
        } else {
        uint32_t u1 = 0xffffffffu, u2 = 0xffffffffu;
        bool bad = false;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const int g = k / kG, kg = k % kG;
          if (AG_POP_SCHED_BARRIER && kg == 0) __builtin_amdgcn_sched_barrier(0);  // one group at a time
          if (AG_POP_NZ_PREFETCH && kg == 0 && k + kG < K) {  // the next group's noise, in flight while this one is scored
#pragma unroll
            for (int c = 0; c < kG * DO; ++c)
              nzv[(g + 1) & 1][c] = (k + kG) * DO + c < K * DO ? ldg(nz + ((k + kG) * DO + c) * 64) : 0.0f;
          }
          if (!AG_POP_NZ_PREFETCH && kg == 0 && k > 0) {  // this group's noise
#pragma unroll
            for (int c = 0; c < kG * DO; ++c)
              nzv[0][c] = k * DO + c < K * DO ? ldg(nz + (k * DO + c) * 64) : 0.0f;
          }
          float wk[DO];
#pragma unroll
          for (int d = 0; d < DO; ++d) wk[d] = m[k * DO + d] + nzv[AG_POP_NZ_PREFETCH ? g & 1 : 0][kg * DO + d];
          const float z = pop_logit<DO>(wk, xo, k, K);
          bad |= !(__builtin_fabsf(z) < 64.0f);
          // score estimate t_k = (1 + 2^(-z log2 e)) / v_k = 1 / (sigmoid(z) v_k), relative
          // error < 2^-16 for |z| < 64 (ts_select's bound, ag_sim.h; the 4 index bits add
          // < 2^-19): the exact first argmax has t <= t_min (1 + 2^-13)
          const float t = fmaf(__builtin_amdgcn_exp2f(z * -1.44269504f), iv[k], iv[k]);
          const uint32_t tt = (__float_as_uint(t) & ~15u) | (uint32_t)k;
          u2 = max(u1, min(u2, tt));  // the median of (u1 <= u2, tt): v_med3_u32
          u1 = min(u1, tt);
        }
        const float uthr = __uint_as_float(u1 & ~15u) * (1.0f + 0x1p-13f);
        tb = (int)(u1 & 15u);
        if ((AG_POP_SLOW & 2) && (bad || !(__uint_as_float(u2 & ~15u) > uthr)))
          tb = pop_ts_slow<K, DO>(m, nz, xo, iv, vv, uthr, bad, s_tab);  // rare
        }
        // MAP CTR of the chosen item (src/Agent.py:40-41, sample=False)
        float wm[DO];
#pragma unroll
        for (int d = 0; d < DO; ++d) wm[d] = m[tb * DO + d];
        est = (double)ts_ctr_scalar(pop_logit<DO>(wm, xo, tb, K), s_tab);
        tru = tb == lead ? c : agexp::sigmoid_fast(dot_ref<D>(itm + tb * D, x), s_tab);
        item = tb;
      }
      const double v = vv[item];
      double b = v * est;  // Bidder.bid: value * estimated CTR (src/Bidder.py:35, :49, :173, ...)
      double g = NAN, prop = NAN;
      if constexpr (MODE == kGenAll) {  // kGenTruthful: every bidder is a TruthfulBidder
        const int bk = *reinterpret_cast<const int32_t *>(rec + R::bkind);
        const int di = *reinterpret_cast<const int32_t *>(rec + R::dri);
        const float *drs = reinterpret_cast<const float *>(rec + R::drs);
        if (bk >= AG_BIDDER_VALUE_LEARNING && di == AG_LEARNER_POLICY) {  // the fitted policy
          policy_bid(drs + 4, est, v, ldg(in.policy_eps + (size_t)s * B + i), s_tab, g, prop);
          b = b * g;
        } else if (bk == AG_BIDDER_VALUE_LEARNING && di == AG_LEARNER_SEARCH) {
          g = search_gamma(drs, est, v, in.gamma_grid + (size_t)s * 128 * B + i, B, s_tab);
          prop = 1.0;  // src/Bidder.py:196
          b = b * g;
        } else if (bk != AG_BIDDER_TRUTHFUL) {
          g = ldg(in.gamma_raw + (size_t)s * B + i);
          if (bk == AG_BIDDER_EMPIRICAL_SHADED) {  // clipped to [0, 1] (src/Bidder.py:52-55)
            if (g < 0.0) g = 0.0;
            if (g > 1.0) g = 1.0;
          } else {
            prop = shading_propensity(*reinterpret_cast<const double *>(rec + R::pg),
                                      *reinterpret_cast<const double *>(rec + R::gs), g, s_tab);
          }
          b = b * g;  // bid *= gamma
        }
      }
      // this slot's log columns (src/Auction.py:44-53) and its winner-independent terms
      const uint32_t o = s * B + i;
      if (out.item) stg(out.item + o, (int32_t)item);
      if (out.bid) stg(out.bid + o, b);
      if (out.est_ctr) stg(out.est_ctr + o, est);
      if (out.true_ctr) stg(out.true_ctr + o, tru);
      if (out.best_ev) stg(out.best_ev + o, bev);
      if constexpr (MODE == kGenAll) {
        if (out.gamma) stg(out.gamma + o, g);
        if (out.propensity) stg(out.propensity + o, prop);
      }
      const double tv = tru * v;
      if (prm.want_counters) {  // src/Agent.py:96-122 terms (count_pre, ag_sim.h)
        const uint32_t addr = (uint32_t)a * cnt_agent + cnt_lane;
        cadd(addr, kSlotBestEv, to_fx(bev));
        cadd_nz(addr, kSlotAlloc, to_fx(bev - tv));
        cadd_nz(addr, kSlotEst, to_fx(est * v - tv));
        const double dd = tru - est;
        cadd_nz(addr, kSlotSqerr, to_fx(dd * dd));
      }
      bidv[s] = b;
      valv[s] = v;
      tvv[s] = tv;
      ratv[s] = est / tru;
      // streaming top-2, ties -> lowest slot (src/AuctionAllocation.py:19-34)
      top2_step(s, b, m1, m2, w);
      if (w == s) ctr_w = tru;  // the current leader's true CTR
    }
    const double price = fp ? m1 : m2;
    const int oc = bernoulli(ctr_w, u);  // src/Auction.py:65
    if (out.winner) stg(out.winner + i, (int32_t)w);
    if (out.price) stg(out.price + i, charged ? price : (double)NAN);
    if (out.second_price) stg(out.second_price + i, charged ? m2 : (double)NAN);
    if (out.outcome) stg(out.outcome + i, (uint8_t)oc);
    if (prm.want_counters) {  // the winner-dependent terms (count_post, ag_sim.h)
      const double lp = charged ? price : 0.0;
#pragma unroll
      for (int s = 0; s < P; ++s) {
        const int a = ag[s];
        const uint32_t addr = (uint32_t)a * cnt_agent + cnt_lane;
        const bool won = charged && s == w;
        if (won) {
          cadd_nz(addr, kSlotGross, to_fx(valv[s] * (double)oc));
          cadd(addr, kSlotPaid, to_fx(price));
          if (fp) cadd_nz(addr, kSlotOverbid, to_fx(lp - m2));
          cadd(addr, kSlotBias, to_fx(ratv[s]));
        } else {
          cadd_nz(addr, kSlotUnderbid, to_fx((lp - bidv[s]) * (double)(lp < tvv[s])));
        }
        if (packed) {
          const uint64_t bit = 1ull << (8 * a);
          n_logs_packed += bit;
          if (won) n_won_packed += bit;
        } else {
          cadd(addr, kSlotCounts, won ? 0x100000001ull : 1ull);
        }
      }
      if (packed && ++since_flush == kPopFlush) flush_counts();
    }
  }

  if (!prm.want_counters) return;
  if (packed) flush_counts();
  __syncthreads();
  // per (agent, slot) pair, one thread each: its replicas summed as two limbs (value = lo +
  // hi * 2^42; counts: logs in lo, wins in hi), written over the pair's replica-0 / -1 words
  // (the replicas' loads pipelined 8 at a time: with one thread per agent looping over every
  // slot and replica this epilogue was ~15 us of every launch, profiles/r03f_*); then the
  // block's partials in k_simulate's format
  unsigned long long *cnt = reinterpret_cast<unsigned long long *>(s_cnt);
  auto split = [&](int j, unsigned long long v, long long &l, long long &h) {
    if (j == kSlotCounts) {
      l = (long long)(v & 0xffffffffull);
      h = (long long)(v >> 32);
    } else {
      l = (long long)v & kLimbMask;
      h = (long long)v >> AG_FX_LIMB_BITS;
    }
  };
  if (Rn >= 2) {
    for (int pr = tid; pr < N * kPopSlots; pr += BT) {
      const int a = pr / kPopSlots, j = pr - a * kPopSlots;
      const unsigned long long *c0 = cnt + (size_t)a * Rn * kPopCntStride + j;
      long long sl = 0, sh = 0;
      for (int r0 = 0; r0 < Rn; r0 += 8) {
        unsigned long long v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = r0 + u < Rn ? c0[(size_t)(r0 + u) * kPopCntStride] : 0ull;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          long long l, h;
          split(j, v[u], l, h);
          sl += l;
          sh += h;
        }
      }
      cnt[(size_t)a * Rn * kPopCntStride + j] = (unsigned long long)sl;
      cnt[((size_t)a * Rn + 1) * kPopCntStride + j] = (unsigned long long)sh;
    }
    __syncthreads();
  }
  for (int a = tid; a < N; a += BT) {
    long long lo_[kPopSlots], hi_[kPopSlots];
#pragma unroll
    for (int j = 0; j < kPopSlots; ++j) {
      if (Rn >= 2) {
        lo_[j] = (long long)cnt[(size_t)a * Rn * kPopCntStride + j];
        hi_[j] = (long long)cnt[((size_t)a * Rn + 1) * kPopCntStride + j];
      } else {
        split(j, cnt[(size_t)a * kPopCntStride + j], lo_[j], hi_[j]);
      }
    }
    int64_t *dst = prm.partials + ((size_t)blockIdx.x * N + a) * kC * 2;
    auto put = [&](int c, long long l, long long h) {
      dst[2 * c] = l;
      dst[2 * c + 1] = h;
    };
    auto put_count = [&](int c, unsigned long long n) {
      put(c, (long long)((n & 63ull) << AG_FX_FRAC_BITS), (long long)(n >> 6));
    };
    put(AG_C_NET, lo_[kSlotGross] - lo_[kSlotPaid], hi_[kSlotGross] - hi_[kSlotPaid]);
    put(AG_C_GROSS, lo_[kSlotGross], hi_[kSlotGross]);
    put(AG_C_ALLOC_REGRET, lo_[kSlotAlloc], hi_[kSlotAlloc]);
    put(AG_C_EST_REGRET, lo_[kSlotEst], hi_[kSlotEst]);
    put(AG_C_OVERBID, lo_[kSlotOverbid], hi_[kSlotOverbid]);
    put(AG_C_UNDERBID, lo_[kSlotUnderbid], hi_[kSlotUnderbid]);
    put(AG_C_CTR_SQERR, lo_[kSlotSqerr], hi_[kSlotSqerr]);
    put(AG_C_CTR_BIAS, lo_[kSlotBias], hi_[kSlotBias]);
    put(AG_C_BEST_EV, lo_[kSlotBestEv], hi_[kSlotBestEv]);
    put_count(AG_C_N_LOGS, (unsigned long long)lo_[kSlotCounts]);
    put_count(AG_C_N_WON, (unsigned long long)hi_[kSlotCounts]);
    put(AG_C_PAID, lo_[kSlotPaid], hi_[kSlotPaid]);
  }
  if (!prm.limbs) return;  // k_reduce_counters sums the partials
  // The last workgroup to finish sums every workgroup's partials into the exact limbs
  // (k_reduce_counters' arithmetic, without its launch): stores released at agent scope, a
  // ticket taken with an acq_rel RMW, the last taker acquires and reads them all.
  __threadfence();
  __syncthreads();
  __shared__ int s_last;
  if (tid == 0) {
    const unsigned t = __hip_atomic_fetch_add(prm.ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    s_last = t == gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  const int NC = N * kC, G = gridDim.x;
  const int nsub = BT / NC > 1 ? BT / NC : 1;
  long long *acc = reinterpret_cast<long long *>(s_cnt);  // [NC][2], the replicas are done
  for (int j = tid; j < 2 * NC; j += BT) acc[j] = 0;
  __syncthreads();
  for (int wk = tid; wk < NC * nsub; wk += BT) {
    const int j = wk % NC, sub = wk / NC;
    long long a0 = 0, a1 = 0;
    for (int b0 = sub; b0 < G; b0 += 8 * nsub) {
      long long v0[8], v1[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int b = b0 + u * nsub;
        v0[u] = b < G ? prm.partials[((size_t)b * NC + j) * 2] : 0;
        v1[u] = b < G ? prm.partials[((size_t)b * NC + j) * 2 + 1] : 0;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        a0 += v0[u];
        a1 += v1[u];
      }
    }
    atomicAdd(reinterpret_cast<unsigned long long *>(acc + 2 * j), (unsigned long long)a0);
    atomicAdd(reinterpret_cast<unsigned long long *>(acc + 2 * j + 1), (unsigned long long)a1);
  }
  __syncthreads();
  for (int j = tid; j < NC; j += BT) {
    int64_t *Lm = prm.limbs + (size_t)j * AG_FX_LIMBS;
    long long l0 = Lm[0] + acc[2 * j], l1 = Lm[1] + acc[2 * j + 1], l2 = Lm[2];
    long long c = l0 >> AG_FX_LIMB_BITS;
    l0 &= kLimbMask;
    l1 += c;
    c = l1 >> AG_FX_LIMB_BITS;
    l1 &= kLimbMask;
    l2 += c;
    Lm[0] = l0;
    Lm[1] = l1;
    Lm[2] = l2;
  }
  if (tid == 0) __hip_atomic_store(prm.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

typedef void (*PopKernel)(PopParams);

typedef void (*TsChoiceKernel)(TsChoiceParams);
typedef void (*PopImageKernel)(PopImageParams);

// Defined per P in ag_sim_p.hip: k_pop<P, 6, 12, 5, mode, bt, tsx> and k_ts_choice<P, 12, 5>
// (the shipped catalogue shape; nullptr for any other shape: k_simulate runs those).
template <int P>
PopKernel pick_pop_for(int D, int K, int DO, int mode, int bt, bool tsx);
template <int P>
TsChoiceKernel pick_ts_choice_for(int K, int DO);
template <> PopKernel pick_pop_for<1>(int, int, int, int, int, bool);
template <> TsChoiceKernel pick_ts_choice_for<1>(int, int);
template <> PopKernel pick_pop_for<2>(int, int, int, int, int, bool);
template <> TsChoiceKernel pick_ts_choice_for<2>(int, int);
template <> PopKernel pick_pop_for<3>(int, int, int, int, int, bool);
template <> TsChoiceKernel pick_ts_choice_for<3>(int, int);
template <> PopKernel pick_pop_for<4>(int, int, int, int, int, bool);
template <> TsChoiceKernel pick_ts_choice_for<4>(int, int);
template <> PopKernel pick_pop_for<5>(int, int, int, int, int, bool);
template <> TsChoiceKernel pick_ts_choice_for<5>(int, int);
template <> PopKernel pick_pop_for<6>(int, int, int, int, int, bool);
template <> TsChoiceKernel pick_ts_choice_for<6>(int, int);
template <> PopKernel pick_pop_for<7>(int, int, int, int, int, bool);
template <> TsChoiceKernel pick_ts_choice_for<7>(int, int);
template <> PopKernel pick_pop_for<8>(int, int, int, int, int, bool);
template <> TsChoiceKernel pick_ts_choice_for<8>(int, int);

}  // namespace ag
