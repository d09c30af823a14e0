// ag_sim_oracle.h -- k_oracle: the simulate kernel for OracleAllocator + TruthfulBidder
// populations (the north-star SP_Oracle workload), written for issue economy.
//
// Same results as k_simulate<P, D, PRUNE=true, 1, GENERAL=false> bit for bit (items, CTRs,
// bids, winners, prices, outcomes and the exact counter limbs; tests/test_gpu_parity.py
// runs both), and the same reference lines: src/Auction.py:28-74 per lane, the item choice
// of src/Agent.py:29-42 with OracleAllocator.estimate_CTR (src/BidderAllocation.py:81-82),
// TruthfulBidder.bid (src/Bidder.py:34-35), {First,Second}Price.allocate
// (src/AuctionAllocation.py:19-34), Agent.charge / set_price (src/Agent.py:70-77).
//
// What is different from k_simulate (which stays for general populations and for
// catalogues outside the bounds below):
//  - the f32 screen keeps its running minimum and second minimum of t_k = (1 + 2^z'_k)/v_k
//    as integers whose 4 low mantissa bits hold the item index (t > 0, so float order ==
//    integer order): v_min3/v_max per item pair instead of compare/select chains, and no
//    array of per-item scores;
//  - the catalogue's intercept column seeds the screen's dot (x_D-1 == 1);
//  - per-record counter terms are added to LDS columns laid out [agent][replica][slot]
//    with one lane-private replica per wave lane (64), so every slot is an immediate offset
//    from one per-record address and no two lanes of a wave hit the same qword;
//  - terms that are identically zero for Oracle + Truthful agents are not formed at all:
//    the loser's underbid term when P >= 2 (a truthful bid IS the true value, and every
//    loser's bid is <= the price under both mechanisms) and all estimation terms;
//  - fixed-point rounding is branch-free: the host admits a catalogue only when every value
//    is in (0, kOraMaxValue), which bounds every term (and every replica sum) in range;
//  - kernel arguments are only the arrays this path touches (no SGPR spills).
#pragma once
#include "ag_philox.h"
#include "ag_sim.h"

namespace ag {

// Slot 1 is PAID when P >= 2 and UNDERBID when P == 1 (nobody is charged, so no price is
// paid, and the log's price stays 0: the underbid term is -bid, src/Agent.py:107-110).
constexpr int kOraSlotGross = 0, kOraSlotPaid = 1, kOraSlotUnderbid1 = 1, kOraSlotOverbid = 2,
              kOraSlotBestEv = 3, kOraSlotCounts = 4;  // counts only when N > 8 (else registers)
constexpr int kOraStride = 5;      // qwords per (agent, replica): odd -> lanes spread over banks
// Catalogue values must lie in (0, kOraMaxValue): then every counter term is < 2^10 (bids,
// prices, best EVs and clicked values are <= max value) and its fixed-point image < 2^46.
// A replica column is shared by 256 / R lanes, each adding at most one term per slot per
// auction, so with at most ora_lane_cap(R) = 512 R auctions per lane per launch a replica
// sums fewer than 2^17 terms: |sum| < 2^63, no int64 overflow. Participation counts are
// 8-bit fields in registers, flushed to LDS every kOraFlush auctions.
constexpr double kOraMaxValue = 1024.0;
#ifndef AG_ORA_PREFETCH
#define AG_ORA_PREFETCH 0  // software-pipelined input loads (A/B: make variant VFLAGS=-DAG_ORA_PREFETCH=1)
#endif
#ifndef AG_ORA_QUEUE
// Waves take 512-auction chunks from 64 work counters (1) instead of the static grid stride
// (0): the chunks in flight stay a narrow address window however the persistent blocks drift,
// which is what the byte pattern's floor rewards (tools/floor: 3.64 ms persistent, 3.50 with
// work counters). 3.87 -> 3.73 ms per 2^27 auctions, outputs identical
// (profiles/r05zk_ab_wq.log); block-level claims with a barrier (4.20 ms) and per-wave
// 64-auction claims (5.24 ms: same-address atomics serialise) lost (r05zg_ab_queue.log)
#define AG_ORA_QUEUE 1
#endif
#ifndef AG_ORA_QUEUE_SUB
#define AG_ORA_QUEUE_SUB 8  // 64-auction tiles per claimed chunk (2 / 4 / 8: 3.46 / 3.41 / 3.38 ms at 5 per CU, r05zm_ab_sub_bpc.log; 8 / 16 / 32: 3.33 / 3.36 / 3.43 ms on another box, r05zn_ab_sub16.log)
#endif
#if AG_ORA_QUEUE && AG_ORA_PREFETCH
#error "AG_ORA_QUEUE and AG_ORA_PREFETCH are exclusive"
#endif
#ifndef AG_ORA_STORE_LATE
#define AG_ORA_STORE_LATE 1  // every per-slot output stored after the slots, field by field (A/B: 0 stores each slot's as it resolves; 3.73 -> 3.59 ms per 2^27, profiles/r05h_ab_packed.log)
#endif
constexpr int kOraFlush = 255;
// default persistent grid (ag_kernels.hip simulate_oracle): as many workgroups as fit (5 per CU
// at 85 VGPRs). With the static stride 4 streamed better than 5 (the blocks drift apart); with
// the work counters 5 per CU is 4.7 % faster than 4 (profiles/r05zm_ab_sub_bpc.log)
constexpr int kOraBlocksPerCu = 8;
__host__ inline int64_t ora_lane_cap(int R) { return 512 * (int64_t)R; }

struct OraLayout {
  int32_t tab, items, values, scr, scr_val, amax, cnt, total;
  int32_t items_stride, values_stride, scr_stride, scr_val_stride, kpairs, replicas;
};

__host__ inline OraLayout make_ora_layout(int N, int K, int D, bool counters) {
  OraLayout L;
  L.items_stride = (K * D) | 1;
  L.values_stride = K | 1;
  L.kpairs = (K + 1) / 2;
  L.scr_stride = L.kpairs * 16 + 4;
  L.scr_val_stride = L.kpairs * 2 + 2;
  int R = 64;  // one replica per wave lane, fewer when N is large (LDS budget 40 KiB)
  while (R > 1 && (int64_t)N * R * kOraStride * 8 > 40960) R >>= 1;
  L.replicas = R;
  int64_t b = 256 * 8;
  L.tab = 0;
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
  b = L.cnt + (counters ? (int64_t)N * R * kOraStride * 8 : 0);
  L.total = align16(b);
  return L;
}

struct OraParams {
  int32_t B;       // SoA leading dimension (B * P < 2^31)
  int32_t lo, hi;  // auctions [lo, hi) of this launch
  int32_t N, K, mech, want_counters;
  OraLayout L;
  const double *items, *values;  // global catalogue [N][K][D], [N][K]
  const double *ctx;             // [D-1][B]
  const int32_t *part;           // [P][B]
  const double *u;               // [B]
  int32_t *winner;
  double *price, *second_price;
  uint8_t *outcome;
  int32_t *item;
  double *bid, *est_ctr, *true_ctr, *best_ev;
  uint32_t *winner_outcome;  // ABI 17: [B] winner | outcome << 31
  int64_t *partials;  // [grid][N][AG_NUM_COUNTERS][2]
  uint32_t *queue;      // AG_ORA_QUEUE: 64 chunk counters, 32 words apart, zero at launch
  uint32_t lane_tiles;  // AG_ORA_QUEUE: auctions one lane may take per launch
  // generate mode (GEN): inputs drawn on the chip as ag_generate draws them
  uint64_t seed, first;  // Philox key; global index of auction 0 of the batch
  double scale;          // embedding_var
};

// Branch-free x * 2^36 rounded to nearest-even for |x| < 2^14 (kOraMaxValue bounds it).
__device__ __forceinline__ unsigned long long ora_fx(double x) {
  const double y = fma(x, kFxScale, kMagic);
  return (unsigned long long)(__double_as_longlong(y) - __double_as_longlong(kMagic));
}

// Item screen of one agent: the running (min, second min) of t_k with the item index in
// the 4 low bits (items 2p, 2p+1 per step; padding items have t = +inf or NaN, which sort
// above every real item).
template <int D>
__device__ __forceinline__ void ora_screen(const float *__restrict__ row, const float *__restrict__ sv, int kpairs,
                                           const float (&xf)[kMaxD], uint32_t &m1, uint32_t &m2) {
  m1 = 0xffffffffu;
  m2 = 0xffffffffu;
  for (int p = 0; p < kpairs; ++p) {
    const float *r = row + p * 16;
    f32x2 z = *reinterpret_cast<const f32x2 *>(r + 2 * (D - 1));  // intercept: x_{D-1} == 1
#pragma unroll
    for (int d = 0; d < D - 1; ++d) {
      const f32x2 a = *reinterpret_cast<const f32x2 *>(r + 2 * d);
      const f32x2 xd = {xf[d], xf[d]};
      z = __builtin_elementwise_fma(a, xd, z);
    }
    const f32x2 e = {__builtin_amdgcn_exp2f(z.x), __builtin_amdgcn_exp2f(z.y)};
    const f32x2 iv = *reinterpret_cast<const f32x2 *>(sv + 2 * p);
    const f32x2 t = __builtin_elementwise_fma(e, iv, iv);
    const uint32_t ta = (__float_as_uint(t.x) & ~15u) | (uint32_t)(2 * p);
    const uint32_t tb = (__float_as_uint(t.y) & ~15u) | (uint32_t)(2 * p + 1);
    const uint32_t lo = min(ta, tb), hi = max(ta, tb);
    m2 = min(min(max(m1, lo), m2), hi);
    m1 = min(m1, lo);
  }
}

// t'_k of one item exactly as ora_screen computes it (slow path only).
template <int D>
__device__ __forceinline__ uint32_t ora_screen_one(const float *__restrict__ row, const float *__restrict__ sv,
                                                   int k, const float (&xf)[kMaxD]) {
  const float *r = row + (k >> 1) * 16 + (k & 1);
  float z = r[2 * (D - 1)];
#pragma unroll
  for (int d = 0; d < D - 1; ++d) z = fmaf(r[2 * d], xf[d], z);
  const float e = __builtin_amdgcn_exp2f(z);
  const float iv = sv[k];
  const float t = fmaf(e, iv, iv);
  return (__float_as_uint(t) & ~15u) | (uint32_t)k;
}

// GEN = false: inputs read from HBM (replay / the HBM-resident synthetic batches).
// GEN = true: inputs drawn in the kernel by gen_auction (ag_philox.h), the same bits as
// ag_generate writes; nothing is read from HBM but the catalogue.
template <int P, int D, bool GEN>
__global__ __launch_bounds__(kThreads) void k_oracle(OraParams prm) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int N = prm.N, K = prm.K;
  const uint32_t B = (uint32_t)prm.B, lo = (uint32_t)prm.lo, hi = (uint32_t)prm.hi;
  const OraLayout L = prm.L;
  uint64_t *s_tab = reinterpret_cast<uint64_t *>(smem + L.tab);
  double *s_items = reinterpret_cast<double *>(smem + L.items);
  double *s_vals = reinterpret_cast<double *>(smem + L.values);
  float *s_scr = reinterpret_cast<float *>(smem + L.scr);
  float *s_scr_val = reinterpret_cast<float *>(smem + L.scr_val);
  float *s_amax = reinterpret_cast<float *>(smem + L.amax);
  unsigned char *s_cnt = smem + L.cnt;

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
  for (int i = tid; i < N * L.kpairs * 16; i += kThreads) {  // [pair][dim][2 items] * -log2(e)
    const int a = i / (L.kpairs * 16), r = i - a * (L.kpairs * 16);
    const int p = r >> 4, d = (r >> 1) & 7, k = 2 * p + (r & 1);
    const float c = (d < D && k < K) ? (float)prm.items[((size_t)a * K + k) * D + d] : 0.0f;
    s_scr[a * L.scr_stride + r] = c * kNegLog2e;
  }
  for (int i = tid; i < N * L.kpairs * 2; i += kThreads) {  // 1/v (padding items: +inf)
    const int a = i / (L.kpairs * 2), k = i - a * (L.kpairs * 2);
    s_scr_val[a * L.scr_val_stride + k] = k < K ? 1.0f / (float)prm.values[(size_t)a * K + k] : INFINITY;
  }
  for (int a = tid; a < N; a += kThreads) {
    float m = 0.0f;
    for (int r = 0; r < K * D; ++r) m = fmaxf(m, (float)fabs(prm.items[(size_t)a * K * D + r]));
    s_amax[a] = m * 1.001f;
  }
  const int R = L.replicas;
  const int cnt_qwords = N * R * kOraStride;
  if (prm.want_counters)
    for (int i = tid; i < cnt_qwords; i += kThreads) reinterpret_cast<unsigned long long *>(s_cnt)[i] = 0ull;
  __syncthreads();

  const bool charged = P >= 2;  // P == 1: empty price arrays, nobody charged (Auction.py:68)
  const bool fp = prm.mech == AG_FIRST_PRICE;
  const bool packed = N <= 8;
  const uint32_t agent_bytes = (uint32_t)R * kOraStride * 8;
  const uint32_t lane_off = (uint32_t)(tid & (R - 1)) * kOraStride * 8;
  uint64_t n_logs_packed = 0, n_won_packed = 0;
  int since_flush = 0;
  auto cadd = [&](uint32_t addr, int slot, unsigned long long v) {
    atomicAdd(reinterpret_cast<unsigned long long *>(s_cnt + addr + slot * 8), v);
  };
  auto flush_counts = [&]() {  // the 8-bit per-agent fields -> the LDS count slot
    for (int a = 0; a < N; ++a) {
      const uint64_t v = ((n_logs_packed >> (8 * a)) & 255ull) | (((n_won_packed >> (8 * a)) & 255ull) << 32);
      if (v) cadd((uint32_t)a * agent_bytes + lane_off, kOraSlotCounts, (unsigned long long)v);
    }
    n_logs_packed = 0;
    n_won_packed = 0;
    since_flush = 0;
  };

  const uint32_t stride = gridDim.x * kThreads;
#if AG_ORA_PREFETCH
  // the next auction's inputs are in flight while this one resolves
  double xn[kMaxD], un = 0.0;
  int an[P];
  if (!GEN && lo + blockIdx.x * kThreads + tid < hi) {
    const uint32_t i0 = lo + blockIdx.x * kThreads + tid;
#pragma unroll
    for (int e = 0; e < D - 1; ++e) xn[e] = ldg(prm.ctx + e * B + i0);
#pragma unroll
    for (int s = 0; s < P; ++s) an[s] = ldg(prm.part + s * B + i0);
    un = ldg(prm.u + i0);
  }
#endif
#if AG_ORA_QUEUE
  // wave w of block b claims from counter q = (4 b + w) mod 64; the k-th claim of counter q is
  // the chunk 64 k + q of q_len = 64 * AG_ORA_QUEUE_SUB auctions, resolved as AG_ORA_QUEUE_SUB
  // tiles of 64 (one auction per lane per tile). Lane 0 claims the chunk after next while the
  // current one resolves; the ticket is read only once that chunk is done. A wave makes at most
  // lane_tiles / AG_ORA_QUEUE_SUB claims, so each lane resolves at most claims * SUB <= lane_tiles
  // = ora_lane_cap(R) auctions: the range that keeps its exact 8-bit count fields and replica sums
  // in range. The host sizes a launch to half of what the grid's waves may take and launches at
  // least one wave per counter the chunks reach (simulate_oracle), so every chunk finds a wave
  // below its cap. Tickets only grow, so a claim left in flight at the exit is past the end too.
  (void)stride;
  const uint32_t q_lane = tid & 63;
  const uint32_t q_idx = ((uint32_t)blockIdx.x * (kThreads / 64) + (uint32_t)(tid >> 6)) & 63u;
  uint32_t *const q_ctr = prm.queue + q_idx * 32;
  constexpr uint32_t q_len = 64 * AG_ORA_QUEUE_SUB;
  const uint32_t q_chunks = (hi - lo + q_len - 1) / q_len;
  uint32_t q_claims = 0;
  auto q_claim = [&]() -> uint32_t {
    uint32_t r = 0xffffffffu;
    if (q_claims < prm.lane_tiles / AG_ORA_QUEUE_SUB) {
      if (q_lane == 0) r = atomicAdd(q_ctr, 1u);
      ++q_claims;
    }
    return r;
  };
  auto q_chunk_of = [&](uint32_t raw) -> uint32_t {
    const uint32_t t = (uint32_t)__builtin_amdgcn_readfirstlane((int)raw);
    return t == 0xffffffffu ? 0xffffffffu : t * 64u + q_idx;
  };
  uint32_t q_cur = q_chunk_of(q_claim());
  uint32_t q_raw = q_claim();
  for (;;) {
    if (q_cur >= q_chunks) break;
#pragma nounroll
    for (int q_s = 0; q_s < AG_ORA_QUEUE_SUB; ++q_s) {
    const uint32_t i = lo + q_cur * q_len + (uint32_t)q_s * 64 + q_lane;
    if (i >= hi) break;
#else
  for (uint32_t i = lo + blockIdx.x * kThreads + tid; i < hi; i += stride) {
#endif
    double x[kMaxD];
    float xf[kMaxD];
    float xabs = 1.0f;
    int ag[P];
    double u;
    if constexpr (GEN) {
      gen_auction<P, kMaxD>((uint32_t)prm.seed, (uint32_t)(prm.seed >> 32), prm.first + i, N, P, D - 1,
                            prm.scale, x, ag, u);
    } else {
#if AG_ORA_PREFETCH
#pragma unroll
      for (int e = 0; e < D - 1; ++e) x[e] = xn[e];
#pragma unroll
      for (int s = 0; s < P; ++s) ag[s] = an[s];
      u = un;
      if (i + stride < hi) {
#pragma unroll
        for (int e = 0; e < D - 1; ++e) xn[e] = ldg(prm.ctx + e * B + i + stride);
#pragma unroll
        for (int s = 0; s < P; ++s) an[s] = ldg(prm.part + s * B + i + stride);
        un = ldg(prm.u + i + stride);
      }
#else
#pragma unroll
      for (int e = 0; e < D - 1; ++e) x[e] = ldg(prm.ctx + e * B + i);
#pragma unroll
      for (int s = 0; s < P; ++s) ag[s] = ldg(prm.part + s * B + i);
      u = ldg(prm.u + i);
#endif
    }
#pragma unroll
    for (int e = 0; e < D - 1; ++e) {
      xf[e] = (float)x[e];
      xabs += fabsf(xf[e]);
    }
    x[D - 1] = 1.0;  // intercept (src/Auction.py:33)
    xf[D - 1] = 1.0f;
    xabs *= 1.001f;

    int w = 0;
    double m1 = 0.0, m2 = -INFINITY, ctr_w = 0.0, val_w = 0.0;
    double bevs[P];
#if AG_ORA_STORE_LATE
    int itv[P];
    double bdv[P], ctv[P];
#endif
#pragma unroll
    for (int s = 0; s < P; ++s) {
      const int a = ag[s];
      const double *itm = s_items + a * L.items_stride;
      const double *vv = s_vals + a * L.values_stride;
      const float *row = s_scr + a * L.scr_stride;
      const float *sv = s_scr_val + a * L.scr_val_stride;
      uint32_t t1, t2;
      ora_screen<D>(row, sv, L.kpairs, xf, t1, t2);
      const bool ok = (s_amax[a] * xabs <= kPruneMaxS) && (__uint_as_float(t1 & ~15u) <= 1e30f);
      const float thr = __uint_as_float(t1 & ~15u) * (1.0f + kPruneDelta);
      // the f32 leader, exactly (every lane)
      int best = (int)(t1 & 15u);
      double c = agexp::sigmoid_fast(dot_ref<D>(itm + best * D, x), s_tab);
      double sc = c * vv[best];
      if (!ok || !(__uint_as_float(t2 & ~15u) > thr)) {
        // near-tie (rare) or unscreenable lane: every item under the threshold, exactly,
        // in increasing k (first maximum)
        const int kf = best;
        const double c_kf = c;
        best = -1;
        for (int k = 0; k < K; ++k) {
          if (ok && k != kf && !(__uint_as_float(ora_screen_one<D>(row, sv, k, xf) & ~15u) <= thr)) continue;
          const double ck = k == kf ? c_kf : agexp::sigmoid_fast(dot_ref<D>(itm + k * D, x), s_tab);
          const double sk = ck * vv[k];
          if (best < 0 || sk > sc || (sk == sc && k < best)) {
            best = k;
            sc = sk;
            c = ck;
          }
        }
      }
      const double v = vv[best];
      const double b = v * c;  // TruthfulBidder.bid: value * estimated CTR (src/Bidder.py:35)
      bevs[s] = sc;  // max_k CTR_k * value_k (src/Auction.py:53); == b for an Oracle agent
#if AG_ORA_STORE_LATE
      itv[s] = best;
      bdv[s] = b;
      ctv[s] = c;
#else
      const uint32_t o = s * B + i;
      if (prm.item) stg(prm.item + o, (int32_t)best);
      if (prm.bid) stg(prm.bid + o, b);
      if (prm.est_ctr) stg(prm.est_ctr + o, c);
      if (prm.true_ctr) stg(prm.true_ctr + o, c);
      if (prm.best_ev) stg(prm.best_ev + o, sc);
#endif
      // streaming top-2, ties -> lowest slot (src/AuctionAllocation.py:19-34)
      if (s == 0) {
        m1 = b;
        ctr_w = c;
        val_w = v;
      } else if (b > m1) {
        m2 = m1;
        m1 = b;
        w = s;
        ctr_w = c;
        val_w = v;
      } else if (b > m2) {
        m2 = b;
      }
    }
    const double price = fp ? m1 : m2;
    const int oc = bernoulli(ctr_w, u);  // src/Auction.py:65 (true CTR of the winner's item)
#if AG_ORA_STORE_LATE
    // every per-slot output after the slots, field by field
#pragma unroll
    for (int s = 0; s < P; ++s)
      if (prm.item) stg(prm.item + s * B + i, (int32_t)itv[s]);
#pragma unroll
    for (int s = 0; s < P; ++s)
      if (prm.bid) stg(prm.bid + s * B + i, bdv[s]);
#pragma unroll
    for (int s = 0; s < P; ++s)
      if (prm.est_ctr) stg(prm.est_ctr + s * B + i, ctv[s]);
#pragma unroll
    for (int s = 0; s < P; ++s)
      if (prm.true_ctr) stg(prm.true_ctr + s * B + i, ctv[s]);
#pragma unroll
    for (int s = 0; s < P; ++s)
      if (prm.best_ev) stg(prm.best_ev + s * B + i, bevs[s]);
#endif
    if (prm.winner) stg(prm.winner + i, (int32_t)w);
    if (prm.price) stg(prm.price + i, charged ? price : (double)NAN);
    if (prm.second_price) stg(prm.second_price + i, charged ? m2 : (double)NAN);
    if (prm.outcome) stg(prm.outcome + i, (uint8_t)oc);
    if (prm.winner_outcome) stg(prm.winner_outcome + i, pack_wo(w, oc));

    if (prm.want_counters) {
#pragma unroll
      for (int s = 0; s < P; ++s) {
        const uint32_t addr = (uint32_t)ag[s] * agent_bytes + lane_off;
        const bool won = charged && s == w;
        cadd(addr, kOraSlotBestEv, ora_fx(bevs[s]));
        if constexpr (P == 1) {  // (0 - bid) * (0 < true CTR * value), true CTR * value == bid
          if (bevs[s] > 0.0) cadd(addr, kOraSlotUnderbid1, ora_fx(-bevs[s]));
        }
        if (won) {
          cadd(addr, kOraSlotPaid, ora_fx(price));
          if (oc) cadd(addr, kOraSlotGross, ora_fx(val_w));
          if (fp && charged) {
            const unsigned long long ob = ora_fx(price - m2);
            if (ob) cadd(addr, kOraSlotOverbid, ob);
          }
        }
        if (packed) {
          const uint64_t bit = 1ull << (8 * ag[s]);
          n_logs_packed += bit;
          if (won) n_won_packed += bit;
        } else {
          cadd(addr, kOraSlotCounts, won ? 0x100000001ull : 1ull);
        }
      }
      if (packed && ++since_flush == kOraFlush) flush_counts();
    }
#if AG_ORA_QUEUE
    }
    q_cur = q_chunk_of(q_raw);
    q_raw = q_claim();
#endif
  }

  if (!prm.want_counters) return;
  if (packed) flush_counts();
  __syncthreads();
  // per (agent, slot) pair, one thread each: its replicas summed as two limbs (value = lo +
  // hi * 2^42; counts: logs in lo, wins in hi), written over the pair's replica-0 / -1 words
  // (loads pipelined 8 at a time; one thread per agent looping over every slot and replica
  // cost ~10 us per launch), then the block's partials in k_simulate's format
  unsigned long long *cnt = reinterpret_cast<unsigned long long *>(s_cnt);
  auto split = [&](int j, unsigned long long c, long long &l, long long &h) {
    if (j == kOraSlotCounts) {
      l = (long long)(c & 0xffffffffull);
      h = (long long)(c >> 32);
    } else {
      l = (long long)c & kLimbMask;
      h = (long long)c >> AG_FX_LIMB_BITS;
    }
  };
  if (R >= 2) {
    for (int pr = tid; pr < N * kOraStride; pr += kThreads) {
      const int a = pr / kOraStride, j = pr - a * kOraStride;
      const unsigned long long *c0 = cnt + (size_t)a * R * kOraStride + j;
      long long sl = 0, sh = 0;
      for (int r0 = 0; r0 < R; r0 += 8) {
        unsigned long long v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = r0 + u < R ? c0[(size_t)(r0 + u) * kOraStride] : 0ull;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          long long l, h;
          split(j, v[u], l, h);
          sl += l;
          sh += h;
        }
      }
      cnt[(size_t)a * R * kOraStride + j] = (unsigned long long)sl;
      cnt[((size_t)a * R + 1) * kOraStride + j] = (unsigned long long)sh;
    }
    __syncthreads();
  }
  for (int a = tid; a < N; a += kThreads) {
    long long lo_[kOraStride], hi_[kOraStride];
    for (int j = 0; j < kOraStride; ++j) {
      if (R >= 2) {
        lo_[j] = (long long)cnt[(size_t)a * R * kOraStride + j];
        hi_[j] = (long long)cnt[((size_t)a * R + 1) * kOraStride + j];
      } else {
        split(j, cnt[(size_t)a * kOraStride + j], lo_[j], hi_[j]);
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
    const unsigned long long nlogs = (unsigned long long)lo_[kOraSlotCounts];
    const unsigned long long nwon = (unsigned long long)hi_[kOraSlotCounts];
    if constexpr (P == 1)
      put(AG_C_NET, lo_[kOraSlotGross], hi_[kOraSlotGross]);
    else
      put(AG_C_NET, lo_[kOraSlotGross] - lo_[kOraSlotPaid], hi_[kOraSlotGross] - hi_[kOraSlotPaid]);
    put(AG_C_GROSS, lo_[kOraSlotGross], hi_[kOraSlotGross]);
    put(AG_C_ALLOC_REGRET, 0, 0);
    put(AG_C_EST_REGRET, 0, 0);
    put(AG_C_OVERBID, lo_[kOraSlotOverbid], hi_[kOraSlotOverbid]);
    if constexpr (P == 1)
      put(AG_C_UNDERBID, lo_[kOraSlotUnderbid1], hi_[kOraSlotUnderbid1]);
    else
      put(AG_C_UNDERBID, 0, 0);
    put(AG_C_CTR_SQERR, 0, 0);
    put_count(AG_C_CTR_BIAS, nwon);
    put(AG_C_BEST_EV, lo_[kOraSlotBestEv], hi_[kOraSlotBestEv]);
    put_count(AG_C_N_LOGS, nlogs);
    put_count(AG_C_N_WON, nwon);
    if constexpr (P == 1)
      put(AG_C_PAID, 0, 0);
    else
      put(AG_C_PAID, lo_[kOraSlotPaid], hi_[kOraSlotPaid]);
  }
}

typedef void (*OraKernel)(OraParams);

// Defined per P in ag_sim_p.hip: k_oracle<P, D, gen> for D in [2, 8].
template <int P>
OraKernel pick_oracle_for(int D, bool gen);
template <> OraKernel pick_oracle_for<0>(int, bool);
template <> OraKernel pick_oracle_for<1>(int, bool);
template <> OraKernel pick_oracle_for<2>(int, bool);
template <> OraKernel pick_oracle_for<3>(int, bool);
template <> OraKernel pick_oracle_for<4>(int, bool);
template <> OraKernel pick_oracle_for<5>(int, bool);
template <> OraKernel pick_oracle_for<6>(int, bool);
template <> OraKernel pick_oracle_for<7>(int, bool);
template <> OraKernel pick_oracle_for<8>(int, bool);

}  // namespace ag
