// ag_lrts.hip -- LR-TS allocator update on the GPU (Agent.update -> PyTorchLogistic-
// RegressionAllocator.update, src/Agent.py:79-91, src/BidderAllocation.py:29-65,
// src/Models.py:35-48), plus the won-sample collection that feeds it.
//
//  1. k_lrts_collect   after each ag_simulate: every auction won by an LR-TS agent
//                      appends (agent, item, outcome, observed context + 1) to a
//                      caller-owned store (one atomic per wave).
//  2. bucket           histogram -> exclusive scan -> scatter: samples grouped by agent.
//  3. k_lrts_train     one workgroup per agent, persistent over the epochs: forward, BCE +
//                      prior loss, gradient, Adam, ReduceLROnPlateau and the early stop all
//                      on the device (no host round trip per epoch), then the Laplace
//                      update of q and prev_m = m.
//
// Every sum over samples is exact (fixed-point terms added as integers: oracle/ag_oracle.c
// ora_lrts_update states the arithmetic), so results do not depend on sample order,
// bucket order or the lane a sample lands on: the update is bit-identical to the oracle
// and identical on every rank of a multi-GPU job that trains on the gathered samples.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <string.h>

#include <vector>

#include "ag_exp.h"
#include "ag_exp_table.h"
#include "ag_host.h"
#include "ag_coop.h"

namespace {

constexpr int kLrThreads = 256;        // 4 waves; one sample per lane per pass
constexpr int kLrEpochs = AG_LRTS_MAX_EPOCHS;
constexpr int kLrMaxKD = 64;           // K * (OE + 1) columns of the accumulator tile
constexpr int kLrAccStride = 144;      // int64 per accumulator row: 2 (KD + 1) <= 130, 128-B multiple
constexpr int kLrCache = 16;           // samples per lane kept in registers (1 workgroup / CU)
constexpr int kAccStride = kLrThreads + 1;  // [column][lane] int64 tile, padded: the column
                                            // reduction (lanes = columns) is conflict-free
constexpr int kHistory = 100;          // losses[-100] of the early stop
constexpr double kGradScale = 0x1p40, kLossScale = 0x1p32;
constexpr int64_t kLo24 = (int64_t(1) << 24) - 1;

__device__ __forceinline__ int64_t fx_round(double v, double scale) {
  return (int64_t)__builtin_rint(v * scale);
}
// (hi, lo) partial sums of values split at bit 24 -> the exact sum S read back as
// (double)(S >> 24) * 2^24 + (double)(S & (2^24 - 1)) (ora_lrts_update's fx_read).
__device__ __forceinline__ double fx_read(int64_t hi, int64_t lo, double inv_scale) {
  hi += lo >> 24;
  lo &= kLo24;
  return ((double)hi * 0x1p24 + (double)lo) * inv_scale;
}

__device__ __forceinline__ int64_t wave_sum(int64_t v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---------------------------------------------------------------------------------------
// 1. collection: Agent.update's won_mask (src/Agent.py:90) over one simulated batch
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(kLrThreads) void k_lrts_collect(
    int64_t B, int P, int OE, const double *__restrict__ ctx, const int32_t *__restrict__ part,
    const int32_t *__restrict__ winner, const int32_t *__restrict__ item, const uint8_t *__restrict__ outcome,
    const uint32_t *__restrict__ winner_outcome, const int32_t *__restrict__ akind, uint32_t *__restrict__ key,
    float *__restrict__ x, int64_t cap, unsigned long long *__restrict__ count) {
  const int lane = threadIdx.x & 63;
  for (int64_t base = (int64_t)blockIdx.x * kLrThreads; base < B; base += (int64_t)gridDim.x * kLrThreads) {
    const int64_t i = base + threadIdx.x;
    bool take = false;
    uint32_t k = 0;
    if (i < B && P >= 2) {  // P == 1: nobody is charged, no record is won (src/Auction.py:68)
      // winner and outcome from their arrays, or from the ABI 17 packed word
      const uint32_t wo = winner ? 0u : winner_outcome[i];
      const int w = winner ? winner[i] : (int)(wo & 0x7fffffffu);
      const int a = part[(size_t)w * B + i];
      if (akind[a] == AG_ALLOCATOR_LRTS) {
        take = true;
        const bool oc = outcome ? outcome[i] != 0 : (wo >> 31) != 0;
        k = ((uint32_t)a << 16) | ((uint32_t)item[(size_t)w * B + i] << 1) | (oc ? 1u : 0u);
      }
    }
    const uint64_t ballot = __ballot(take);
    if (ballot == 0) continue;
    unsigned long long first = 0;
    const int leader = __ffsll((unsigned long long)ballot) - 1;
    if (lane == leader) first = atomicAdd(count, (unsigned long long)__popcll(ballot));
    first = __shfl(first, leader, 64);
    if (!take) continue;
    const int64_t slot = (int64_t)first + __popcll(ballot & ((1ull << lane) - 1));
    if (slot >= cap) continue;  // overflow: reported by ag_lrts_update
    key[slot] = k;
    for (int d = 0; d < OE; ++d) x[(size_t)d * cap + slot] = (float)ctx[(size_t)d * B + i];
    x[(size_t)OE * cap + slot] = 1.0f;
  }
}

// ---------------------------------------------------------------------------------------
// 2. bucket by agent
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(kLrThreads) void k_lrts_hist(const uint32_t *__restrict__ key, int64_t n, int N,
                                                          int64_t *__restrict__ counts) {
  extern __shared__ unsigned int s_hist[];
  for (int a = threadIdx.x; a < N; a += kLrThreads) s_hist[a] = 0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * kLrThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kLrThreads)
    atomicAdd(&s_hist[key[i] >> 16], 1u);
  __syncthreads();
  for (int a = threadIdx.x; a < N; a += kLrThreads)
    if (s_hist[a]) atomicAdd((unsigned long long *)&counts[a], (unsigned long long)s_hist[a]);
}

// counts [N] -> offsets [N + 1] (exclusive scan) and cursors [N] = offsets; one block.
__global__ __launch_bounds__(kLrThreads) void k_lrts_scan(int64_t *__restrict__ counts, int N,
                                                          int64_t *__restrict__ offsets,
                                                          int64_t *__restrict__ cursors) {
  __shared__ int64_t s_carry;
  __shared__ int64_t s_w[kLrThreads / 64];
  if (threadIdx.x == 0) s_carry = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int base = 0; base < N; base += kLrThreads) {
    const int a = base + threadIdx.x;
    const int64_t v = a < N ? counts[a] : 0;
    int64_t incl = v;
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
    if (lane == 63) s_w[wv] = incl;
    __syncthreads();
    int64_t pre = s_carry;
    for (int j = 0; j < wv; ++j) pre += s_w[j];
    if (a < N) {
      offsets[a] = pre + incl - v;
      cursors[a] = pre + incl - v;
    }
    __syncthreads();
    if (threadIdx.x == kLrThreads - 1) s_carry = pre + incl;
    __syncthreads();
  }
  if (threadIdx.x == 0) offsets[N] = s_carry;
}

__global__ __launch_bounds__(kLrThreads) void k_lrts_scatter(const uint32_t *__restrict__ key,
                                                             const float *__restrict__ x, int64_t n,
                                                             int64_t cap_in, int Do,
                                                             int64_t *__restrict__ cursors,
                                                             uint32_t *__restrict__ okey,
                                                             float *__restrict__ ox, int64_t cap_out) {
  for (int64_t i = (int64_t)blockIdx.x * kLrThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kLrThreads) {
    const uint32_t k = key[i];
    const int64_t pos = (int64_t)atomicAdd((unsigned long long *)&cursors[k >> 16], 1ull);
    okey[pos] = k;
    for (int d = 0; d < Do; ++d) ox[(size_t)d * cap_out + pos] = x[(size_t)d * cap_in + i];
  }
}

// ---------------------------------------------------------------------------------------
// 3. training: up to kLrCache * 256 samples per workgroup, several workgroups per agent
// ---------------------------------------------------------------------------------------
struct LrSample {
  float x[AG_LRTS_MAX_DO];
  int item;
  int y;
};

template <int DO>
__device__ __forceinline__ float lr_logit(const float *__restrict__ w, const float (&x)[AG_LRTS_MAX_DO]) {
  float z = w[0] * x[0];
#pragma unroll
  for (int d = 1; d < DO; ++d) z = z + w[d] * x[d];
  return z;
}

template <int DO>
__device__ __forceinline__ void lr_load(const uint32_t *__restrict__ key, const float *__restrict__ x,
                                        int64_t cap, int64_t i, LrSample &s) {
  const uint32_t k = key[i];
  s.item = (int)((k >> 1) & 0x7fffu);
  s.y = (int)(k & 1u);
#pragma unroll
  for (int d = 0; d < DO; ++d) s.x[d] = x[(size_t)d * cap + i];
}

// One sample's contribution to the epoch: BCE term (fixed point, returned) and gradient
// terms added to this lane's accumulator column.
template <int DO>
__device__ __forceinline__ int64_t lr_epoch_sample(const LrSample &s, const float *__restrict__ sm,
                                                   int64_t *__restrict__ acc, const uint64_t *tab) {
  const float z = lr_logit<DO>(sm + s.item * DO, s.x);
  const float p = 1.0f / (1.0f + (float)agexp::exp_fast(-(double)z, tab));
  const double t = s.y ? -fmax(log((double)p), -100.0) : -fmax(log1p(-(double)p), -100.0);
  const double gz = (double)p - (double)s.y;
#pragma unroll
  for (int d = 0; d < DO; ++d) acc[(s.item * DO + d) * kAccStride] += fx_round(gz * (double)s.x[d], kGradScale);
  return fx_round(t, kLossScale);
}

template <int DO>
__device__ __forceinline__ void lr_laplace_sample(const LrSample &s, const float *__restrict__ sm,
                                                  int64_t *__restrict__ acc, const uint64_t *tab) {
  const float z = lr_logit<DO>(sm + s.item * DO, s.x);
  const float P = 1.0f / (1.0f + (float)agexp::exp_fast((double)(1.0f - z), tab));
  const float w = P * (1.0f - P);
#pragma unroll
  for (int d = 0; d < DO; ++d)
    acc[(s.item * DO + d) * kAccStride] += fx_round((double)w * (double)(s.x[d] * s.x[d]), kGradScale);
}

// Per-block column sums of the lane accumulator tile (thread = column c, row group r;
// each value split at bit 24 so no partial can overflow) into the block's slot of the
// agent's partials [rank][KD + 1][2] (column KD: the loss); the tile is zeroed for reuse.
__device__ __forceinline__ void lr_block_partials(int64_t *__restrict__ s_acc, int KD, int64_t lsum_hi,
                                                  int64_t lsum_lo, int64_t (*s_hi)[kLrMaxKD + 1],
                                                  int64_t (*s_lo)[kLrMaxKD + 1], int64_t *__restrict__ dst) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  {
    const int64_t h = wave_sum(lsum_hi), l = wave_sum(lsum_lo);
    if (lane == 0) {
      s_hi[wv][KD] = h;
      s_lo[wv][KD] = l;
    }
  }
  const int c = tid & 63, r = tid >> 6;
  if (c < KD) {
    int64_t h = 0, l = 0;
    int64_t *col = s_acc + c * kAccStride + r * 64;
    for (int j = 0; j < 64; ++j) {
      const int64_t v = col[j];
      col[j] = 0;
      h += v >> 24;
      l += v & kLo24;
    }
    s_hi[r][c] = h;
    s_lo[r][c] = l;
  }
  __syncthreads();
  if (tid <= KD) {
    dst[2 * tid] = s_hi[0][tid] + s_hi[1][tid] + s_hi[2][tid] + s_hi[3][tid];
    dst[2 * tid + 1] = s_lo[0][tid] + s_lo[1][tid] + s_lo[2][tid] + s_lo[3][tid];
  }
}

// The training of one LR-TS agent is spread over `nblk` co-resident workgroups, each
// owning a contiguous chunk of the agent's samples (the first kLrCache per lane in
// registers). Every epoch each workgroup writes its exact partial sums; after the agent
// barrier EVERY workgroup adds all partials (integers: identical totals everywhere) and
// runs the same Adam / scheduler / early-stop step on its LDS copy of the parameters, so
// the workgroups stay in lockstep without a second barrier. Partials are double-buffered
// by epoch parity.
template <int DO>
__global__ __launch_bounds__(kLrThreads) void k_lrts_train(
    int K, const int32_t *__restrict__ blk_agent, const int32_t *__restrict__ blk_rank,
    const int32_t *__restrict__ agent_nblk, const int64_t *__restrict__ agent_pbase,
    const int64_t *__restrict__ offsets, const uint32_t *__restrict__ key, const float *__restrict__ xs,
    int64_t cap, float *__restrict__ gm, float *__restrict__ gq, float *__restrict__ gpm,
    const double *__restrict__ adam_tab, int32_t *__restrict__ epochs_out, float *__restrict__ loss_trace,
    int64_t *__restrict__ partials, unsigned *__restrict__ barriers, const int32_t *__restrict__ bar_off) {
  const int a = blk_agent[blockIdx.x], rank = blk_rank[blockIdx.x], nblk = agent_nblk[a];
  const int tid = threadIdx.x;
  const int64_t s0 = offsets[a], n = offsets[a + 1] - s0;
  const int KD = K * DO;
  const int PW = 2 * (KD + 1);  // int64 per partial record
  // the agent's accumulator rows [bar_lines(nblk)][kLrAccStride] (agcoop::agent_allreduce_i64)
  int64_t *accrows = partials + agent_pbase[a];
  unsigned *bar = barriers + (size_t)bar_off[a] * agcoop::kBarLineWords;
  // this workgroup's samples: [c0, c1) of the agent's n
  const int64_t per = (n + nblk - 1) / nblk;
  const int64_t c0 = (int64_t)rank * per, c1 = c0 + per < n ? c0 + per : n;
  const int64_t nb = c1 > c0 ? c1 - c0 : 0;

  extern __shared__ int64_t s_acc[];  // [KD][kAccStride]
  __shared__ uint64_t s_tab[256];
  __shared__ float s_m[kLrMaxKD], s_pm[kLrMaxKD], s_q[kLrMaxKD], s_ea[kLrMaxKD], s_es[kLrMaxKD];
  __shared__ int64_t s_hi[4][kLrMaxKD + 1], s_lo[4][kLrMaxKD + 1];
  __shared__ float s_hist[kHistory];
  __shared__ float s_loss, s_negstep, s_bc2;
  __shared__ double s_lr, s_best;
  __shared__ int s_bad, s_stop, s_flag;
  __shared__ int64_t s_part[2 * (kLrMaxKD + 1)], s_tot[2 * (kLrMaxKD + 1)];

  for (int i = tid; i < 256; i += kLrThreads) s_tab[i] = ag_exp_tab[i];
  float *m_g = gm + (size_t)a * KD, *q_g = gq + (size_t)a * KD, *pm_g = gpm + (size_t)a * KD;
  for (int c = tid; c < KD; c += kLrThreads) {
    s_m[c] = m_g[c];
    s_pm[c] = pm_g[c];
    s_q[c] = q_g[c];
    s_ea[c] = 0.0f;
    s_es[c] = 0.0f;
  }
  for (int i = tid; i < KD * kAccStride; i += kLrThreads) s_acc[i] = 0;
  if (tid == 0) {
    s_lr = 2e-3;
    s_best = INFINITY;
    s_bad = 0;
    s_stop = 0;
  }
  LrSample cache[kLrCache];
  int ncached = 0;
#pragma unroll
  for (int j = 0; j < kLrCache; ++j) {
    const int64_t i = (int64_t)j * kLrThreads + tid;
    if (i < nb) {
      lr_load<DO>(key, xs, cap, s0 + c0 + i, cache[j]);
      ncached = j + 1;
    }
  }
  const int64_t stream_from = (int64_t)kLrCache * kLrThreads;
  int64_t *acc = s_acc + tid;
  __syncthreads();

  int epoch = 0;
  for (; epoch < kLrEpochs; ++epoch) {
    // ---- A: forward + BCE + gradient terms of this lane's samples
    int64_t lsum = 0;
#pragma unroll
    for (int j = 0; j < kLrCache; ++j)
      if (j < ncached) lsum += lr_epoch_sample<DO>(cache[j], s_m, acc, s_tab);
    for (int64_t i = stream_from + tid; i < nb; i += kLrThreads) {
      LrSample sm;
      lr_load<DO>(key, xs, cap, s0 + c0 + i, sm);
      lsum += lr_epoch_sample<DO>(sm, s_m, acc, s_tab);
    }
    __syncthreads();
    // ---- B: this workgroup's exact partials, summed over the agent's workgroups up the
    // barrier tree (exact integer atomics; every workgroup gets the same totals)
    lr_block_partials(s_acc, KD, lsum >> 24, lsum & kLo24, s_hi, s_lo, s_part);
    agcoop::agent_allreduce_i64(bar, accrows, kLrAccStride, rank, nblk, s_part, PW, s_tot, &s_flag);
    // ---- C: totals (identical in every workgroup), loss, Adam; scheduler on thread 0
    if (tid == 0) {
      const int64_t h = s_tot[2 * KD], l = s_tot[2 * KD + 1];
      double prior = 0.0;
      for (int k = 0; k < K; ++k)
        for (int d = 0; d < DO - 1; ++d) {
          const double df = (double)s_pm[k * DO + d] - (double)s_m[k * DO + d];
          prior += (double)s_q[k * DO + d] * (df * df);
        }
      s_loss = (float)(0.5 * prior + fx_read(h, l, 1.0 / kLossScale));
      s_negstep = (float)(-(s_lr / adam_tab[epoch]));
      s_bc2 = (float)adam_tab[kLrEpochs + epoch];
    }
    __syncthreads();
    if (tid < KD) {
      const int c = tid;
      const int64_t h = s_tot[2 * c], l = s_tot[2 * c + 1];
      const double gp = (c % DO) < DO - 1 ? -(double)s_q[c] * ((double)s_pm[c] - (double)s_m[c]) : 0.0;
      const float g = (float)(fx_read(h, l, 1.0 / kGradScale) + gp);
      const float ea = s_ea[c] + 0.1f * (g - s_ea[c]);
      const float es = s_es[c] * 0.999f + (0.001f * g) * g;
      // float32 sqrt correctly rounded (as the CPU sqrtss): via the refined FP64 sqrt --
      // double rounding is innocuous for sqrt (53 >= 2 * 24 + 2); v_sqrt_f32 is 1 ulp.
      const float den = (float)__builtin_sqrt((double)es) / s_bc2 + 1e-8f;
      s_ea[c] = ea;
      s_es[c] = es;
      s_m[c] = s_m[c] + s_negstep * (ea / den);
    }
    if (tid == 0) {
      const float loss = s_loss;
      if (loss_trace && rank == 0) loss_trace[(size_t)a * kLrEpochs + epoch] = loss;
      s_hist[epoch % kHistory] = loss;
      if ((double)loss < s_best * (1.0 - 1e-4)) {
        s_best = (double)loss;
        s_bad = 0;
      } else {
        s_bad += 1;
      }
      if (s_bad > 10) {
        const double nl = s_lr * 0.5;
        if (s_lr - nl > 1e-8) s_lr = nl;
        s_bad = 0;
      }
      if (epoch > 1024 && fabs((double)s_hist[(epoch - 99) % kHistory] - (double)loss) < 1e-6) s_stop = 1;
    }
    __syncthreads();
    if (s_stop) {
      ++epoch;
      break;
    }
  }

  // ---- Laplace approximation of q (src/Models.py:43-45), then prev_m = m
#pragma unroll
  for (int j = 0; j < kLrCache; ++j)
    if (j < ncached) lr_laplace_sample<DO>(cache[j], s_m, acc, s_tab);
  for (int64_t i = stream_from + tid; i < nb; i += kLrThreads) {
    LrSample sm;
    lr_load<DO>(key, xs, cap, s0 + c0 + i, sm);
    lr_laplace_sample<DO>(sm, s_m, acc, s_tab);
  }
  __syncthreads();
  lr_block_partials(s_acc, KD, 0, 0, s_hi, s_lo, s_part);
  agcoop::agent_allreduce_i64(bar, accrows, kLrAccStride, rank, nblk, s_part, PW, s_tot, &s_flag);
  if (rank == 0) {
    if (tid < KD) {
      const int c = tid;
      const int64_t h = s_tot[2 * c], l = s_tot[2 * c + 1];
      q_g[c] = s_q[c] + (float)fx_read(h, l, 1.0 / kGradScale);
      m_g[c] = s_m[c];
      pm_g[c] = s_m[c];
    }
    if (tid == 0) epochs_out[a] = epoch;
  }
}

// ---------------------------------------------------------------------------------------
// 4. resumable / record-parallel training (ag_lrts_rp_*): the same fit as k_lrts_train, one
//    launch per epoch, each agent's state (m, Adam moments, scheduler, loss history, phase) in
//    HBM between launches. Launch k steps the state with the totals of launch k - 1 (this
//    rank's workgroups summed up the agent's combining tree without waiting, then -- G ranks --
//    the caller's int64 all-reduce), then adds the next epoch's exact partials at the new m:
//    every rank holding a shard of an agent's won samples steps to the posterior one process
//    computes from all of them (ag_dr.hip k_bidder_epoch has the same structure).
// ---------------------------------------------------------------------------------------
enum { kLrTrain = 0, kLrLaplace, kLrDone };
struct LrSt {
  int32_t phase, epoch, have_tot, bad;
  double lr, best;
  float m[kLrMaxKD], ea[kLrMaxKD], es[kLrMaxKD];
  float hist[kHistory];
};

// Both parities of the state ([2][N]) are initialised: k_lrts_epoch writes st_out only for
// the masked agents, so an unmasked agent's parity-1 row must already read Done when
// ag_lrts_rp_poll looks at it after an odd number of launches.
__global__ void k_lrts_rp_init(int N, int KD, const int32_t *__restrict__ mask, const float *__restrict__ gm,
                               LrSt *__restrict__ st) {
  const int a = blockIdx.x;
  if (a >= N) return;
  for (int par = 0; par < 2; ++par) {
    LrSt &f = st[(size_t)par * N + a];
    for (int c = threadIdx.x; c < kLrMaxKD; c += blockDim.x) {
      f.m[c] = c < KD ? gm[(size_t)a * KD + c] : 0.0f;
      f.ea[c] = f.es[c] = 0.0f;
    }
    for (int c = threadIdx.x; c < kHistory; c += blockDim.x) f.hist[c] = 0.0f;
    if (threadIdx.x == 0) {
      f.phase = mask[a] ? kLrTrain : kLrDone;
      f.epoch = f.have_tot = f.bad = 0;
      f.lr = 2e-3;
      f.best = INFINITY;
    }
  }
}

template <int DO>
__global__ __launch_bounds__(kLrThreads) void k_lrts_epoch(
    int K, const int32_t *__restrict__ blk_agent, const int32_t *__restrict__ blk_rank,
    const int32_t *__restrict__ agent_nblk, const int64_t *__restrict__ offsets, const uint32_t *__restrict__ key,
    const float *__restrict__ xs, int64_t cap, float *__restrict__ gm, float *__restrict__ gq,
    float *__restrict__ gpm, const double *__restrict__ adam_tab, int32_t *__restrict__ epochs_out,
    const LrSt *__restrict__ st_in, LrSt *__restrict__ st_out, const int64_t *__restrict__ tot_in,
    int64_t *__restrict__ tot_out, int64_t *__restrict__ acc_rows, unsigned *__restrict__ bars,
    const int32_t *__restrict__ bar_off) {
  const int a = blk_agent[blockIdx.x], rank = blk_rank[blockIdx.x], nblk = agent_nblk[a];
  const int tid = threadIdx.x;
  const int KD = K * DO;
  const int PW = 2 * (KD + 1);
  extern __shared__ int64_t s_acc[];  // [KD][kAccStride]
  __shared__ uint64_t s_tab[256];
  __shared__ LrSt st;
  __shared__ float s_q[kLrMaxKD], s_pm[kLrMaxKD];
  __shared__ int64_t s_hi[4][kLrMaxKD + 1], s_lo[4][kLrMaxKD + 1];
  __shared__ float s_loss, s_negstep, s_bc2;
  __shared__ int s_flag;
  __shared__ int64_t s_part[2 * (kLrMaxKD + 1)];
  for (int i = tid; i < 256; i += kLrThreads) s_tab[i] = ag_exp_tab[i];
  for (int i = tid; i < (int)(sizeof(LrSt) / 4); i += kLrThreads)
    reinterpret_cast<uint32_t *>(&st)[i] = reinterpret_cast<const uint32_t *>(st_in + a)[i];
  float *q_g = gq + (size_t)a * KD, *pm_g = gpm + (size_t)a * KD, *m_g = gm + (size_t)a * KD;
  for (int c = tid; c < KD; c += kLrThreads) {
    s_q[c] = q_g[c];
    s_pm[c] = pm_g[c];
  }
  for (int i = tid; i < KD * kAccStride; i += kLrThreads) s_acc[i] = 0;
  __syncthreads();
  const int64_t *T = tot_in + (size_t)a * kLrAccStride;
  if (st.phase == kLrTrain && st.have_tot) {
    // k_lrts_train's step C from the summed partials of epoch st.epoch
    const int epoch = st.epoch;
    if (tid == 0) {
      double prior = 0.0;
      for (int k = 0; k < K; ++k)
        for (int d = 0; d < DO - 1; ++d) {
          const double df = (double)s_pm[k * DO + d] - (double)st.m[k * DO + d];
          prior += (double)s_q[k * DO + d] * (df * df);
        }
      s_loss = (float)(0.5 * prior + fx_read(T[2 * KD], T[2 * KD + 1], 1.0 / kLossScale));
      s_negstep = (float)(-(st.lr / adam_tab[epoch]));
      s_bc2 = (float)adam_tab[kLrEpochs + epoch];
    }
    __syncthreads();
    if (tid < KD) {
      const int c = tid;
      const double gp = (c % DO) < DO - 1 ? -(double)s_q[c] * ((double)s_pm[c] - (double)st.m[c]) : 0.0;
      const float g = (float)(fx_read(T[2 * c], T[2 * c + 1], 1.0 / kGradScale) + gp);
      const float ea = st.ea[c] + 0.1f * (g - st.ea[c]);
      const float es = st.es[c] * 0.999f + (0.001f * g) * g;
      const float den = (float)__builtin_sqrt((double)es) / s_bc2 + 1e-8f;
      st.ea[c] = ea;
      st.es[c] = es;
      st.m[c] = st.m[c] + s_negstep * (ea / den);
    }
    __syncthreads();
    if (tid == 0) {
      const float loss = s_loss;
      st.hist[epoch % kHistory] = loss;
      if ((double)loss < st.best * (1.0 - 1e-4)) {
        st.best = (double)loss;
        st.bad = 0;
      } else {
        st.bad += 1;
      }
      if (st.bad > 10) {
        const double nl = st.lr * 0.5;
        if (st.lr - nl > 1e-8) st.lr = nl;
        st.bad = 0;
      }
      const bool stop = epoch > 1024 && fabs((double)st.hist[(epoch - 99) % kHistory] - (double)loss) < 1e-6;
      st.epoch = epoch + 1;
      if (stop || st.epoch >= kLrEpochs) st.phase = kLrLaplace;
      st.have_tot = 0;
    }
    __syncthreads();
  } else if (st.phase == kLrLaplace && st.have_tot) {
    // the Laplace q from the summed terms, then prev_m = m (src/Models.py:43-48)
    if (rank == 0) {
      for (int c = tid; c < KD; c += kLrThreads) {
        q_g[c] = s_q[c] + (float)fx_read(T[2 * c], T[2 * c + 1], 1.0 / kGradScale);
        m_g[c] = st.m[c];
        pm_g[c] = st.m[c];
      }
      if (tid == 0) epochs_out[a] = st.epoch;
    }
    __syncthreads();
    if (tid == 0) {
      st.phase = kLrDone;
      st.have_tot = 0;
    }
    __syncthreads();
  }
  const bool active = st.phase != kLrDone;
  if (active) {
    const int64_t s0 = offsets[a], n = offsets[a + 1] - s0;
    const int64_t per = (n + nblk - 1) / nblk;
    const int64_t c0 = (int64_t)rank * per < n ? (int64_t)rank * per : n;
    const int64_t c1 = c0 + per < n ? c0 + per : n;
    int64_t *acc = s_acc + tid;
    int64_t lsum = 0;
    const bool train = st.phase == kLrTrain;
    for (int64_t i = c0 + tid; i < c1; i += kLrThreads) {
      LrSample sm;
      lr_load<DO>(key, xs, cap, s0 + i, sm);
      if (train)
        lsum += lr_epoch_sample<DO>(sm, st.m, acc, s_tab);
      else
        lr_laplace_sample<DO>(sm, st.m, acc, s_tab);
    }
    __syncthreads();
    lr_block_partials(s_acc, KD, lsum >> 24, lsum & kLo24, s_hi, s_lo, s_part);
    agcoop::agent_reduce_nowait(bars + (size_t)bar_off[a] * agcoop::kBarLineWords,
                                acc_rows + (size_t)bar_off[a] * kLrAccStride, kLrAccStride, rank, nblk, s_part, PW,
                                tot_out + (size_t)a * kLrAccStride, &s_flag);
  }
  if (rank == 0 && tid == 0) {
    st.have_tot = active ? 1 : 0;
    st_out[a] = st;
  }
}

using EpochKernel = void (*)(int, const int32_t *, const int32_t *, const int32_t *, const int64_t *,
                             const uint32_t *, const float *, int64_t, float *, float *, float *, const double *,
                             int32_t *, const LrSt *, LrSt *, const int64_t *, int64_t *, int64_t *, unsigned *,
                             const int32_t *);
EpochKernel pick_epoch(int Do) {
  switch (Do) {
    case 1: return k_lrts_epoch<1>;
    case 2: return k_lrts_epoch<2>;
    case 3: return k_lrts_epoch<3>;
    case 4: return k_lrts_epoch<4>;
    case 5: return k_lrts_epoch<5>;
    case 6: return k_lrts_epoch<6>;
    case 7: return k_lrts_epoch<7>;
    case 8: return k_lrts_epoch<8>;
    default: return nullptr;
  }
}

using TrainKernel = void (*)(int, const int32_t *, const int32_t *, const int32_t *, const int64_t *,
                             const int64_t *, const uint32_t *, const float *, int64_t, float *, float *,
                             float *, const double *, int32_t *, float *, int64_t *, unsigned *, const int32_t *);

TrainKernel pick_train(int Do) {
  switch (Do) {
    case 1: return k_lrts_train<1>;
    case 2: return k_lrts_train<2>;
    case 3: return k_lrts_train<3>;
    case 4: return k_lrts_train<4>;
    case 5: return k_lrts_train<5>;
    case 6: return k_lrts_train<6>;
    case 7: return k_lrts_train<7>;
    case 8: return k_lrts_train<8>;
    default: return nullptr;
  }
}

int grid_over(int64_t n) {
  int64_t g = (n + kLrThreads - 1) / kLrThreads;
  if (g > 4096) g = 4096;
  return (int)(g < 1 ? 1 : g);
}

int check_store(const ag_ctx *c, const ag_lrts_samples *s, const char *who) {
  if (!c || !s) return ag_set_error(AG_ERR_INVALID, "%s: null argument", who);
  AG_CHECK_STRUCT(s, who, "ag_lrts_samples");
  if (!s->key || !s->x || !s->count || s->capacity < 0)
    return ag_set_error(AG_ERR_INVALID, "%s: sample store needs key, x, count and capacity >= 0", who);
  return AG_OK;
}

}  // namespace

void ag_lrts_release(ag_ctx *c) {
  ag_lrts_ws &w = c->lrts;
  (void)hipFree(w.key);
  (void)hipFree(w.x);
  (void)hipFree(w.offsets);
  (void)hipFree(w.adam_tab);
  (void)hipFree(w.epochs);
  (void)hipFree(w.tables);
  (void)hipFree(w.partials);
  (void)hipFree(w.rp.st);
  (void)hipFree(w.rp.acc);
  (void)hipFree(w.rp.tables);
  w = ag_lrts_ws();
}

extern "C" {

int ag_lrts_collect(ag_ctx *c, int64_t B, const ag_batch_in *in, const ag_batch_out *out_arg,
                    const ag_lrts_samples *s, void *stream) {
  if (int rc = check_store(c, s, "ag_lrts_collect")) return rc;
  if (!in || !out_arg) return ag_set_error(AG_ERR_INVALID, "ag_lrts_collect: null argument");
  AG_CHECK_STRUCT(in, "ag_lrts_collect", "ag_batch_in");
  ag_batch_out outv;
  AG_READ_OUT(out_arg, outv, "ag_lrts_collect");
  const ag_batch_out *out = &outv;
  if (B < 0) return ag_set_error(AG_ERR_INVALID, "ag_lrts_collect: B < 0");
  if (B == 0 || !c->has_lrts) return AG_OK;
  if (c->shape.num_agents > 65536 || c->shape.num_items > 32768)
    return ag_set_error(AG_ERR_UNSUPPORTED, "ag_lrts_collect: sample keys hold N <= 65536, K <= 32768");
  if (!in->ctx || !in->part || !out->item || !((out->winner && out->outcome) || out->winner_outcome))
    return ag_set_error(AG_ERR_INVALID, "ag_lrts_collect: needs in.ctx, in.part, out.item and out.winner + "
                                        "out.outcome (or out.winner_outcome)");
  AgDeviceGuard g(c->device);
  hipLaunchKernelGGL(k_lrts_collect, dim3(grid_over(B)), dim3(kLrThreads), 0, (hipStream_t)stream, B,
                     c->shape.num_participants, c->shape.obs_embedding_size, in->ctx, in->part,
                     out->winner && out->outcome ? out->winner : nullptr, out->item,
                     out->winner && out->outcome ? out->outcome : nullptr, out->winner_outcome, c->d_akind, s->key, s->x, s->capacity,
                     (unsigned long long *)s->count);
  AG_HIP(hipGetLastError());
  return AG_OK;
}

// The won samples of a store bucketed by agent into the workspace (w.key, w.x with stride
// w.cap; w.offsets [N + 1]): histogram -> exclusive scan -> scatter. Shared by ag_lrts_update
// and ag_lrts_rp_begin. Synchronises for the count.
static int bucket_samples(ag_ctx *c, const ag_lrts_samples *s, hipStream_t st, const char *who) {
  const int N = c->shape.num_agents, Do = c->shape.obs_embedding_size + 1;
  uint64_t n = 0;
  AG_HIP(hipMemcpyAsync(&n, s->count, sizeof n, hipMemcpyDeviceToHost, st));
  AG_HIP(hipStreamSynchronize(st));
  if ((int64_t)n > s->capacity)
    return ag_set_error(AG_ERR_INVALID, "%s: %llu won samples overflowed the store (capacity %lld)",
                        who, (unsigned long long)n, (long long)s->capacity);
  ag_lrts_ws &w = c->lrts;
  if (!w.adam_tab) {
    double *tab = new double[2 * kLrEpochs];
    for (int t = 0; t < kLrEpochs; ++t) {  // torch.optim.Adam: Python floats, libm pow
      tab[t] = 1.0 - pow(0.9, (double)(t + 1));
      tab[kLrEpochs + t] = pow(1.0 - pow(0.999, (double)(t + 1)), 0.5);
    }
    hipError_t e = hipMalloc(&w.adam_tab, sizeof(double) * 2 * kLrEpochs);
    if (e == hipSuccess) e = hipMemcpy(w.adam_tab, tab, sizeof(double) * 2 * kLrEpochs, hipMemcpyHostToDevice);
    delete[] tab;
    if (e == hipSuccess) e = hipMalloc(&w.offsets, sizeof(int64_t) * (3 * (size_t)N + 1));
    if (e == hipSuccess) e = hipMalloc(&w.epochs, sizeof(int32_t) * N);
    if (e != hipSuccess) {
      ag_lrts_release(c);
      return ag_set_error(AG_ERR_HIP, "%s: workspace: %s", who, hipGetErrorString(e));
    }
  }
  if ((int64_t)n > w.cap) {
    (void)hipFree(w.key);
    (void)hipFree(w.x);
    w.key = nullptr;
    w.x = nullptr;
    const int64_t cap = (int64_t)n + ((int64_t)n >> 2) + 1024;
    hipError_t e = hipMalloc(&w.key, sizeof(uint32_t) * cap);
    if (e == hipSuccess) e = hipMalloc(&w.x, sizeof(float) * (size_t)Do * cap);
    if (e != hipSuccess) {
      w.cap = 0;
      return ag_set_error(AG_ERR_HIP, "%s: sample workspace: %s", who, hipGetErrorString(e));
    }
    w.cap = cap;
  }
  int64_t *counts = w.offsets + N + 1, *cursors = counts + N;
  AG_HIP(hipMemsetAsync(counts, 0, sizeof(int64_t) * N, st));
  if (n > 0) {
    if ((size_t)N * 4 > 64 * 1024)
      return ag_set_error(AG_ERR_UNSUPPORTED, "%s: N=%d agents > 16384", who, N);
    hipLaunchKernelGGL(k_lrts_hist, dim3(grid_over((int64_t)n)), dim3(kLrThreads), (size_t)N * 4, st, s->key,
                       (int64_t)n, N, counts);
    AG_HIP(hipGetLastError());
  }
  hipLaunchKernelGGL(k_lrts_scan, dim3(1), dim3(kLrThreads), 0, st, counts, N, w.offsets, cursors);
  AG_HIP(hipGetLastError());
  if (n > 0) {
    hipLaunchKernelGGL(k_lrts_scatter, dim3(grid_over((int64_t)n)), dim3(kLrThreads), 0, st, s->key, s->x,
                       (int64_t)n, s->capacity, Do, cursors, w.key, w.x, w.cap);
    AG_HIP(hipGetLastError());
  }
  return AG_OK;
}

int ag_lrts_update(ag_ctx *c, const ag_lrts_samples *s, int32_t *epochs, float *loss_trace, void *stream) {
  if (int rc = check_store(c, s, "ag_lrts_update")) return rc;
  if (!c->has_lrts) return AG_OK;
  if (!c->lrts_loaded) return ag_set_error(AG_ERR_STATE, "ag_lrts_update: ag_load_lrts not called");
  const int N = c->shape.num_agents, K = c->shape.num_items, Do = c->shape.obs_embedding_size + 1;
  TrainKernel train = pick_train(Do);
  if (!train || K * Do > kLrMaxKD)
    return ag_set_error(AG_ERR_UNSUPPORTED, "ag_lrts_update: needs OE+1 <= %d and K*(OE+1) <= %d (K=%d, OE+1=%d)",
                        AG_LRTS_MAX_DO, kLrMaxKD, K, Do);
  AgDeviceGuard g(c->device);
  hipStream_t st = (hipStream_t)stream;
  if (int rc = bucket_samples(c, s, st, "ag_lrts_update")) return rc;
  ag_lrts_ws &w = c->lrts;
  // agents' sample counts -> workgroups per agent (kLrCache samples per lane each)
  int64_t *h_off = new int64_t[N + 1];
  hipError_t e = hipMemcpyAsync(h_off, w.offsets, sizeof(int64_t) * (N + 1), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) {
    delete[] h_off;
    return ag_set_error(AG_ERR_HIP, "ag_lrts_update: %s", hipGetErrorString(e));
  }
  const size_t lds = sizeof(int64_t) * (size_t)K * Do * kAccStride;
  AG_HIP(hipFuncSetAttribute((const void *)train, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  if (!w.coop_blocks) {
    int per_cu = 0, cus = 0;
    AG_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)train, kLrThreads, lds));
    AG_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device));
    w.coop_blocks = per_cu * cus > 0 ? per_cu * cus : 1;
  }
  std::vector<int32_t> nblk(N, 0), blk_agent, blk_rank;
  std::vector<int64_t> pbase(N, 0);
  int64_t want = 0;
  int agents = 0;
  const int64_t chunk = c->lrts_chunk > 0 ? c->lrts_chunk : (int64_t)kLrCache * kLrThreads;
  for (int a = 0; a < N; ++a) {
    const int64_t na = h_off[a + 1] - h_off[a];
    if (c->h_akind[a] != AG_ALLOCATOR_LRTS || na < 2) continue;
    nblk[a] = (int32_t)((na + chunk - 1) / chunk);
    want += nblk[a];
    ++agents;
  }
  delete[] h_off;
  if (want > w.coop_blocks) {  // more samples than the resident grid caches: share it out
    const double f = (double)w.coop_blocks / (double)want;
    want = 0;
    for (int a = 0; a < N; ++a)
      if (nblk[a] > 0) {
        nblk[a] = (int32_t)(nblk[a] * f) > 1 ? (int32_t)(nblk[a] * f) : 1;
        want += nblk[a];
      }
  }
  int64_t pwords = 0;
  int lines = 0;
  std::vector<int32_t> bar_off(N, 0);
  bool multi = false;
  for (int a = 0; a < N; ++a) {
    bar_off[a] = lines;
    lines += agcoop::bar_lines(nblk[a]);
    pbase[a] = pwords;
    pwords += (int64_t)agcoop::bar_lines(nblk[a]) * kLrAccStride;
    multi |= nblk[a] > 1;
    for (int r = 0; r < nblk[a]; ++r) {
      blk_agent.push_back(a);
      blk_rank.push_back(r);
    }
  }
  AG_HIP(hipMemsetAsync(w.epochs, 0, sizeof(int32_t) * N, st));
  const int G = (int)blk_agent.size();
  if (G > 0) {
    if (multi && G > w.coop_blocks)
      return ag_set_error(AG_ERR_UNSUPPORTED, "ag_lrts_update: %d agents need more co-resident workgroups "
                                              "(%d) than the device holds (%d)", agents, G, w.coop_blocks);
    if ((size_t)G > w.tab_cap || (size_t)pwords > w.part_cap || (size_t)lines > w.bar_cap) {
      (void)hipFree(w.tables);
      (void)hipFree(w.partials);
      w.tables = nullptr;
      w.partials = nullptr;
      w.tab_cap = (size_t)G + 256;
      w.part_cap = (size_t)pwords + 4096;
      w.bar_cap = (size_t)lines + 64;
      hipError_t e2 = hipMalloc(&w.tables, sizeof(int64_t) * (w.tab_cap + 2 * (size_t)N) + sizeof(int32_t) * N +
                                               sizeof(unsigned) * agcoop::kBarLineWords * w.bar_cap);
      if (e2 == hipSuccess) e2 = hipMalloc(&w.partials, sizeof(int64_t) * w.part_cap);
      if (e2 != hipSuccess) {
        w.tab_cap = w.part_cap = w.bar_cap = 0;
        return ag_set_error(AG_ERR_HIP, "ag_lrts_update: tables: %s", hipGetErrorString(e2));
      }
    }
    // tables: blk_agent [G] i32, blk_rank [G] i32, agent_nblk [N] i32, agent_pbase [N] i64,
    // bar_off [N] i32, barrier lines [lines][32] u32 (all inside w.tables)
    char *tb = (char *)w.tables;
    int32_t *d_bagent = (int32_t *)tb;
    int32_t *d_brank = d_bagent + w.tab_cap;
    int32_t *d_nblk = d_brank + w.tab_cap;
    int64_t *d_pbase = (int64_t *)(d_nblk + 2 * (size_t)N);  // 8-B aligned (even count of i32 before)
    int32_t *d_baroff = (int32_t *)(d_pbase + N);
    unsigned *d_bar = (unsigned *)(d_baroff + N);
    AG_HIP(hipMemcpyAsync(d_bagent, blk_agent.data(), sizeof(int32_t) * G, hipMemcpyHostToDevice, st));
    AG_HIP(hipMemcpyAsync(d_brank, blk_rank.data(), sizeof(int32_t) * G, hipMemcpyHostToDevice, st));
    AG_HIP(hipMemcpyAsync(d_nblk, nblk.data(), sizeof(int32_t) * N, hipMemcpyHostToDevice, st));
    AG_HIP(hipMemcpyAsync(d_pbase, pbase.data(), sizeof(int64_t) * N, hipMemcpyHostToDevice, st));
    AG_HIP(hipMemcpyAsync(d_baroff, bar_off.data(), sizeof(int32_t) * N, hipMemcpyHostToDevice, st));
    if (lines) AG_HIP(hipMemsetAsync(d_bar, 0, sizeof(unsigned) * agcoop::kBarLineWords * lines, st));
    if (pwords) AG_HIP(hipMemsetAsync(w.partials, 0, sizeof(int64_t) * pwords, st));  // accumulator rows
    int Kv = K;
    const int32_t *cbagent = d_bagent, *cbrank = d_brank, *cnblk = d_nblk;
    const int64_t *cpbase = d_pbase, *coffsets = w.offsets;
    const uint32_t *ckey = w.key;
    const float *cx = w.x;
    int64_t ccap = w.cap;
    float *gm = c->d_tsm, *gq = c->d_tsq, *gpm = c->d_tsprev;
    const double *ctab = w.adam_tab;
    int32_t *cep = w.epochs;
    float *ctr = loss_trace;
    int64_t *cpart = w.partials;
    unsigned *cbar = d_bar;
    const int32_t *cbaroff = d_baroff;
    void *args[] = {&Kv, &cbagent, &cbrank, &cnblk, &cpbase, &coffsets, &ckey, &cx, &ccap, &gm, &gq, &gpm,
                    &ctab, &cep, &ctr, &cpart, &cbar, &cbaroff};
    if (multi)  // workgroups of one agent wait for each other: they must all be resident
      AG_HIP(hipLaunchCooperativeKernel((const void *)train, dim3(G), dim3(kLrThreads), args, (unsigned)lds, st));
    else
      AG_HIP(hipLaunchKernel((const void *)train, dim3(G), dim3(kLrThreads), args, lds, st));
  }
  if (epochs) {
    AG_HIP(hipMemcpyAsync(epochs, w.epochs, sizeof(int32_t) * N, hipMemcpyDeviceToHost, st));
    AG_HIP(hipStreamSynchronize(st));
  }
  return AG_OK;
}

// ---- resumable / record-parallel LR-TS training (k_lrts_epoch) ----
int ag_lrts_rp_begin(ag_ctx *c, const ag_lrts_samples *s, const int32_t *agents, const int64_t *samples_total,
                     int64_t *totals, void *stream) {
  if (int rc = check_store(c, s, "ag_lrts_rp_begin")) return rc;
  if (!totals) return ag_set_error(AG_ERR_INVALID, "ag_lrts_rp_begin: null totals");
  if (!c->lrts_loaded) return ag_set_error(AG_ERR_STATE, "ag_lrts_rp_begin: ag_load_lrts not called");
  const int N = c->shape.num_agents, K = c->shape.num_items, Do = c->shape.obs_embedding_size + 1;
  EpochKernel kern = pick_epoch(Do);
  if (!kern || K * Do > kLrMaxKD)
    return ag_set_error(AG_ERR_UNSUPPORTED, "ag_lrts_rp_begin: needs OE+1 <= %d and K*(OE+1) <= %d", AG_LRTS_MAX_DO,
                        kLrMaxKD);
  AgDeviceGuard g(c->device);
  hipStream_t st = (hipStream_t)stream;
  if (int rc = bucket_samples(c, s, st, "ag_lrts_rp_begin")) return rc;
  ag_lrts_ws &w = c->lrts;
  auto &rp = w.rp;
  std::vector<int64_t> off((size_t)N + 1);
  AG_HIP(hipMemcpyAsync(off.data(), w.offsets, sizeof(int64_t) * (N + 1), hipMemcpyDeviceToHost, st));
  AG_HIP(hipStreamSynchronize(st));
  // agents trained: LR-TS allocators in the mask with >= 2 won samples over all ranks (the
  // reference skips the update below that, src/BidderAllocation.py:33-34)
  constexpr int64_t kRpChunk = 2048;
  std::vector<int32_t> mask(N, 0), nblk(N, 0), blk_agent, blk_rank, bar_off(N, 0);
  int lines = 0;
  for (int a = 0; a < N; ++a) {
    const int64_t na = off[a + 1] - off[a], nt = samples_total ? samples_total[a] : na;
    if (c->h_akind[a] != AG_ALLOCATOR_LRTS || (agents && !agents[a]) || nt < 2) continue;
    mask[a] = 1;
    nblk[a] = (int32_t)std::max<int64_t>(1, (na + kRpChunk - 1) / kRpChunk);
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
    AG_HIP(hipMalloc(&rp.st, sizeof(LrSt) * 2 * (size_t)N));
    AG_HIP(hipMalloc(&rp.acc, sizeof(int64_t) * kLrAccStride * cap_lines + sizeof(unsigned) * 32 * cap_lines));
    AG_HIP(hipMalloc(&rp.tables, sizeof(int32_t) * (2 * cap_g + 3 * (size_t)N)));
    rp.cap_g = cap_g;
    rp.cap_lines = cap_lines;
  }
  rp.bar = (unsigned *)(rp.acc + kLrAccStride * rp.cap_lines);
  int32_t *d_bagent = rp.tables, *d_brank = d_bagent + rp.cap_g, *d_nblk = d_brank + rp.cap_g,
          *d_baroff = d_nblk + N, *d_mask = d_baroff + N;
  if (G) {
    AG_HIP(hipMemcpyAsync(d_bagent, blk_agent.data(), sizeof(int32_t) * G, hipMemcpyHostToDevice, st));
    AG_HIP(hipMemcpyAsync(d_brank, blk_rank.data(), sizeof(int32_t) * G, hipMemcpyHostToDevice, st));
  }
  AG_HIP(hipMemcpyAsync(d_nblk, nblk.data(), sizeof(int32_t) * N, hipMemcpyHostToDevice, st));
  AG_HIP(hipMemcpyAsync(d_baroff, bar_off.data(), sizeof(int32_t) * N, hipMemcpyHostToDevice, st));
  AG_HIP(hipMemcpyAsync(d_mask, mask.data(), sizeof(int32_t) * N, hipMemcpyHostToDevice, st));
  AG_HIP(hipMemsetAsync(rp.acc, 0, sizeof(int64_t) * kLrAccStride * rp.cap_lines + sizeof(unsigned) * 32 * rp.cap_lines,
                        st));
  AG_HIP(hipMemsetAsync(totals, 0, sizeof(int64_t) * 2 * kLrAccStride * (size_t)N, st));
  AG_HIP(hipMemsetAsync(w.epochs, 0, sizeof(int32_t) * N, st));
  hipLaunchKernelGGL(k_lrts_rp_init, dim3(N), dim3(64), 0, st, N, K * Do, d_mask, c->d_tsm, (LrSt *)rp.st);
  AG_HIP(hipGetLastError());
  const size_t lds = sizeof(int64_t) * (size_t)K * Do * kAccStride;
  AG_HIP(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  rp.G = G;
  rp.k = 0;
  rp.totals = totals;
  rp.active = true;
  return AG_OK;
}

int ag_lrts_rp_epoch(ag_ctx *c, int32_t launches, int64_t *launch_index, void *stream) {
  if (!c || !c->lrts.rp.active) return ag_set_error(AG_ERR_STATE, "ag_lrts_rp_epoch: no ag_lrts_rp_begin");
  if (launches < 0) return ag_set_error(AG_ERR_INVALID, "ag_lrts_rp_epoch: launches < 0");
  AgDeviceGuard g(c->device);
  const int N = c->shape.num_agents, K = c->shape.num_items, Do = c->shape.obs_embedding_size + 1;
  ag_lrts_ws &w = c->lrts;
  auto &rp = w.rp;
  EpochKernel kern = pick_epoch(Do);
  const size_t lds = sizeof(int64_t) * (size_t)K * Do * kAccStride;
  int32_t *d_bagent = rp.tables, *d_brank = d_bagent + rp.cap_g, *d_nblk = d_brank + rp.cap_g, *d_baroff = d_nblk + N;
  LrSt *S = (LrSt *)rp.st;
  hipStream_t st = (hipStream_t)stream;
  for (int32_t l = 0; l < launches; ++l) {
    const int64_t k = rp.k;
    if (rp.G > 0)
      hipLaunchKernelGGL(kern, dim3(rp.G), dim3(kLrThreads), lds, st, K, d_bagent, d_brank, d_nblk, w.offsets, w.key,
                         w.x, w.cap, c->d_tsm, c->d_tsq, c->d_tsprev, w.adam_tab, w.epochs, S + (size_t)(k & 1) * N,
                         S + (size_t)((k + 1) & 1) * N, rp.totals + (size_t)((k + 1) & 1) * kLrAccStride * N,
                         rp.totals + (size_t)(k & 1) * kLrAccStride * N, rp.acc, rp.bar, d_baroff);
    AG_HIP(hipGetLastError());
    rp.k = k + 1;
  }
  if (launch_index) *launch_index = rp.k - 1;
  return AG_OK;
}

int ag_lrts_rp_poll(ag_ctx *c, int32_t *training, void *stream) {
  if (!c || !c->lrts.rp.active) return ag_set_error(AG_ERR_STATE, "ag_lrts_rp_poll: no ag_lrts_rp_begin");
  AgDeviceGuard g(c->device);
  const int N = c->shape.num_agents;
  auto &rp = c->lrts.rp;
  hipStream_t st = (hipStream_t)stream;
  std::vector<int32_t> ph(N);
  // the phase word of every agent's latest state (LrSt starts with it)
  AG_HIP(hipMemcpy2DAsync(ph.data(), sizeof(int32_t), (LrSt *)rp.st + (size_t)(rp.k & 1) * N, sizeof(LrSt),
                          sizeof(int32_t), N, hipMemcpyDeviceToHost, st));
  AG_HIP(hipStreamSynchronize(st));
  int32_t n = 0;
  for (int a = 0; a < N; ++a) n += ph[a] != kLrDone;
  if (training) *training = n;
  return AG_OK;
}

int ag_lrts_rp_end(ag_ctx *c, int32_t *epochs, void *stream) {
  if (!c || !c->lrts.rp.active) return ag_set_error(AG_ERR_STATE, "ag_lrts_rp_end: no ag_lrts_rp_begin");
  int32_t training = 0;
  if (int rc = ag_lrts_rp_poll(c, &training, stream)) return rc;
  c->lrts.rp.active = false;
  if (training) return ag_set_error(AG_ERR_STATE, "ag_lrts_rp_end: %d agents still training", training);
  if (epochs) {
    AG_HIP(hipMemcpyAsync(epochs, c->lrts.epochs, sizeof(int32_t) * c->shape.num_agents, hipMemcpyDeviceToHost,
                          (hipStream_t)stream));
    AG_HIP(hipStreamSynchronize((hipStream_t)stream));
  }
  return AG_OK;
}

int ag_lrts_read(ag_ctx *c, float *m, float *q, float *prev_m) {
  if (!c) return ag_set_error(AG_ERR_INVALID, "ag_lrts_read: null ctx");
  AgDeviceGuard g(c->device);
  const size_t n = (size_t)c->shape.num_agents * c->shape.num_items * (c->shape.obs_embedding_size + 1);
  AG_HIP(hipDeviceSynchronize());
  if (m) AG_HIP(hipMemcpy(m, c->d_tsm, n * sizeof(float), hipMemcpyDeviceToHost));
  if (q) AG_HIP(hipMemcpy(q, c->d_tsq, n * sizeof(float), hipMemcpyDeviceToHost));
  if (prev_m) AG_HIP(hipMemcpy(prev_m, c->d_tsprev, n * sizeof(float), hipMemcpyDeviceToHost));
  return AG_OK;
}

}  // extern "C"
