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

#include <algorithm>
#include <string>

#include "ag_host.h"
#include "ag_philox.h"
#include "ag_sim.h"
#include "ag_sim_oracle.h"

#ifndef AG_SIM_WIDE_AB
#define AG_SIM_WIDE_AB 0  // AG_SIM_KERNEL_WIDE (the runtime-P kernel at any P): A/B variant builds only
#endif

// ------------------------------------------------------------------------------------
// error plumbing (declared in ag_host.h)
// ------------------------------------------------------------------------------------
static thread_local std::string g_last_error;

int ag_set_error(int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

namespace {
using namespace ag;

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

constexpr int kMaxGenE = 16;  // ag_generate: E <= 16 (the simulate kernels take E + 1 <= 16)

__global__ __launch_bounds__(kThreads) void k_generate(uint64_t seed, uint64_t first, int64_t B, int N, int P,
                                                      int E, double scale, double *ctx, int32_t *part,
                                                      double *u) {
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < B;
       i += (int64_t)gridDim.x * kThreads) {
    double x[kMaxGenE], uu;
    int picked[64];
    gen_auction<64, kMaxGenE>(k0, k1, first + (uint64_t)i, N, P, E, scale, x, picked, uu);
    u[i] = uu;
    for (int s = 0; s < P; ++s) part[(int64_t)s * B + i] = picked[s];
    for (int e = 0; e < E; ++e) ctx[(int64_t)e * B + i] = x[e];
  }
}

// Synthetic per-participant noise (ag_philox.h gen_normals4 / gen_normal1 / gen_shading_raw,
// which the general kernel's generate mode draws in place): shading bidders' gamma_raw =
// prev_gamma + sigma * z (numpy normal(loc, scale)), LR-TS agents' ts_noise = z * (1 / sqrt(q))
// (torch.normal(0, 1 / sqrt(q)), src/Models.py:31), fitted policies' rsample draws.
__global__ __launch_bounds__(kThreads) void k_generate_noise(uint64_t seed, uint64_t first, int64_t B, int P,
                                                            int KDo, const int32_t *part,
                                                            const int32_t *akind, const int32_t *bkind,
                                                            const double *pg, const double *gs,
                                                            const float *q, double *gamma_raw,
                                                            float *ts_noise, float *policy_eps,
                                                            const int32_t *ts_index) {
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  const int64_t T = (B + 63) >> 6;  // 64-auction tiles of ts_noise
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < B;
       i += (int64_t)gridDim.x * kThreads) {
    const uint64_t idx = first + (uint64_t)i;
    const uint32_t c0 = (uint32_t)idx, c1 = (uint32_t)(idx >> 32);
    for (int s = 0; s < P; ++s) {
      const int a = part[(int64_t)s * B + i];
      if (gamma_raw)
        gamma_raw[(int64_t)s * B + i] =
            bkind[a] != AG_BIDDER_TRUTHFUL ? gen_shading_raw(c0, c1, s, k0, k1, pg[a], gs[a]) : NAN;
      if (policy_eps)  // the rsample draw of a fitted policy
        policy_eps[(int64_t)s * B + i] = gen_normal1(c0, c1, 0, 16 + (uint32_t)s, k0, k1);
      if (ts_noise && (!ts_index || akind[a] == AG_ALLOCATOR_LRTS)) {
        const bool lr = akind[a] == AG_ALLOCATOR_LRTS;
        // dense tiles: pair (s, i) at s*T*64 + i; compact: the LR-TS pair's rank j
        const int64_t pj = ts_index ? (int64_t)(uint32_t)ts_index[(int64_t)s * B + i] : s * T * 64 + i;
        const float *qa = q + (size_t)a * KDo;
        for (int j = 0; j < KDo; j += 4) {
          float z[4] = {0.0f, 0.0f, 0.0f, 0.0f};
          if (lr) gen_normals4(c0, c1, (uint32_t)(j >> 2), 4 + (uint32_t)s, k0, k1, z);
          float *row = ts_noise + ((pj >> 6) * KDo + j) * 64 + (pj & 63);
          for (int t = 0; t < 4 && j + t < KDo; ++t) row[64 * t] = lr ? z[t] * (1.0f / sqrtf(qa[j + t])) : 0.0f;
        }
      }
    }
  }
}

// Compact Thompson-noise index (ag_ts_noise_index): the exclusive prefix count of LR-TS
// pairs in (slot, auction) order over [P][B] -- three passes: per-workgroup counts, one
// workgroup scanning the counts, per-workgroup local scans writing the ranks.
constexpr int kScanTile = kThreads * 4;  // pairs per workgroup
__device__ __forceinline__ int lrts_flag(const int32_t *part, const int32_t *akind, int64_t n, int64_t k) {
  return k < n && akind[part[k]] == AG_ALLOCATOR_LRTS;
}
__device__ __forceinline__ int block_excl_scan(int v, int *s_w, int &total) {
  // wave inclusive scan by DPP-free shuffles, then the waves' totals
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_w[wv] = x;
  __syncthreads();
  int base = 0, tot = 0;
  for (int w = 0; w < kThreads / 64; ++w) {
    if (w < wv) base += s_w[w];
    tot += s_w[w];
  }
  __syncthreads();
  total = tot;
  return base + x - v;
}
__global__ __launch_bounds__(kThreads) void k_ts_index_count(const int32_t *part, const int32_t *akind, int64_t n,
                                                            int64_t *counts) {
  __shared__ int s_w[kThreads / 64];
  const int64_t k0 = (int64_t)blockIdx.x * kScanTile + threadIdx.x * 4;
  int v = 0;
  for (int e = 0; e < 4; ++e) v += lrts_flag(part, akind, n, k0 + e);
  int tot;
  block_excl_scan(v, s_w, tot);
  if (threadIdx.x == 0) counts[blockIdx.x] = tot;
}
__global__ __launch_bounds__(kThreads) void k_ts_index_offsets(int64_t *counts, int64_t nb) {
  // one workgroup: exclusive scan of nb counts in place, counts[nb] = the total
  __shared__ int64_t s_run;
  if (threadIdx.x == 0) s_run = 0;
  __syncthreads();
  for (int64_t b0 = 0; b0 < nb; b0 += kThreads) {
    __shared__ int64_t s_v[kThreads];
    const int64_t b = b0 + threadIdx.x;
    s_v[threadIdx.x] = b < nb ? counts[b] : 0;
    __syncthreads();
    if (threadIdx.x == 0) {  // nb / kThreads rounds of a serial kThreads-long scan: tiny
      int64_t r = s_run;
      for (int t = 0; t < kThreads; ++t) {
        const int64_t c = s_v[t];
        s_v[t] = r;
        r += c;
      }
      s_run = r;
    }
    __syncthreads();
    if (b < nb) counts[b] = s_v[threadIdx.x];
    __syncthreads();
  }
  if (threadIdx.x == 0) counts[nb] = s_run;
}
__global__ __launch_bounds__(kThreads) void k_ts_index_write(const int32_t *part, const int32_t *akind, int64_t n,
                                                            const int64_t *offsets, int32_t *index) {
  __shared__ int s_w[kThreads / 64];
  const int64_t k0 = (int64_t)blockIdx.x * kScanTile + threadIdx.x * 4;
  int f[4], v = 0;
  for (int e = 0; e < 4; ++e) {
    f[e] = lrts_flag(part, akind, n, k0 + e);
    v += f[e];
  }
  int tot;
  int64_t r = offsets[blockIdx.x] + block_excl_scan(v, s_w, tot);
  for (int e = 0; e < 4; ++e)
    if (k0 + e < n) {
      index[k0 + e] = f[e] ? (int32_t)r : -1;
      r += f[e];
    }
}

// Synthetic search grids: U(0.1, 1) with 53-bit uniforms, streams 32 + slot (two per
// Philox block), grid point j of slot s of auction i at (s*128 + j)*B + i.
__global__ __launch_bounds__(kThreads) void k_generate_grid(uint64_t seed, uint64_t first, int64_t B, int P,
                                                           double *grid) {
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < B; i += (int64_t)gridDim.x * kThreads) {
    const uint64_t idx = first + (uint64_t)i;
    const uint32_t c0 = (uint32_t)idx, c1 = (uint32_t)(idx >> 32);
    for (int s = 0; s < P; ++s)
      for (int j = 0; j < 128; j += 2) {
        uint32_t w[4];
        philox(c0, c1, (uint32_t)(j >> 1), 32 + (uint32_t)s, k0, k1, w);
        const double u0 = (double)((((uint64_t)w[0] << 32) | w[1]) >> 11) * 0x1p-53;
        const double u1 = (double)((((uint64_t)w[2] << 32) | w[3]) >> 11) * 0x1p-53;
        grid[((int64_t)s * 128 + j) * B + i] = 0.1 + 0.9 * u0;
        grid[((int64_t)s * 128 + j + 1) * B + i] = 0.1 + 0.9 * u1;
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

// Streaming copy, one 16-B element per lane, non-temporal both ways, one tile per workgroup
// (bench.py's measured HBM peak: the fastest of the copy shapes tools/floor/copy_peak.py
// measured -- 6.6 TB/s against 5.0-6.0 for persistent grid-stride copies).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(kThreads) void k_stream_copy(const u32x4 *__restrict__ src, u32x4 *__restrict__ dst,
                                                          int64_t n16) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i < n16) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

// ------------------------------------------------------------------------------------
// dispatch
// ------------------------------------------------------------------------------------
SimKernel pick_kernel(int P, int D, bool prune, int W, int general, int bt) {
  if (P > kMaxP) return pick_kernel_for<0>(D, prune, W, general, bt);  // runtime-P kernel
  switch (P) {
    case 1: return pick_kernel_for<1>(D, prune, W, general, bt);
    case 2: return pick_kernel_for<2>(D, prune, W, general, bt);
    case 3: return pick_kernel_for<3>(D, prune, W, general, bt);
    case 4: return pick_kernel_for<4>(D, prune, W, general, bt);
    case 5: return pick_kernel_for<5>(D, prune, W, general, bt);
    case 6: return pick_kernel_for<6>(D, prune, W, general, bt);
    case 7: return pick_kernel_for<7>(D, prune, W, general, bt);
    case 8: return pick_kernel_for<8>(D, prune, W, general, bt);
    default: return nullptr;
  }
}

OraKernel pick_oracle(int P, int D, bool gen) {
  switch (P) {
    case 1: return pick_oracle_for<1>(D, gen);
    case 2: return pick_oracle_for<2>(D, gen);
    case 3: return pick_oracle_for<3>(D, gen);
    case 4: return pick_oracle_for<4>(D, gen);
    case 5: return pick_oracle_for<5>(D, gen);
    case 6: return pick_oracle_for<6>(D, gen);
    case 7: return pick_oracle_for<7>(D, gen);
    case 8: return pick_oracle_for<8>(D, gen);
    default: return nullptr;
  }
}

// Resident blocks of a kernel (grid of the persistent launches), capped by the partials
// workspace.
int resident_blocks(const ag_ctx *c, const void *k, size_t lds, int *out) {
  int per_cu = 0, cus = 0;
  AG_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, kThreads, lds));
  AG_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device));
  int res = per_cu * cus;
  if (res < 1) res = 1;
  if (res > c->partial_blocks) res = c->partial_blocks;
  *out = res;
  return AG_OK;
}

// ag_simulate for OracleAllocator + TruthfulBidder populations: k_oracle (ag_sim_oracle.h).
int simulate_oracle(ag_ctx *c, OraKernel k, int64_t B, const ag_batch_in *in, const ag_batch_out *out,
                    int64_t *counters_fx, hipStream_t st, uint64_t seed = 0, uint64_t first = 0) {
  const ag_shape &s = c->shape;
  OraParams prm;
  prm.B = (int32_t)B;
  prm.N = s.num_agents;
  prm.K = s.num_items;
  prm.mech = s.mechanism;
  prm.want_counters = counters_fx != nullptr;
  prm.L = make_ora_layout(s.num_agents, s.num_items, c->D, prm.want_counters);
  prm.items = c->d_items;
  prm.values = c->d_values;
  prm.ctx = in ? in->ctx : nullptr;
  prm.part = in ? in->part : nullptr;
  prm.u = in ? in->u : nullptr;
  prm.seed = seed;
  prm.first = first;
  prm.scale = s.embedding_var;
  prm.winner = out->winner;
  prm.price = out->price;
  prm.second_price = out->second_price;
  prm.outcome = out->outcome;
  prm.item = out->item;
  prm.bid = out->bid;
  prm.est_ctr = out->est_ctr;
  prm.true_ctr = out->true_ctr;
  prm.best_ev = out->best_ev;
  prm.winner_outcome = out->winner_outcome;
  prm.partials = c->d_partials;
  prm.queue = c->d_queue;
  const size_t lds = (size_t)prm.L.total;
  if (lds > 160 * 1024)
    return ag_set_error(AG_ERR_UNSUPPORTED, "ag_simulate: population needs %zu B of LDS (> 160 KiB)", lds);
  if (lds > 64 * 1024)
    AG_HIP(hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  int &res_max = c->resident_ora[(prm.want_counters ? 1 : 0) + (in ? 0 : 2)];
  if (res_max == 0)
    if (int rc = resident_blocks(c, (const void *)k, lds, &res_max)) return rc;
  // Persistent grid of kOraBlocksPerCu workgroups per CU, capped by residency
  // (AG_OPT_SIM_BLOCKS_PER_CU overrides). With the static stride fewer than the 5 the
  // registers allow streamed better (round 4: 4 per CU 0.473 ms vs 5 per CU 0.503 ms); with
  // the work counters (AG_ORA_QUEUE) all 5 do (3.57 -> 3.41 ms per 2^27, r05zm_ab_sub_bpc.log)
  int res = res_max;
  {
    // generate mode (no input stream, VALU-heavier): as many as fit (5 at 87 VGPRs) --
    // 4.02 -> 3.87 ms per 2^27 auctions (profiles/r05w_ab_gen.log)
    const int per_cu = c->grid_per_cu > 0 ? c->grid_per_cu : (in ? kOraBlocksPerCu : 8);
    int cus = 0;
    AG_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device));
    if ((int64_t)per_cu * cus < res) res = per_cu * cus;
  }
  // a lane resolves at most ora_lane_cap(R) auctions per launch (replica sums in range):
  // larger batches run as consecutive launches
  int64_t chunk_max = (int64_t)res * kThreads * ora_lane_cap(prm.L.replicas);
#if AG_ORA_QUEUE
  // a wave may take up to ora_lane_cap(R) auctions per lane; a launch holds half of what the
  // grid could take (every counter has as many waves), so the rest always finds a wave
  if (res >= 16) res &= ~15;
  chunk_max = (int64_t)res * kThreads * (ora_lane_cap(prm.L.replicas) / 2);
  prm.lane_tiles = (uint32_t)ora_lane_cap(prm.L.replicas);
#endif
  if (chunk_max > INT32_MAX) chunk_max = INT32_MAX;
  if (c->launch_cap > 0 && c->launch_cap < chunk_max) chunk_max = c->launch_cap;
  if (chunk_max < 1) chunk_max = 1;
  const int nc = s.num_agents * kC;
  for (int64_t lo = 0; lo < B; lo += chunk_max) {
    const int64_t hi = lo + chunk_max < B ? lo + chunk_max : B;
    const int64_t tiles = (hi - lo + kThreads - 1) / kThreads;
    int grid = (int)(tiles < res ? tiles : res);
#if AG_ORA_QUEUE
    // wave w of block b serves work counter (4 b + w) mod 64, and chunk c belongs to counter
    // c mod 64: every counter the launch's chunks reach needs a wave. A grid below 16 blocks
    // (a small device or partition: res < 16) covers only 4 * grid counters -- raise it (the
    // extra blocks wait for a CU; nothing in k_oracle waits on another block)
    const int64_t chunks = (hi - lo + 64 * AG_ORA_QUEUE_SUB - 1) / (64 * AG_ORA_QUEUE_SUB);
    if (grid < 16 && chunks > 4 * (int64_t)grid) grid = (int)std::min<int64_t>(16, (chunks + 3) / 4);
#endif
    prm.lo = (int32_t)lo;
    prm.hi = (int32_t)hi;
#if AG_ORA_QUEUE
    AG_HIP(hipMemsetAsync(c->d_queue, 0, sizeof(uint32_t) * 64 * 32, st));
#endif
    hipLaunchKernelGGL(k, dim3(grid), dim3(kThreads), lds, st, prm);  // generate mode: same lo/hi
    AG_HIP(hipGetLastError());
    if (counters_fx) {
      hipLaunchKernelGGL(k_reduce_counters, dim3(nc), dim3(kThreads), 0, st, c->d_partials, grid, nc, counters_fx);
      AG_HIP(hipGetLastError());
    }
  }
  return AG_OK;
}

// k_simulate over a batch (replay / HBM-resident inputs, or generate mode: gen, every input drawn
// in the kernel from (seed, first + auction index) as ag_generate + ag_generate_noise draw them)
int simulate_general(ag_ctx *c, int64_t B, const ag_batch_in *in, const ag_batch_out *out, int64_t *counters_fx,
                     hipStream_t st, bool gen, uint64_t seed, uint64_t first) {
  const ag_shape &s = c->shape;
  const int nc = s.num_agents * kC;
  const int D = c->D;
  const bool prune = c->item_search == AG_ITEM_SEARCH_AUTO && D <= 8 && s.num_items <= 2 * kMaxKPairs &&
                     c->values_positive;
  SimParams prm;
  prm.B = B;
  prm.N = s.num_agents;
  prm.K = s.num_items;
  prm.mech = s.mechanism;
  prm.want_counters = counters_fx != nullptr;
  prm.lds = make_layout(s.num_agents, s.num_items, D, prm.want_counters, c->general,
                        s.obs_embedding_size + 1, gen);
  prm.ts_sample = c->ts_sample;
  prm.akind = c->d_akind;
  prm.bkind = c->d_bkind;
  prm.pg = c->d_pg;
  prm.gs = c->d_gs;
  prm.tsm = c->d_tsm;
  prm.drs = c->dr_loaded ? c->dr.state : nullptr;
  prm.dri = c->dr_loaded ? c->dr.init : nullptr;
  prm.kag = c->ragged ? c->d_kag : nullptr;
  prm.items = c->d_items;
  prm.values = c->d_values;
  prm.in = in ? *in : ag_batch_in{};
  prm.out = *out;
  prm.partials = c->d_partials;
  prm.P = s.num_participants;
  prm.tsq = c->d_tsq;
  prm.seed = seed;
  prm.first = first;
  prm.scale = s.embedding_var;
  // (round 4 retired k_pop, the dedicated shipped-shape population kernel: k_simulate was as
  // fast or faster on every line, P = 8 included once its slots stream -- configs_1 at P = 8
  // 0.665 against 0.680 ms, profiles/r04k_ab_c1p8.log; at P = 2 on every line,
  // profiles/r03_ab_pop_vs_generic.log)
  int W = (prune && (B % 2) == 0 && c->wide && !c->general && s.num_participants <= kMaxP) ? 2 : 1;
  size_t lds = (size_t)prm.lds.total;
  if (lds > 160 * 1024)
    return ag_set_error(AG_ERR_UNSUPPORTED, "ag_simulate: population needs %zu B of LDS (> 160 KiB)", lds);
  // Lanes per workgroup: the LDS image (catalogue, screen, LR-TS means, counter replicas) is
  // per workgroup, so a large population with 256-lane workgroups keeps few waves resident
  // (N = 32: ~75 KB -> 2 workgroups = 2 waves per SIMD); 1024-lane workgroups share one
  // image among 16 waves. Same results (the counters are exact sums).
  int bt = c->block_threads;
  if (bt == 0) bt = (c->general && prune && lds > 40 * 1024) ? kLargeThreads : kThreads;
  // AG_OPT_SIM_GENERAL_MODE 0 (auto): TruthfulBidder-only populations take the build
  // without the bid-shading code (kGenTruthful); 1: always the full general build
  const int gmode = !c->general ? kGenOracle : (c->has_shading || c->gen_mode_all) ? kGenAll : kGenTruthful;
  // the shipped shape (E = 5, LR-TS width OE + 1 = 5 in the layout) has builds with the LR-TS
  // width compile-time (k_simulate's DOS); AG_OPT_SIM_SHIPPED_SHAPE 0 turns them off (A/B)
  const int ship = (c->general && c->ship_shape && D == 6 && prm.lds.ts_do == kShipDo) ? kGenShip : 0;
  // the full mix at P >= 3 in the large-image case: the streamed 768-lane build (shipped shape)
  if (bt == kLargeThreads && c->block_threads == 0 && gmode == kGenAll && ship && s.num_participants >= AG_STREAM_MIN_P &&
      s.num_participants <= kMaxP)
    bt = kMidThreads;
  const int genb = gen ? kGenGen : 0;  // generate mode: the shipped shape's GEN builds
  SimKernel k = pick_kernel(s.num_participants, D, prune, W, gmode | ship | genb, bt);
  if (!k && bt == kMidThreads) {
    bt = kLargeThreads;
    k = pick_kernel(s.num_participants, D, prune, W, gmode | ship | genb, bt);
  }
  if (!k && W == 2) {  // the two-auctions-per-lane build is an A/B variant only (AG_LANE_PAIRS)
    W = 1;
    k = pick_kernel(s.num_participants, D, prune, W, gmode | ship | genb, bt);
  }
  if (!k && bt != kThreads) {
    bt = kThreads;
    k = pick_kernel(s.num_participants, D, prune, W, gmode | ship | genb, bt);
  }
  bool wide_ab = false;
#if AG_SIM_WIDE_AB
  if (c->general && c->sim_kernel == AG_SIM_KERNEL_WIDE) {  // the runtime-P kernel at any P (A/B)
    bt = kThreads;
    k = pick_kernel_for<0>(D, prune, 1, kGenAll, kThreads);
    wide_ab = true;
  }
#endif
  if (!k && gen)
    return ag_set_error(AG_ERR_UNSUPPORTED,
                        "ag_simulate_generated: general populations in the shipped shape only (E = 5, OE = 4, "
                        "K <= %d, positive catalogue values, P <= %d; P=%d D=%d)",
                        2 * kMaxKPairs, kMaxP, s.num_participants, D);
  if (!k) return ag_set_error(AG_ERR_UNSUPPORTED, "ag_simulate: no kernel for P=%d D=%d", s.num_participants, D);
  if (gmode == kGenAll && bt == kLargeThreads) {  // the compacted fitted-policy pass's per-wave task slots
    add_policy_tasks(prm.lds, bt);
    lds = (size_t)prm.lds.total;
    if (lds > 160 * 1024)
      return ag_set_error(AG_ERR_UNSUPPORTED, "ag_simulate: population needs %zu B of LDS (> 160 KiB)", lds);
  }
  // Persistent grid: exactly the blocks the device keeps resident (no partial last round),
  // each striding over bt-auction tiles.
  // (the WIDE A/B kernel has slots of its own: its occupancy is not the AUTO kernel's)
  int &res = wide_ab ? c->resident_wide[prm.want_counters ? 1 : 0]
                     : c->resident[(gen ? 256 : 0) + (bt == kMidThreads ? 128 : 0) + (ship ? 64 : 0) +
                                   (gmode == kGenTruthful ? 32 : 0) +
                                   (bt == kThreads ? 0 : 16) + (c->general ? 8 : 0) + (W == 2 ? 4 : 0) +
                                   (prune ? 2 : 0) + (prm.want_counters ? 1 : 0)];
  if (res == 0) {  // first launch of this build: the kernel's static LDS (AG_TS_DMA's noise rings) on top
    hipFuncAttributes fa;
    AG_HIP(hipFuncGetAttributes(&fa, (const void *)k));
    if (lds + fa.sharedSizeBytes > 160 * 1024)
      return ag_set_error(AG_ERR_UNSUPPORTED, "ag_simulate: population needs %zu + %zu B of LDS (> 160 KiB)", lds,
                          (size_t)fa.sharedSizeBytes);
  }
  if (lds > 64 * 1024)
    AG_HIP(hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  if (res == 0) {
    int per_cu = 0, cus = 0;
    AG_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)k, bt, lds));
    AG_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device));
    res = per_cu * cus;
    if (res < 1) res = 1;
    if (res > c->partial_blocks) res = c->partial_blocks;
  }
  // AG_OPT_SIM_BLOCKS_PER_CU caps the grid below residency (A/B; 0 = every resident block)
  int grid_max = res;
  if (c->grid_per_cu > 0) {
    int cus = 0;
    AG_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device));
    if ((int64_t)c->grid_per_cu * cus < grid_max) grid_max = c->grid_per_cu * cus;
  }
  // Batches larger than one launch's exact-counter capacity (resident blocks x
  // kAuctionsPerReplica x replicas) run as consecutive launches over auction ranges.
  const int64_t per_block = (int64_t)kAuctionsPerReplica * prm.lds.replicas;
  int64_t chunk_max = (int64_t)grid_max * per_block;
  if (c->launch_cap > 0 && c->launch_cap < chunk_max) chunk_max = c->launch_cap;
  chunk_max &= ~(int64_t)1;
  if (chunk_max < 2) chunk_max = 2;
  for (int64_t lo = 0; lo < B; lo += chunk_max) {
    const int64_t hi = lo + chunk_max < B ? lo + chunk_max : B;
    const int64_t tiles = (hi - lo + bt * W - 1) / (bt * W);
    const int grid = (int)(tiles < grid_max ? tiles : grid_max);
    prm.lo = (int32_t)lo;
    prm.hi = (int32_t)hi;
    hipLaunchKernelGGL(k, dim3(grid), dim3(bt), lds, st, prm);  // generate mode: same lo/hi
    AG_HIP(hipGetLastError());
    if (counters_fx) {
      hipLaunchKernelGGL(k_reduce_counters, dim3(nc), dim3(kThreads), 0, st, c->d_partials, grid, nc,
                         counters_fx);
      AG_HIP(hipGetLastError());
    }
  }
  return AG_OK;
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
extern "C" {

const char *ag_last_error(void) { return g_last_error.c_str(); }
int32_t ag_abi_version(void) { return AG_ABI_VERSION; }

int ag_create(int32_t device, const ag_shape *s, ag_ctx **out) {
  if (!s || !out) return ag_set_error(AG_ERR_INVALID, "ag_create: null argument");
  *out = nullptr;
  if (s->num_agents < 1 || s->num_items < 1 || s->embedding_size < 1)
    return ag_set_error(AG_ERR_INVALID, "ag_create: N, K, E must be >= 1 (N=%d K=%d E=%d)",
                     s->num_agents, s->num_items, s->embedding_size);
  if (s->num_participants < 1 || s->num_participants > s->num_agents)
    return ag_set_error(AG_ERR_INVALID,
                     "ag_create: Cannot take a larger sample than population when replace is "
                     "False (P=%d, N=%d; src/Auction.py:42)",
                     s->num_participants, s->num_agents);
  if (s->mechanism != AG_FIRST_PRICE && s->mechanism != AG_SECOND_PRICE)
    return ag_set_error(AG_ERR_INVALID, "ag_create: unknown mechanism %d", s->mechanism);
  if (s->num_slots != 1)
    return ag_set_error(AG_ERR_UNSUPPORTED, "ag_create: num_slots must be 1 (src/main.py:37)");
  const int D = s->embedding_size + 1;
  if (s->num_participants > 4096)
    return ag_set_error(AG_ERR_UNSUPPORTED, "ag_create: P=%d > 4096", s->num_participants);
  if (s->obs_embedding_size < 0 || s->obs_embedding_size > s->embedding_size)
    return ag_set_error(AG_ERR_INVALID, "ag_create: obs_embedding_size out of range");
  ag_ctx *c = new ag_ctx();
  c->device = device;
  c->shape = *s;
  c->D = D;
  const int nc = s->num_agents * kC;
  // simulate needs a kernel for (P, D) and the catalogue in LDS; allocate-only contexts
  // (any P) do not.
  const LdsLayout lay = make_layout(s->num_agents, s->num_items, D, true);
  c->can_simulate = pick_kernel(s->num_participants, D, false, 1, false, kThreads) &&
                    lay.total <= 160 * 1024;
  AgDeviceGuard g(device);
  hipError_t e = hipMalloc(&c->d_items, sizeof(double) * s->num_agents * s->num_items * D);
  if (e == hipSuccess) e = hipMalloc(&c->d_values, sizeof(double) * s->num_agents * s->num_items);
  // partials for the largest grid a call can use: grids grow past kMinGrid only to keep
  // <= kAuctionsPerReplica * replicas auctions per block; allocate lazily beyond the default.
  c->partial_blocks = kMaxSimGrid;
  if (e == hipSuccess) e = hipMalloc(&c->d_partials, sizeof(int64_t) * 2 * (size_t)kMaxSimGrid * nc);
  const size_t nkd = (size_t)s->num_agents * s->num_items * (s->obs_embedding_size + 1);
  if (e == hipSuccess) e = hipMalloc(&c->d_akind, sizeof(int32_t) * s->num_agents);
  if (e == hipSuccess) e = hipMalloc(&c->d_bkind, sizeof(int32_t) * s->num_agents);
  if (e == hipSuccess) e = hipMalloc(&c->d_pg, sizeof(double) * s->num_agents);
  if (e == hipSuccess) e = hipMalloc(&c->d_gs, sizeof(double) * s->num_agents);
  if (e == hipSuccess) e = hipMalloc(&c->d_tsm, sizeof(float) * nkd);
  if (e == hipSuccess) e = hipMalloc(&c->d_tsq, sizeof(float) * nkd);
  if (e == hipSuccess) e = hipMalloc(&c->d_tsprev, sizeof(float) * nkd);
  if (e == hipSuccess) e = hipMalloc(&c->d_queue, sizeof(uint32_t) * 64 * 32);
  if (e != hipSuccess) {
    (void)hipFree(c->d_queue);
    (void)hipFree(c->d_items);
    (void)hipFree(c->d_values);
    (void)hipFree(c->d_partials);
    (void)hipFree(c->d_akind);
    (void)hipFree(c->d_bkind);
    (void)hipFree(c->d_pg);
    (void)hipFree(c->d_gs);
    (void)hipFree(c->d_tsm);
    (void)hipFree(c->d_tsq);
    (void)hipFree(c->d_tsprev);
    delete c;
    return ag_set_error(AG_ERR_HIP, "ag_create: hipMalloc: %s", hipGetErrorString(e));
  }
  *out = c;
  return AG_OK;
}

int ag_destroy(ag_ctx *c) {
  if (!c) return AG_OK;
  AgDeviceGuard g(c->device);
  (void)hipFree(c->d_items);
  (void)hipFree(c->d_values);
  (void)hipFree(c->d_partials);
  (void)hipFree(c->d_queue);
  (void)hipFree(c->d_akind);
  (void)hipFree(c->d_bkind);
  (void)hipFree(c->d_kag);
  (void)hipFree(c->d_pg);
  (void)hipFree(c->d_gs);
  (void)hipFree(c->d_tsm);
  (void)hipFree(c->d_tsq);
  (void)hipFree(c->d_tsprev);
  ag_lrts_release(c);
  ag_dr_release(c);
  (void)hipFree(c->d_status);
  delete[] c->h_akind;
  delete[] c->h_bkind;
  delete c;
  return AG_OK;
}

int ag_set_agent_items(ag_ctx *c, const int32_t *num_items) {
  if (!c) return ag_set_error(AG_ERR_INVALID, "ag_set_agent_items: null ctx");
  const int N = c->shape.num_agents, K = c->shape.num_items;
  bool ragged = false;
  for (int a = 0; num_items && a < N; ++a) {
    if (num_items[a] < 1 || num_items[a] > K)
      return ag_set_error(AG_ERR_INVALID, "ag_set_agent_items: agent %d has %d items, not in [1, K = %d]", a,
                          num_items[a], K);
    ragged |= num_items[a] < K;
  }
  AgDeviceGuard g(c->device);
  if (ragged) {
    if (!c->d_kag) AG_HIP(hipMalloc(&c->d_kag, sizeof(int32_t) * N));
    AG_HIP(hipMemcpy(c->d_kag, num_items, sizeof(int32_t) * N, hipMemcpyHostToDevice));
  }
  c->ragged = ragged;
  return AG_OK;
}

int ag_set_agent_params(ag_ctx *c, const int32_t *alloc_kind, const int32_t *bid_kind,
                        const double *prev_gamma, const double *gamma_sigma) {
  if (!c) return ag_set_error(AG_ERR_INVALID, "ag_set_agent_params: null ctx");
  const int N = c->shape.num_agents;
  bool general = false, lrts = false, shading = false;
  for (int a = 0; a < N; ++a) {
    const int ak = alloc_kind ? alloc_kind[a] : AG_ALLOCATOR_ORACLE;
    const int bk = bid_kind ? bid_kind[a] : AG_BIDDER_TRUTHFUL;
    if (ak != AG_ALLOCATOR_ORACLE && ak != AG_ALLOCATOR_LRTS)
      return ag_set_error(AG_ERR_UNSUPPORTED, "agent %d: allocator kind %d not implemented", a, ak);
    if (bk < AG_BIDDER_TRUTHFUL || bk > AG_BIDDER_DOUBLY_ROBUST)
      return ag_set_error(AG_ERR_UNSUPPORTED, "agent %d: bidder kind %d not implemented", a, bk);
    if (bk != AG_BIDDER_TRUTHFUL && (!prev_gamma || !gamma_sigma))
      return ag_set_error(AG_ERR_INVALID, "agent %d: shading bidder needs prev_gamma and gamma_sigma", a);
    if (bk != AG_BIDDER_TRUTHFUL && !(gamma_sigma[a] > 0.0))
      return ag_set_error(AG_ERR_INVALID, "agent %d: gamma_sigma must be > 0", a);
    lrts |= ak == AG_ALLOCATOR_LRTS;
    shading |= bk != AG_BIDDER_TRUTHFUL;
  }
  general = lrts || shading;
  if (general && (c->D > 8 || c->shape.obs_embedding_size + 1 > kMaxD))
    return ag_set_error(AG_ERR_UNSUPPORTED, "general populations support E+1 <= 8 (D=%d)", c->D);
  AgDeviceGuard g(c->device);
  int32_t *ak = new int32_t[N], *bk = new int32_t[N];
  double *pg = new double[N], *gs = new double[N];
  for (int a = 0; a < N; ++a) {
    ak[a] = alloc_kind ? alloc_kind[a] : AG_ALLOCATOR_ORACLE;
    bk[a] = bid_kind ? bid_kind[a] : AG_BIDDER_TRUTHFUL;
    pg[a] = prev_gamma ? prev_gamma[a] : 1.0;
    gs[a] = gamma_sigma ? gamma_sigma[a] : 1.0;
  }
  hipError_t e = hipMemcpy(c->d_akind, ak, sizeof(int32_t) * N, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(c->d_bkind, bk, sizeof(int32_t) * N, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(c->d_pg, pg, sizeof(double) * N, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(c->d_gs, gs, sizeof(double) * N, hipMemcpyHostToDevice);
  delete[] pg;
  delete[] gs;
  if (e != hipSuccess) {
    delete[] ak;
    delete[] bk;
    return ag_set_error(AG_ERR_HIP, "ag_set_agent_params: %s", hipGetErrorString(e));
  }
  delete[] c->h_akind;
  c->h_akind = ak;
  delete[] c->h_bkind;
  c->h_bkind = bk;
  c->general = general;
  c->has_lrts = lrts;
  c->has_shading = shading;
  return AG_OK;
}

int ag_set_agent_kinds(ag_ctx *c, const int32_t *alloc_kind, const int32_t *bid_kind) {
  if (!c) return ag_set_error(AG_ERR_INVALID, "ag_set_agent_kinds: null ctx");
  for (int a = 0; a < c->shape.num_agents; ++a)
    if (bid_kind && bid_kind[a] != AG_BIDDER_TRUTHFUL)
      return ag_set_error(AG_ERR_INVALID, "agent %d: shading bidders need ag_set_agent_params", a);
  return ag_set_agent_params(c, alloc_kind, bid_kind, nullptr, nullptr);
}

int ag_load_lrts(ag_ctx *c, const float *m, const float *q, const float *prev_m,
                 int32_t thompson_sampling) {
  if (!c || !m || !q) return ag_set_error(AG_ERR_INVALID, "ag_load_lrts: null argument");
  AgDeviceGuard g(c->device);
  const size_t n = (size_t)c->shape.num_agents * c->shape.num_items * (c->shape.obs_embedding_size + 1);
  AG_HIP(hipMemcpy(c->d_tsm, m, n * sizeof(float), hipMemcpyHostToDevice));
  AG_HIP(hipMemcpy(c->d_tsq, q, n * sizeof(float), hipMemcpyHostToDevice));
  AG_HIP(hipMemcpy(c->d_tsprev, prev_m ? prev_m : m, n * sizeof(float), hipMemcpyHostToDevice));
  c->ts_sample = thompson_sampling ? 1 : 0;
  c->lrts_loaded = true;
  return AG_OK;
}

int ag_set_option(ag_ctx *c, int32_t option, int64_t value) {
  if (!c) return ag_set_error(AG_ERR_INVALID, "ag_set_option: null ctx");
  switch (option) {
    case AG_OPT_ITEM_SEARCH:
      if (value != AG_ITEM_SEARCH_AUTO && value != AG_ITEM_SEARCH_EXACT)
        return ag_set_error(AG_ERR_INVALID, "ag_set_option: bad item search mode %lld", (long long)value);
      c->item_search = (int32_t)value;
      return AG_OK;
    case AG_OPT_LANE_AUCTIONS:
      if (value != 1 && value != 2)
        return ag_set_error(AG_ERR_INVALID, "ag_set_option: lane auctions must be 1 or 2");
      c->wide = value == 2;
      return AG_OK;
    case AG_OPT_LAUNCH_AUCTIONS:
      if (value < 0) return ag_set_error(AG_ERR_INVALID, "ag_set_option: launch auctions must be >= 0");
      c->launch_cap = value;
      return AG_OK;
    case AG_OPT_LRTS_BLOCK_SAMPLES:
      if (value < 0) return ag_set_error(AG_ERR_INVALID, "ag_set_option: block samples must be >= 0");
      c->lrts_chunk = value;
      return AG_OK;
    case AG_OPT_BIDDER_BLOCK_SAMPLES:
      if (value < 0) return ag_set_error(AG_ERR_INVALID, "ag_set_option: block samples must be >= 0");
      c->bidder_chunk = value;
      return AG_OK;
    case AG_OPT_FIT_NOISE_SEED:
      c->fit_noise_seed = (uint64_t)value;
      return AG_OK;
    case AG_OPT_BIDDER_RECORD_CACHE:
      c->bidder_cache = value;
      return AG_OK;
    case AG_OPT_SIM_BLOCKS_PER_CU:
      if (value < 0 || value > 64) return ag_set_error(AG_ERR_INVALID, "ag_set_option: blocks per CU in [0, 64]");
      c->grid_per_cu = (int32_t)value;
      return AG_OK;
    case AG_OPT_SIM_BLOCK_THREADS:
      if (value != 0 && value != kThreads && value != kLargeThreads)
        return ag_set_error(AG_ERR_INVALID, "ag_set_option: block threads must be 0, %d or %d", kThreads,
                            kLargeThreads);
      c->block_threads = (int32_t)value;
      return AG_OK;
    case AG_OPT_SIM_GENERAL_MODE:
      if (value != 0 && value != 1) return ag_set_error(AG_ERR_INVALID, "ag_set_option: general mode must be 0 or 1");
      c->gen_mode_all = value == 1;
      return AG_OK;
    case AG_OPT_SIM_SHIPPED_SHAPE:
      if (value != 0 && value != 1) return ag_set_error(AG_ERR_INVALID, "ag_set_option: shipped shape must be 0 or 1");
      c->ship_shape = value == 1;
      return AG_OK;
    case AG_OPT_SIMULATE_KERNEL:
      if (value < AG_SIM_KERNEL_AUTO || value > AG_SIM_KERNEL_WIDE)
        return ag_set_error(AG_ERR_INVALID, "ag_set_option: bad simulate kernel %lld", (long long)value);
      if (value == AG_SIM_KERNEL_FUSED || value == AG_SIM_KERNEL_SPLIT)
        return ag_set_error(AG_ERR_UNSUPPORTED, "ag_set_option: k_pop (AG_SIM_KERNEL_FUSED / SPLIT) was retired in "
                                                "round 4: k_simulate is as fast on every population line");
      if (value == AG_SIM_KERNEL_WIDE && !AG_SIM_WIDE_AB)  // the round-3 A/B (2.3x slower): variant builds only
        return ag_set_error(AG_ERR_UNSUPPORTED, "ag_set_option: AG_SIM_KERNEL_WIDE is built only in the A/B "
                                                "variant (make variant VFLAGS=-DAG_SIM_WIDE_AB=1)");
      c->sim_kernel = (int32_t)value;
      return AG_OK;
    default:
      return ag_set_error(AG_ERR_INVALID, "ag_set_option: unknown option %d", option);
  }
}

int ag_load_catalog(ag_ctx *c, const double *item_emb, const double *item_val) {
  if (!c || !item_emb || !item_val) return ag_set_error(AG_ERR_INVALID, "ag_load_catalog: null argument");
  AgDeviceGuard g(c->device);
  const size_t n = (size_t)c->shape.num_agents * c->shape.num_items;
  AG_HIP(hipMemcpy(c->d_items, item_emb, n * c->D * sizeof(double), hipMemcpyHostToDevice));
  AG_HIP(hipMemcpy(c->d_values, item_val, n * sizeof(double), hipMemcpyHostToDevice));
  c->catalog = true;
  // k_oracle's bounds (ag_sim_oracle.h): finite embeddings, every value in (0, kOraMaxValue)
  // the f32 screens rank items by 1 / (CTR * value): valid when every value is positive
  bool pos = true, ok = true;
  for (size_t j = 0; j < n; ++j) {
    pos = pos && item_val[j] > 0.0 && isfinite(item_val[j]);
    ok = ok && item_val[j] > 0.0 && item_val[j] < kOraMaxValue;
  }
  for (size_t j = 0; j < n * c->D && ok; ++j) ok = isfinite(item_emb[j]);
  c->values_positive = pos;
  c->ora_catalog = ok;
  return AG_OK;
}

int ag_allocate(ag_ctx *c, const double *bids, int64_t B, int32_t *winner, double *price,
                double *second_price, void *stream) {
  if (!c || (!bids && B > 0)) return ag_set_error(AG_ERR_INVALID, "ag_allocate: null argument");
  if (B < 0) return ag_set_error(AG_ERR_INVALID, "ag_allocate: B < 0");
  if (B == 0) return AG_OK;
  AgDeviceGuard g(c->device);
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

int ag_simulate(ag_ctx *c, int64_t B, const ag_batch_in *in, ag_batch_out *out_arg, int64_t *counters_fx,
                void *stream) {
  if (!c || !in || !out_arg) return ag_set_error(AG_ERR_INVALID, "ag_simulate: null argument");
  AG_CHECK_STRUCT(in, "ag_simulate", "ag_batch_in");
  ag_batch_out outv;
  AG_READ_OUT(out_arg, outv, "ag_simulate");
  const ag_batch_out *out = &outv;
  if (!c->can_simulate)
    return ag_set_error(AG_ERR_UNSUPPORTED,
                     "ag_simulate: supports E+1 in {2..9,11,13,16} (E+1 <= 8 when P > %d) and a catalogue "
                     "that fits LDS (P=%d, D=%d, N=%d, K=%d)",
                     kMaxP, c->shape.num_participants, c->D, c->shape.num_agents, c->shape.num_items);
  if (!c->catalog) return ag_set_error(AG_ERR_STATE, "ag_simulate: ag_load_catalog not called");
  if (B < 0) return ag_set_error(AG_ERR_INVALID, "ag_simulate: B < 0");
  if (B == 0) return AG_OK;
  if (!in->ctx || !in->part || !in->u) return ag_set_error(AG_ERR_INVALID, "ag_simulate: null input array");
  if (B * c->shape.num_participants > INT32_MAX)
    return ag_set_error(AG_ERR_UNSUPPORTED, "ag_simulate: B * P must be < 2^31 (32-bit SoA indexing); "
                     "split the batch");
  AgDeviceGuard g(c->device);
  const ag_shape &s = c->shape;
  const int D = c->D;
  const bool prune = c->item_search == AG_ITEM_SEARCH_AUTO && D <= 8 && s.num_items <= 2 * kMaxKPairs &&
                     c->values_positive;
  if (c->has_lrts && !c->lrts_loaded)
    return ag_set_error(AG_ERR_STATE, "ag_simulate: LR-TS agents need ag_load_lrts");
  if (c->has_lrts && c->ts_sample && !in->ts_noise)
    return ag_set_error(AG_ERR_INVALID, "ag_simulate: Thompson sampling needs ts_noise");
  if (c->has_shading && !in->gamma_raw)
    return ag_set_error(AG_ERR_INVALID, "ag_simulate: shading bidders need gamma_raw");
  if (c->dr_any_init && !in->policy_eps)
    return ag_set_error(AG_ERR_INVALID, "ag_simulate: learning bidders with a fitted policy need policy_eps");
  if (c->vl_any_search && !in->gamma_grid)
    return ag_set_error(AG_ERR_INVALID, "ag_simulate: ValueLearningBidders bidding by search need gamma_grid");
  if (prune && !c->general && c->ora_catalog && c->sim_kernel != AG_SIM_KERNEL_GENERIC && !c->wide)
    if (OraKernel ok = pick_oracle(s.num_participants, D, false))
      return simulate_oracle(c, ok, B, in, out, counters_fx, (hipStream_t)stream);
  return simulate_general(c, B, in, out, counters_fx, (hipStream_t)stream, false, 0, 0);
}


int ag_simulate_generated(ag_ctx *c, uint64_t seed, uint64_t first, int64_t B, ag_batch_out *out_arg,
                          int64_t *counters_fx, void *stream) {
  if (!c || !out_arg) return ag_set_error(AG_ERR_INVALID, "ag_simulate_generated: null argument");
  ag_batch_out outv;
  AG_READ_OUT(out_arg, outv, "ag_simulate_generated");
  const ag_batch_out *out = &outv;
  if (!c->catalog) return ag_set_error(AG_ERR_STATE, "ag_simulate_generated: ag_load_catalog not called");
  if (B < 0) return ag_set_error(AG_ERR_INVALID, "ag_simulate_generated: B < 0");
  if (B == 0) return AG_OK;
  const ag_shape &s = c->shape;
  if (B * s.num_participants > INT32_MAX)
    return ag_set_error(AG_ERR_UNSUPPORTED, "ag_simulate_generated: B * P must be < 2^31; split the batch");
  if (c->general) {
    // every draw in the kernel (k_simulate<..., GEN>): contexts, participants, uniforms, the
    // LR-TS agents' Thompson noise, the fitted policies' rsample draws, the shading draws
    if (c->has_lrts && !c->lrts_loaded)
      return ag_set_error(AG_ERR_STATE, "ag_simulate_generated: LR-TS agents need ag_load_lrts");
    if (c->vl_any_search)
      return ag_set_error(AG_ERR_UNSUPPORTED, "ag_simulate_generated: ValueLearningBidders bidding by search "
                                              "(their 128-point grids are not drawn in the kernel)");
    if (c->shape.num_participants > 64)
      return ag_set_error(AG_ERR_UNSUPPORTED, "ag_simulate_generated: P > 64");
    AgDeviceGuard g(c->device);
    return simulate_general(c, B, nullptr, out, counters_fx, (hipStream_t)stream, true, seed, first);
  }
  OraKernel k = (!c->general && c->ora_catalog && s.num_items <= 2 * kMaxKPairs)
                    ? pick_oracle(s.num_participants, c->D, true) : nullptr;
  if (!k)
    return ag_set_error(AG_ERR_UNSUPPORTED,
                        "ag_simulate_generated: OracleAllocator + TruthfulBidder populations with P <= %d, "
                        "E + 1 <= 8, K <= %d and catalogue values in (0, %g) only (general populations: the "
                        "shipped shape)",
                        kMaxP, 2 * kMaxKPairs, kOraMaxValue);
  AgDeviceGuard g(c->device);
  // a launch covers auctions [lo, hi) of the batch: their global indices are first + lo ...
  return simulate_oracle(c, k, B, nullptr, out, counters_fx, (hipStream_t)stream, seed, first);
}

int ag_generate(ag_ctx *c, uint64_t seed, uint64_t first, int64_t B, double *ctx_out, int32_t *part_out,
                double *u_out, void *stream) {
  if (!c || !ctx_out || !part_out || !u_out) return ag_set_error(AG_ERR_INVALID, "ag_generate: null argument");
  if (B < 0) return ag_set_error(AG_ERR_INVALID, "ag_generate: B < 0");
  if (B == 0) return AG_OK;
  if (c->shape.num_participants > 64) return ag_set_error(AG_ERR_UNSUPPORTED, "ag_generate: P > 64");
  if (c->shape.embedding_size > kMaxGenE)
    return ag_set_error(AG_ERR_UNSUPPORTED, "ag_generate: E > %d", kMaxGenE);
  AgDeviceGuard g(c->device);
  const int grid = grid_for(B, (int64_t)1 << 40);
  hipLaunchKernelGGL(k_generate, dim3(grid), dim3(kThreads), 0, (hipStream_t)stream, seed, first, B,
                     c->shape.num_agents, c->shape.num_participants, c->shape.embedding_size,
                     c->shape.embedding_var, ctx_out, part_out, u_out);
  AG_HIP(hipGetLastError());
  return AG_OK;
}

int ag_generate_search_grid(ag_ctx *c, uint64_t seed, uint64_t first, int64_t B, double *grid, void *stream) {
  if (!c || !grid) return ag_set_error(AG_ERR_INVALID, "ag_generate_search_grid: null argument");
  if (B < 0) return ag_set_error(AG_ERR_INVALID, "ag_generate_search_grid: B < 0");
  if (B == 0) return AG_OK;
  AgDeviceGuard g(c->device);
  const int grid_n = grid_for(B, (int64_t)1 << 40);
  hipLaunchKernelGGL(k_generate_grid, dim3(grid_n), dim3(kThreads), 0, (hipStream_t)stream, seed, first, B,
                     c->shape.num_participants, grid);
  AG_HIP(hipGetLastError());
  return AG_OK;
}

int ag_generate_noise(ag_ctx *c, uint64_t seed, uint64_t first, int64_t B, const int32_t *part,
                      double *gamma_raw, float *ts_noise, float *policy_eps, void *stream) {
  if (!c || !part) return ag_set_error(AG_ERR_INVALID, "ag_generate_noise: null argument");
  if (B < 0) return ag_set_error(AG_ERR_INVALID, "ag_generate_noise: B < 0");
  if (B == 0) return AG_OK;
  if (ts_noise && !c->lrts_loaded) return ag_set_error(AG_ERR_STATE, "ag_generate_noise: ag_load_lrts first");
  AgDeviceGuard g(c->device);
  const int grid = grid_for(B, (int64_t)1 << 40);
  const int KDo = c->shape.num_items * (c->shape.obs_embedding_size + 1);
  hipLaunchKernelGGL(k_generate_noise, dim3(grid), dim3(kThreads), 0, (hipStream_t)stream, seed, first, B,
                     c->shape.num_participants, KDo, part, c->d_akind, c->d_bkind, c->d_pg, c->d_gs,
                     c->d_tsq, gamma_raw, ts_noise, policy_eps, (const int32_t *)nullptr);
  AG_HIP(hipGetLastError());
  return AG_OK;
}

int ag_ts_noise_index(ag_ctx *c, int64_t B, const int32_t *part, int32_t *index, int64_t *pairs, void *stream) {
  if (!c || !part || !index || !pairs) return ag_set_error(AG_ERR_INVALID, "ag_ts_noise_index: null argument");
  if (B < 0) return ag_set_error(AG_ERR_INVALID, "ag_ts_noise_index: B < 0");
  const int64_t n = B * c->shape.num_participants;
  if (n >= ((int64_t)1 << 31)) return ag_set_error(AG_ERR_INVALID, "ag_ts_noise_index: P * B >= 2^31");
  *pairs = 0;
  if (n == 0) return AG_OK;
  AgDeviceGuard g(c->device);
  hipStream_t st = (hipStream_t)stream;
  if (!c->has_lrts) {  // no LR-TS agent: no pair
    AG_HIP(hipMemsetAsync(index, 0xff, (size_t)n * sizeof(int32_t), st));
    return AG_OK;
  }
  const int64_t nb = (n + kScanTile - 1) / kScanTile;
  int64_t *counts = nullptr;
  AG_HIP(hipMallocAsync((void **)&counts, (size_t)(nb + 1) * sizeof(int64_t), st));
  hipLaunchKernelGGL(k_ts_index_count, dim3((unsigned)nb), dim3(kThreads), 0, st, part, c->d_akind, n, counts);
  hipLaunchKernelGGL(k_ts_index_offsets, dim3(1), dim3(kThreads), 0, st, counts, nb);
  hipLaunchKernelGGL(k_ts_index_write, dim3((unsigned)nb), dim3(kThreads), 0, st, part, c->d_akind, n,
                     (const int64_t *)counts, index);
  hipError_t e = hipGetLastError();
  int64_t total = 0;
  if (e == hipSuccess) e = hipMemcpyAsync(&total, counts + nb, sizeof(int64_t), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  (void)hipFreeAsync(counts, st);
  AG_HIP(e);
  *pairs = total;
  return AG_OK;
}

int ag_generate_ts_noise_compact(ag_ctx *c, uint64_t seed, uint64_t first, int64_t B, const int32_t *part,
                                 const int32_t *index, float *ts_noise, void *stream) {
  if (!c || !part || !index || !ts_noise) return ag_set_error(AG_ERR_INVALID, "ag_generate_ts_noise_compact: null argument");
  if (B < 0) return ag_set_error(AG_ERR_INVALID, "ag_generate_ts_noise_compact: B < 0");
  if (B == 0) return AG_OK;
  if (!c->lrts_loaded) return ag_set_error(AG_ERR_STATE, "ag_generate_ts_noise_compact: ag_load_lrts first");
  AgDeviceGuard g(c->device);
  const int grid = grid_for(B, (int64_t)1 << 40);
  const int KDo = c->shape.num_items * (c->shape.obs_embedding_size + 1);
  hipLaunchKernelGGL(k_generate_noise, dim3(grid), dim3(kThreads), 0, (hipStream_t)stream, seed, first, B,
                     c->shape.num_participants, KDo, part, c->d_akind, c->d_bkind, c->d_pg, c->d_gs,
                     c->d_tsq, (double *)nullptr, ts_noise, (float *)nullptr, index);
  AG_HIP(hipGetLastError());
  return AG_OK;
}

int ag_counters_to_double(const int64_t *fx, int64_t n, double *out) {
  if ((!fx || !out) && n > 0) return ag_set_error(AG_ERR_INVALID, "ag_counters_to_double: null argument");
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

int ag_stream_copy(const void *src, void *dst, int64_t nbytes, void *stream) {
  if ((!src || !dst) && nbytes > 0) return ag_set_error(AG_ERR_INVALID, "ag_stream_copy: null argument");
  if (nbytes < 0 || nbytes % 16 || ((uintptr_t)src | (uintptr_t)dst) % 16)
    return ag_set_error(AG_ERR_INVALID, "ag_stream_copy: nbytes and both pointers must be multiples of 16");
  const int64_t n16 = nbytes / 16;
  for (int64_t lo = 0; lo < n16; lo += (int64_t)INT32_MAX * kThreads / 2) {  // grid.x < 2^31
    const int64_t n = n16 - lo < (int64_t)INT32_MAX * kThreads / 2 ? n16 - lo : (int64_t)INT32_MAX * kThreads / 2;
    hipLaunchKernelGGL(k_stream_copy, dim3((unsigned)((n + kThreads - 1) / kThreads)), dim3(kThreads), 0,
                       (hipStream_t)stream, (const u32x4 *)src + lo, (u32x4 *)dst + lo, n);
    AG_HIP(hipGetLastError());
  }
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
