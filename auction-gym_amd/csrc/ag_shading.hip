// ag_shading.hip -- shading bidders' per-iteration update on the GPU:
// EmpiricalShadedBidder.update (src/Agent.py:79-94 -> src/Bidder.py:60-147).
//
//  1. k_shading_collect  after each ag_simulate: every participation of a shading bidder
//                        appends (agent, gamma, net utility) to a caller-owned store
//                        (the update's `gammas` and `utilities`).
//  2. k_empirical_update one workgroup per EmpiricalShadedBidder agent: min / max of its
//                        gammas, the reference's bucket grid (Python floor division,
//                        numpy.linspace edges), per-bucket counts and EXACT fixed-point sums
//                        of u and (u - mean)^2 (LDS integer atomics: order-free), the lower
//                        confidence bound per bucket and the last best bucket -> prev_gamma,
//                        written where the simulate kernel reads it.
// Arithmetic: oracle/ag_oracle.c ora_empirical_update.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>

#include "ag_host.h"

namespace {

constexpr int kShThreads = 256;
constexpr int kMaxBuckets = 1024;  // gammas of EmpiricalShadedBidder are in [0, 1]: <= 200
constexpr double kFx = 0x1p40;
constexpr int64_t kLo24 = (int64_t(1) << 24) - 1;

__global__ __launch_bounds__(kShThreads) void k_shading_collect(
    int64_t first, int64_t B, int P, int K, const int32_t *__restrict__ part, ag_batch_out out,
    const int32_t *__restrict__ bkind, const double *__restrict__ values, ag_shading_samples st,
    unsigned long long *__restrict__ count) {
  const int lane = threadIdx.x & 63;
  const bool charged = P >= 2;  // P == 1: nobody is charged (src/Auction.py:68)
  for (int64_t base = (int64_t)blockIdx.x * kShThreads; base < B; base += (int64_t)gridDim.x * kShThreads) {
    const int64_t i = base + threadIdx.x;
    const bool live = i < B;
    // winner and outcome from their arrays, or from the ABI 17 packed word
    const uint32_t wo = (live && !out.winner) ? out.winner_outcome[i] : 0u;
    const int w = live ? (out.winner ? out.winner[i] : (int)(wo & 0x7fffffffu)) : -1;
    for (int s = 0; s < P; ++s) {
      int a = -1;
      bool take = false;
      if (live) {
        a = part[(size_t)s * B + i];
        take = bkind[a] != AG_BIDDER_TRUTHFUL;  // Empirical, ValueLearning, PolicyLearning, DR
      }
      const uint64_t ballot = __ballot(take);
      if (ballot == 0) continue;
      unsigned long long base_slot = 0;
      const int leader = __ffsll((unsigned long long)ballot) - 1;
      if (lane == leader) base_slot = atomicAdd(count, (unsigned long long)__popcll(ballot));
      base_slot = __shfl(base_slot, leader, 64);
      if (!take) continue;
      const int64_t slot = (int64_t)base_slot + __popcll(ballot & ((1ull << lane) - 1));
      if (slot >= st.capacity) continue;  // overflow: reported by the update
      const size_t o = (size_t)s * B + i;
      const bool won = charged && s == w;
      const double v = values[(size_t)a * K + out.item[o]];
      st.agent[slot] = a;
      st.gamma[slot] = out.gamma[o];
      const bool oc = out.winner ? out.outcome[i] != 0 : (wo >> 31) != 0;
      st.utility[slot] = won ? v * (oc ? 1.0 : 0.0) - out.price[i] : 0.0;  // src/Bidder.py:62-63
      if (st.ctr) st.ctr[slot] = out.est_ctr[o];
      if (st.value) st.value[slot] = v;
      if (st.propensity) st.propensity[slot] = out.propensity[o];
      if (st.won) st.won[slot] = won ? 1 : 0;
      if (st.order) st.order[slot] = (uint64_t)(first + i) * (uint64_t)P + (uint64_t)s;
    }
  }
}

__device__ __forceinline__ double py_floordiv(double vx, double wx) {  // CPython float //
  const double mod = fmod(vx, wx);
  double div = (vx - mod) / wx;
  if (mod != 0.0 && ((wx < 0) != (mod < 0))) div -= 1.0;
  double fd;
  if (div != 0.0) {
    fd = floor(div);
    if (div - fd > 0.5) fd += 1.0;
  } else {
    fd = copysign(0.0, vx / wx);
  }
  return fd;
}

__device__ __forceinline__ double fx_read(int64_t hi, int64_t lo) {
  hi += lo >> 24;
  lo &= kLo24;
  return ((double)hi * 0x1p24 + (double)lo) * (1.0 / kFx);
}

// bucket j with edge[j] <= g < edge[j + 1], or -1 (g == max lies in none)
__device__ __forceinline__ int find_bucket(const double *edge, int M, double g) {
  if (!(g >= edge[0]) || !(g < edge[M])) return -1;
  int lo = 0, hi = M - 1;  // largest j with edge[j] <= g
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (edge[mid] <= g) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__global__ __launch_bounds__(kShThreads) void k_empirical_update(
    int N, const int32_t *__restrict__ bkind, const int32_t *__restrict__ s_agent,
    const double *__restrict__ s_gamma, const double *__restrict__ s_util, int64_t n,
    double *__restrict__ prev_gamma, int32_t *__restrict__ status, const int32_t *__restrict__ mask) {
  const int a = blockIdx.x, tid = threadIdx.x;
  if (bkind[a] != AG_BIDDER_EMPIRICAL_SHADED || (mask && !mask[a])) {
    if (tid == 0) status[a] = 0;
    return;
  }
  __shared__ double s_edge[kMaxBuckets + 1], s_mean[kMaxBuckets];
  __shared__ int s_cnt[kMaxBuckets];
  __shared__ unsigned long long s_S[2][kMaxBuckets], s_S2[2][kMaxBuckets];
  __shared__ double s_min[kShThreads / 64], s_max[kShThreads / 64];
  __shared__ unsigned long long s_n[kShThreads / 64];
  __shared__ int s_M;

  // ---- min / max / count of this agent's gammas
  double mn = INFINITY, mx = -INFINITY;
  unsigned long long cnt = 0;
  for (int64_t i = tid; i < n; i += kShThreads)
    if (s_agent[i] == a) {
      const double g = s_gamma[i];
      mn = fmin(mn, g);
      mx = fmax(mx, g);
      ++cnt;
    }
  for (int o = 32; o > 0; o >>= 1) {
    mn = fmin(mn, __shfl_xor(mn, o, 64));
    mx = fmax(mx, __shfl_xor(mx, o, 64));
    cnt += __shfl_xor(cnt, o, 64);
  }
  if ((tid & 63) == 0) {
    s_min[tid >> 6] = mn;
    s_max[tid >> 6] = mx;
    s_n[tid >> 6] = cnt;
  }
  __syncthreads();
  if (tid == 0) {
    double lo = s_min[0], hi = s_max[0];
    unsigned long long tot = s_n[0];
    for (int w = 1; w < kShThreads / 64; ++w) {
      lo = fmin(lo, s_min[w]);
      hi = fmax(hi, s_max[w]);
      tot += s_n[w];
    }
    int M = 0;
    if (tot == 0) {
      status[a] = -1;  // np.min of an empty array
    } else {
      const double nb = py_floordiv(hi - lo, 0.005) + 1.0;
      if (nb < 2.0) status[a] = -2;                       // argmax of an empty sequence
      else if (nb - 1.0 > kMaxBuckets) status[a] = -4;    // grid larger than this kernel holds
      else M = (int)nb - 1;
    }
    s_M = M;
    s_min[0] = lo;
    s_max[0] = hi;
  }
  __syncthreads();
  const int M = s_M;
  if (M == 0) return;
  {
    const double lo = s_min[0], hi = s_max[0], step = (hi - lo) / (double)M;  // numpy.linspace
    for (int j = tid; j <= M; j += kShThreads) s_edge[j] = j == M ? hi : (double)j * step + lo;
    for (int j = tid; j < M; j += kShThreads) {
      s_cnt[j] = 0;
      s_S[0][j] = s_S[1][j] = s_S2[0][j] = s_S2[1][j] = 0;
    }
  }
  __syncthreads();
  // ---- counts and exact sums of u per bucket
  for (int64_t i = tid; i < n; i += kShThreads)
    if (s_agent[i] == a) {
      const int j = find_bucket(s_edge, M, s_gamma[i]);
      if (j < 0) continue;
      const int64_t t = (int64_t)__builtin_rint(s_util[i] * kFx);
      atomicAdd(&s_cnt[j], 1);
      atomicAdd(&s_S[0][j], (unsigned long long)(t >> 24));
      atomicAdd(&s_S[1][j], (unsigned long long)(t & kLo24));
    }
  __syncthreads();
  for (int j = tid; j < M; j += kShThreads)
    s_mean[j] = s_cnt[j] > 1 ? fx_read((int64_t)s_S[0][j], (int64_t)s_S[1][j]) / (double)s_cnt[j] : 0.0;
  __syncthreads();
  // ---- exact sums of (u - mean)^2
  for (int64_t i = tid; i < n; i += kShThreads)
    if (s_agent[i] == a) {
      const int j = find_bucket(s_edge, M, s_gamma[i]);
      if (j < 0 || s_cnt[j] <= 1) continue;
      const double d = s_util[i] - s_mean[j];
      const int64_t t = (int64_t)__builtin_rint(d * d * kFx);
      atomicAdd(&s_S2[0][j], (unsigned long long)(t >> 24));
      atomicAdd(&s_S2[1][j], (unsigned long long)(t & kLo24));
    }
  __syncthreads();
  if (tid == 0) {
    int best = -1;
    double bestU = 0.0;
    for (int j = 0; j < M; ++j) {
      const int c = s_cnt[j];
      if (c <= 1) continue;
      const double se = sqrt(fx_read((int64_t)s_S2[0][j], (int64_t)s_S2[1][j]) / (double)c) / sqrt((double)c);
      const double U = s_mean[j] - 1.96 * se;
      if (best < 0 || U >= bestU) {  // the last maximum (reversed nanargmax)
        best = j;
        bestU = U;
      }
    }
    if (best < 0) {
      status[a] = -3;  // All-NaN slice
    } else {
      double g = (s_edge[best + 1] - s_edge[best]) / 2.0 + s_edge[best];
      if (g < 0) g = 0;
      if (g > 1.0) g = 1.0;
      prev_gamma[a] = g;
      status[a] = 0;
    }
  }
}

int grid_over(int64_t n) {
  int64_t g = (n + kShThreads - 1) / kShThreads;
  if (g > 4096) g = 4096;
  return (int)(g < 1 ? 1 : g);
}

int check_store(const ag_ctx *c, const ag_shading_samples *s, const char *who) {
  if (!c || !s) return ag_set_error(AG_ERR_INVALID, "%s: null argument", who);
  AG_CHECK_STRUCT(s, who, "ag_shading_samples");
  if (!s->agent || !s->gamma || !s->utility || !s->count || s->capacity < 0)
    return ag_set_error(AG_ERR_INVALID, "%s: sample store needs agent, gamma, utility, count, capacity", who);
  return AG_OK;
}

}  // namespace

extern "C" {

int ag_shading_collect(ag_ctx *c, int64_t first, int64_t B, const ag_batch_in *in, const ag_batch_out *out_arg,
                       const ag_shading_samples *s, void *stream) {
  if (int rc = check_store(c, s, "ag_shading_collect")) return rc;
  if (!in || !out_arg) return ag_set_error(AG_ERR_INVALID, "ag_shading_collect: null argument");
  AG_CHECK_STRUCT(in, "ag_shading_collect", "ag_batch_in");
  ag_batch_out outv;
  AG_READ_OUT(out_arg, outv, "ag_shading_collect");
  if (!(outv.winner && outv.outcome)) outv.winner = nullptr;  // then the packed word is read
  const ag_batch_out *out = &outv;
  if (B < 0) return ag_set_error(AG_ERR_INVALID, "ag_shading_collect: B < 0");
  if (B == 0 || !c->has_shading) return AG_OK;
  if (!in->part || !(out->winner || out->winner_outcome) || !out->item || !out->price || !out->gamma)
    return ag_set_error(AG_ERR_INVALID, "ag_shading_collect: needs in.part, out.winner + out.outcome (or "
                                        "out.winner_outcome), out.item, out.price, out.gamma");
  if ((s->ctr && !out->est_ctr) || (s->propensity && !out->propensity))
    return ag_set_error(AG_ERR_INVALID, "ag_shading_collect: the store's ctr / propensity need "
                                        "out.est_ctr / out.propensity");
  AgDeviceGuard g(c->device);
  hipLaunchKernelGGL(k_shading_collect, dim3(grid_over(B)), dim3(kShThreads), 0, (hipStream_t)stream, first, B,
                     c->shape.num_participants, c->shape.num_items, in->part, *out, c->d_bkind, c->d_values, *s,
                     (unsigned long long *)s->count);
  AG_HIP(hipGetLastError());
  return AG_OK;
}

int ag_empirical_update(ag_ctx *c, const ag_shading_samples *s, double *prev_gamma, void *stream) {
  return ag_empirical_update_agents(c, s, nullptr, prev_gamma, stream);
}

int ag_empirical_update_agents(ag_ctx *c, const ag_shading_samples *s, const int32_t *agents, double *prev_gamma,
                               void *stream) {
  if (int rc = check_store(c, s, "ag_empirical_update")) return rc;
  const int N = c->shape.num_agents;
  AgDeviceGuard g(c->device);
  hipStream_t st = (hipStream_t)stream;
  uint64_t n = 0;
  AG_HIP(hipMemcpyAsync(&n, s->count, sizeof n, hipMemcpyDeviceToHost, st));
  AG_HIP(hipStreamSynchronize(st));
  if ((int64_t)n > s->capacity)
    return ag_set_error(AG_ERR_INVALID, "ag_empirical_update: %llu samples overflowed the store (capacity %lld)",
                        (unsigned long long)n, (long long)s->capacity);
  if (!c->d_status) AG_HIP(hipMalloc(&c->d_status, sizeof(int32_t) * 2 * N));  // status [N], mask [N]
  int32_t *d_mask = nullptr;
  if (agents) {
    d_mask = c->d_status + N;
    AG_HIP(hipMemcpyAsync(d_mask, agents, sizeof(int32_t) * N, hipMemcpyHostToDevice, st));
  }
  hipLaunchKernelGGL(k_empirical_update, dim3(N), dim3(kShThreads), 0, st, N, c->d_bkind, s->agent, s->gamma,
                     s->utility, (int64_t)n, c->d_pg, c->d_status, d_mask);
  AG_HIP(hipGetLastError());
  int32_t *status = new int32_t[N];
  hipError_t e = hipMemcpyAsync(status, c->d_status, sizeof(int32_t) * N, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess && prev_gamma) e = hipMemcpyAsync(prev_gamma, c->d_pg, sizeof(double) * N, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  int rc = AG_OK;
  if (e != hipSuccess) {
    rc = ag_set_error(AG_ERR_HIP, "ag_empirical_update: %s", hipGetErrorString(e));
  } else {
    for (int a = 0; a < N && rc == AG_OK; ++a) {
      switch (status[a]) {
        case 0: break;
        case -1:  // the reference's exceptions (numpy), in the reference's words
          rc = ag_set_error(AG_ERR_INVALID, "agent %d: zero-size array to reduction operation minimum "
                                            "which has no identity", a);
          break;
        case -2: rc = ag_set_error(AG_ERR_INVALID, "agent %d: attempt to get argmax of an empty sequence", a); break;
        case -3: rc = ag_set_error(AG_ERR_INVALID, "agent %d: All-NaN slice encountered", a); break;
        default: rc = ag_set_error(AG_ERR_UNSUPPORTED, "agent %d: more than %d gamma buckets", a, kMaxBuckets);
      }
    }
  }
  delete[] status;
  return rc;
}

}  // extern "C"
