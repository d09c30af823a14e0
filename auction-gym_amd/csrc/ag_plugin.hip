// ag_plugin.hip -- the per-call plugin surface: Allocator.estimate_CTR and Bidder.bid of one
// agent for n requests (n = 1 is the reference's call), with the arithmetic the simulate
// kernels use for the same plugin (ag_sim.h), so a per-call answer equals the batched one.
//
//  - OracleAllocator.estimate_CTR (src/BidderAllocation.py:81-82): sigmoid(items @ context)
//    in FP64 with the OpenBLAS dot order and the glibc-identical exp (dot_ref, sigmoid);
//  - PyTorchLogisticRegressionAllocator.estimate_CTR (src/BidderAllocation.py:67-68,
//    src/Models.py:28-33): float32 sigmoid(linear(x32, m [+ noise])) (ts_ctr);
//  - Bidder.bid (src/Bidder.py:34-35, :47-58, :171-208, :348-367, :455-475): value * CTR,
//    times the shading factor of the bidder's state (Gaussian draw, fitted policy rsample,
//    or the 'search' argmax over the 128-point grid).
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>

#include "ag_host.h"
#include "ag_sim.h"

namespace ag {
namespace {

constexpr int kPlThreads = 256;

template <int D>
__device__ __forceinline__ double oracle_ctr_one(const double *__restrict__ items, const double *__restrict__ xin,
                                                 const uint64_t *tab) {
  double x[kMaxD];
#pragma unroll
  for (int d = 0; d < kMaxD; ++d) x[d] = d < D ? xin[d] : 0.0;
  return agexp::sigmoid(dot_ref<D>(items, x), tab);
}

// one thread per (request, item): ctr[i][k]
template <int D>
__global__ __launch_bounds__(kPlThreads) void k_estimate_oracle(const double *__restrict__ items, int K, int64_t n,
                                                                 const double *__restrict__ context,
                                                                 double *__restrict__ ctr) {
  __shared__ uint64_t s_tab[256];
  for (int i = threadIdx.x; i < 256; i += kPlThreads) s_tab[i] = ag_exp_tab[i];
  __syncthreads();
  for (int64_t j = (int64_t)blockIdx.x * kPlThreads + threadIdx.x; j < n * K; j += (int64_t)gridDim.x * kPlThreads) {
    const int64_t i = j / K;
    const int k = (int)(j - i * K);
    ctr[j] = oracle_ctr_one<D>(items + (size_t)k * D, context + i * D, s_tab);
  }
}

__global__ __launch_bounds__(kPlThreads) void k_estimate_lrts(const float *__restrict__ m, int K, int Do, int64_t n,
                                                              const double *__restrict__ context,
                                                              const float *__restrict__ noise,
                                                              double *__restrict__ ctr) {
  __shared__ uint64_t s_tab[agexp::kExpTabLds];
  for (int i = threadIdx.x; i < 256; i += kPlThreads) s_tab[i] = ag_exp_tab[i];
  for (int j = threadIdx.x; j < 32; j += kPlThreads) s_tab[256 + j] = agexp::expf_tab_entry(ag_exp_tab, j);
  __syncthreads();
  for (int64_t j = (int64_t)blockIdx.x * kPlThreads + threadIdx.x; j < n * K; j += (int64_t)gridDim.x * kPlThreads) {
    const int64_t i = j / K;
    const int k = (int)(j - i * K);
    float x[AG_LRTS_MAX_DO];
    for (int d = 0; d < Do; ++d) x[d] = (float)context[i * Do + d];  // torch.from_numpy(context.astype(float32))
    const float *nz = noise ? noise + (i * K + k) * Do : nullptr;
    ctr[j] = (double)ts_ctr(m + (size_t)k * Do, x, Do, nz, 1u, k, K, s_tab);
  }
}

// one thread per request: the bid rule resolve() applies to a participant of this kind
__global__ __launch_bounds__(kPlThreads) void k_bid(int kind, int state, double pg, double gs,
                                                    const float *__restrict__ model, int64_t n,
                                                    const double *__restrict__ value,
                                                    const double *__restrict__ ctr,
                                                    const double *__restrict__ gamma_raw,
                                                    const float *__restrict__ eps,
                                                    const double *__restrict__ grid, double *__restrict__ bid,
                                                    double *__restrict__ gamma, double *__restrict__ prop) {
  __shared__ uint64_t s_tab[256];
  for (int i = threadIdx.x; i < 256; i += kPlThreads) s_tab[i] = ag_exp_tab[i];
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * kPlThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kPlThreads) {
    const double v = value[i], c = ctr[i];
    double b = v * c;  // Bidder.bid: value * estimated CTR
    double g = NAN, p = NAN;
    const bool learner = kind >= AG_BIDDER_VALUE_LEARNING;
    if (learner && state == AG_LEARNER_POLICY) {
      policy_bid(model + 4, c, v, eps[i], s_tab, g, p);
      b = b * g;
    } else if (kind == AG_BIDDER_VALUE_LEARNING && state == AG_LEARNER_SEARCH) {
      g = search_gamma(model, c, v, grid + i, (uint32_t)n, s_tab);
      p = 1.0;  // src/Bidder.py:196
      b = b * g;
    } else if (kind != AG_BIDDER_TRUTHFUL) {
      g = gamma_raw[i];
      if (kind == AG_BIDDER_EMPIRICAL_SHADED) {  // clipped to [0, 1] (src/Bidder.py:52-55)
        if (g < 0.0) g = 0.0;
        if (g > 1.0) g = 1.0;
      } else {
        p = shading_propensity(pg, gs, g, s_tab);
      }
      b = b * g;
    }
    bid[i] = b;
    if (gamma) gamma[i] = g;
    if (prop) prop[i] = p;
  }
}

int grid_of(int64_t work) {
  const int64_t g = (work + kPlThreads - 1) / kPlThreads;
  return (int)(g < 1 ? 1 : (g > 4096 ? 4096 : g));
}

}  // namespace
}  // namespace ag

using namespace ag;

extern "C" {

int ag_estimate_ctr(ag_ctx *c, int32_t agent, int64_t n, const double *context, const float *noise, double *ctr,
                    void *stream) {
  if (!c || (n > 0 && (!context || !ctr))) return ag_set_error(AG_ERR_INVALID, "ag_estimate_ctr: null argument");
  const int N = c->shape.num_agents, K = c->shape.num_items, D = c->D, Do = c->shape.obs_embedding_size + 1;
  if (agent < 0 || agent >= N) return ag_set_error(AG_ERR_INVALID, "ag_estimate_ctr: agent %d out of range", agent);
  if (n < 0) return ag_set_error(AG_ERR_INVALID, "ag_estimate_ctr: n < 0");
  if (n == 0) return AG_OK;
  AgDeviceGuard g(c->device);
  hipStream_t st = (hipStream_t)stream;
  const int ak = c->h_akind ? c->h_akind[agent] : AG_ALLOCATOR_ORACLE;
  if (ak == AG_ALLOCATOR_ORACLE) {
    if (!c->catalog) return ag_set_error(AG_ERR_STATE, "ag_estimate_ctr: ag_load_catalog not called");
    const double *items = c->d_items + (size_t)agent * K * D;
    const int grid = grid_of(n * K);
    switch (D) {
#define AG_EST_CASE(d)                                                                              \
  case d:                                                                                           \
    hipLaunchKernelGGL(k_estimate_oracle<d>, dim3(grid), dim3(kPlThreads), 0, st, items, K, n, context, ctr); \
    break;
      AG_EST_CASE(2) AG_EST_CASE(3) AG_EST_CASE(4) AG_EST_CASE(5) AG_EST_CASE(6) AG_EST_CASE(7) AG_EST_CASE(8)
      AG_EST_CASE(9) AG_EST_CASE(10) AG_EST_CASE(11) AG_EST_CASE(12) AG_EST_CASE(13) AG_EST_CASE(14)
      AG_EST_CASE(15) AG_EST_CASE(16)
#undef AG_EST_CASE
      default:
        return ag_set_error(AG_ERR_UNSUPPORTED, "ag_estimate_ctr: E + 1 = %d > %d", D, kMaxD);
    }
  } else {
    if (!c->lrts_loaded) return ag_set_error(AG_ERR_STATE, "ag_estimate_ctr: ag_load_lrts not called");
    if (Do > AG_LRTS_MAX_DO) return ag_set_error(AG_ERR_UNSUPPORTED, "ag_estimate_ctr: OE + 1 > %d", AG_LRTS_MAX_DO);
    hipLaunchKernelGGL(k_estimate_lrts, dim3(grid_of(n * K)), dim3(kPlThreads), 0, st,
                       c->d_tsm + (size_t)agent * K * Do, K, Do, n, context, noise, ctr);
  }
  AG_HIP(hipGetLastError());
  return AG_OK;
}

int ag_bid(ag_ctx *c, int32_t agent, int64_t n, const double *value, const double *est_ctr, const double *gamma_raw,
           const float *policy_eps, const double *gamma_grid, double *bid, double *gamma, double *propensity,
           void *stream) {
  if (!c || (n > 0 && (!value || !est_ctr || !bid))) return ag_set_error(AG_ERR_INVALID, "ag_bid: null argument");
  const int N = c->shape.num_agents;
  if (agent < 0 || agent >= N) return ag_set_error(AG_ERR_INVALID, "ag_bid: agent %d out of range", agent);
  if (n < 0) return ag_set_error(AG_ERR_INVALID, "ag_bid: n < 0");
  if (n == 0) return AG_OK;
  AgDeviceGuard g(c->device);
  const int kind = c->h_bkind ? c->h_bkind[agent] : AG_BIDDER_TRUTHFUL;
  const bool learner = kind >= AG_BIDDER_VALUE_LEARNING;
  int32_t state = AG_LEARNER_UNINITIALISED;
  const float *model = nullptr;
  // the learner state and shading parameters are read back after the caller's stream has
  // drained: an ag_bidder_update / ag_set_* queued on it (even a non-blocking stream) is seen
  if (kind != AG_BIDDER_TRUTHFUL) AG_HIP(hipStreamSynchronize((hipStream_t)stream));
  if (learner && c->dr_loaded) {
    AG_HIP(hipMemcpy(&state, c->dr.init + agent, sizeof(int32_t), hipMemcpyDeviceToHost));
    model = c->dr.state + (size_t)agent * 16;
  }
  if (learner && state == AG_LEARNER_POLICY && !policy_eps)
    return ag_set_error(AG_ERR_INVALID, "ag_bid: agent %d bids from its fitted policy: needs policy_eps", agent);
  if (learner && state == AG_LEARNER_SEARCH && !gamma_grid)
    return ag_set_error(AG_ERR_INVALID, "ag_bid: agent %d bids by search: needs gamma_grid [128][n]", agent);
  if (kind != AG_BIDDER_TRUTHFUL && !(learner && state != AG_LEARNER_UNINITIALISED) && !gamma_raw)
    return ag_set_error(AG_ERR_INVALID, "ag_bid: agent %d draws a Gaussian shading factor: needs gamma_raw", agent);
  double pg = 1.0, gs = 1.0;
  if (kind != AG_BIDDER_TRUTHFUL) {
    AG_HIP(hipMemcpy(&pg, c->d_pg + agent, sizeof(double), hipMemcpyDeviceToHost));
    AG_HIP(hipMemcpy(&gs, c->d_gs + agent, sizeof(double), hipMemcpyDeviceToHost));
  }
  hipLaunchKernelGGL(k_bid, dim3(grid_of(n)), dim3(kPlThreads), 0, (hipStream_t)stream, kind, state, pg, gs, model, n,
                     value, est_ctr, gamma_raw, policy_eps, gamma_grid, bid, gamma, propensity);
  AG_HIP(hipGetLastError());
  return AG_OK;
}

}  // extern "C"
