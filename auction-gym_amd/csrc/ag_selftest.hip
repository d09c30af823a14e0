// ag_selftest.hip -- stress test of the learners' cross-workgroup exact sums (ag_coop.h), the
// hand-off every trainer relies on (k_lrts_train, k_bidder_train, the pipe, the per-epoch
// kernels; regions = 0: agent_allreduce_grouped, the learning bidders' per-epoch sums): many cooperative workgroups -- spread over every XCD -- run generation after
// generation of interleaved combining-tree all-reduces of int64 words whose totals each
// workgroup also knows in closed form, and count every total that differs. A stale read (a
// node row or total seen before another XCD's addition, or a counter / generation observed
// out of order) shows up as a wrong total or a hang, so tests/test_gpu_coop.py runs it under a
// time limit on the built form (AG_COOP_FENCED 0 by default; the fenced form is the A/B build
// `make variant NAME=fenced VFLAGS=-DAG_COOP_FENCED=1`).
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "ag_coop.h"
#include "ag_div.h"
#include "ag_host.h"

namespace {

constexpr int kStThreads = 256;
constexpr int kStWords = 32;     // words per all-reduce (the pipe's row width)
constexpr int kStMaxRegions = 4;

// the word a workgroup contributes: any function of (generation, region, rank, word) that
// changes every generation
__device__ __forceinline__ int64_t st_val(uint32_t gen, int region, int rank, int j) {
  uint64_t x = ((uint64_t)gen << 40) ^ ((uint64_t)region << 32) ^ ((uint64_t)rank << 8) ^ (uint64_t)j;
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return (int64_t)x;
}

// Every workgroup is a member of every region (as in k_bidder_pipe, where each workgroup takes
// part in every learner's sum): generation g starts the regions' sums one after the other and
// then finishes them in the same order, so up to `regions` sums climb the trees at once.
__global__ __launch_bounds__(kStThreads) void k_coop_stress(unsigned *bars, int64_t *acc, int lines, int regions,
                                                            int gens, unsigned long long *bad) {
  __shared__ int64_t s_vals[kStMaxRegions][kStWords], s_tot[kStMaxRegions][kStWords], s_want[kStWords];
  __shared__ unsigned s_gen[kStMaxRegions];
  __shared__ int s_flag;
  __shared__ bool s_root[kStMaxRegions];
  const int t = threadIdx.x, rank = blockIdx.x, nblk = gridDim.x;
  unsigned long long nbad = 0;
  for (int g = 0; g < gens; ++g) {
    for (int r = 0; r < regions; ++r) {
      if (t < kStWords) s_vals[r][t] = st_val((uint32_t)g, r, rank, t);
      // (agent_allreduce_start's leading workgroup barrier publishes s_vals)
      const bool root = agcoop::agent_allreduce_start(bars + (size_t)r * lines * agcoop::kBarLineWords,
                                                      acc + (size_t)r * lines * kStWords, kStWords, rank, nblk,
                                                      s_vals[r], kStWords, &s_gen[r], &s_flag);
      if (t == 0) s_root[r] = root;
    }
    for (int r = 0; r < regions; ++r) {
      __syncthreads();
      agcoop::agent_allreduce_finish(bars + (size_t)r * lines * agcoop::kBarLineWords,
                                     acc + (size_t)r * lines * kStWords, nblk, s_root[r], &s_gen[r], kStWords,
                                     s_tot[r]);
      // the closed form: every rank's word summed mod 2^64 (the threads split the ranks)
      if (t < kStWords) s_want[t] = 0;
      __syncthreads();
      for (int j = 0; j < kStWords; ++j) {
        uint64_t part = 0;
        for (int q = t; q < nblk; q += kStThreads) part += (uint64_t)st_val((uint32_t)g, r, q, j);
        for (int o = 32; o > 0; o >>= 1) part += (uint64_t)__shfl_xor((long long)part, o, 64);
        if ((t & 63) == 0) atomicAdd((unsigned long long *)&s_want[j], (unsigned long long)part);
      }
      __syncthreads();
      if (t < kStWords && s_tot[r][t] != s_want[t]) ++nbad;
    }
  }
  if (nbad) atomicAdd(bad, nbad);
}

// ag_div.h's split division against the compiler's `a / b`, bit for bit, over operands in
// div_safe's range: per thread `iters` pairs of three kinds -- anywhere in the range; the BCE
// row's (1 or e) / (1 + e) and log1p's c / (1 + e) with e down to 2^-740; log1p's f / (2 + f)
__device__ __forceinline__ uint64_t st_mix(uint64_t x) {
  x ^= x >> 31;
  x *= 0x7fb5d329728ea185ull;
  x ^= x >> 27;
  x *= 0x81dadef4bc2dd44dull;
  x ^= x >> 33;
  return x;
}
__device__ __forceinline__ double st_num(uint64_t h, int lo, int hi) {  // +-(1 + m) 2^k, k in [lo, hi)
  const int k = lo + (int)((h >> 52) % (uint64_t)(hi - lo));
  const double m = __builtin_bit_cast(double, 0x3ff0000000000000ull | (h & 0x000fffffffffffffull));
  return __builtin_ldexp((h >> 63) ? -m : m, k);
}
__global__ __launch_bounds__(256) void k_div_stress(uint64_t seed, int iters, unsigned long long *bad,
                                                    unsigned long long *tested) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long nbad = 0, n = 0;
  for (int i = 0; i < iters; ++i) {
    const uint64_t h1 = st_mix(seed ^ (t * 0x9e3779b97f4a7c15ull) ^ ((uint64_t)i << 40) ^ 1),
                   h2 = st_mix(h1 ^ 0x2545f4914f6cdd1dull), h3 = st_mix(h2 + 7);
    double a, b;
    switch (i % 3) {
      case 0:
        a = st_num(h1, -900, 600);
        b = st_num(h2, -60, 60);
        break;
      case 1: {
        const double e = __builtin_fabs(st_num(h1, -740, 0));
        b = 1.0 + e;
        const int w = (int)(h3 % 3);
        a = w == 0 ? 1.0 : (w == 1 ? e : (e - (b - 1.0)));  // the last: log1p's c (may be +0)
        break;
      }
      default: {
        const double f = (double)(int64_t)(h1 >> 11) * 0x1p-53 * 0.71 - 0.29;  // [-0.29, 0.42)
        a = f;
        b = 2.0 + f;
        break;
      }
    }
    if (!agdiv::div_safe(a, b)) continue;
    ++n;
    const double want = a / b, got = agdiv::div_core(a, b, agdiv::recip(b));
    if (__builtin_bit_cast(uint64_t, want) != __builtin_bit_cast(uint64_t, got)) ++nbad;
  }
  if (nbad) atomicAdd(bad, nbad);
  atomicAdd(tested, n);
}

// agent_allreduce_grouped (the trainers' per-epoch sums) under the same stress: every
// workgroup one member, `gens` rounds of 32-word sums checked against the closed form
__global__ __launch_bounds__(kStThreads) void k_group_stress(unsigned *cnt, int64_t *rows, int gens,
                                                             unsigned long long *bad) {
  __shared__ int64_t s_vals[kStWords], s_want[kStWords];
  __shared__ uint64_t s_prev[2][32];
  const int t = threadIdx.x, rank = blockIdx.x, nblk = gridDim.x;
  if (t < 64) s_prev[t >> 5][t & 31] = 0;
  unsigned long long nbad = 0;
  for (int g = 0; g < gens; ++g) {
    __syncthreads();
    if (t < kStWords) s_vals[t] = st_val((uint32_t)g, 0, rank, t);
    agcoop::agent_allreduce_grouped(cnt, rows, kStWords, rank, nblk, s_vals, kStWords, s_vals, (unsigned)g + 1u,
                                    s_prev);
    if (t < kStWords) s_want[t] = 0;
    __syncthreads();
    for (int j = 0; j < kStWords; ++j) {
      uint64_t part = 0;
      for (int q = t; q < nblk; q += kStThreads) part += (uint64_t)st_val((uint32_t)g, 0, q, j);
      for (int o = 32; o > 0; o >>= 1) part += (uint64_t)__shfl_xor((long long)part, o, 64);
      if ((t & 63) == 0) atomicAdd((unsigned long long *)&s_want[j], (unsigned long long)part);
    }
    __syncthreads();
    if (t < kStWords && s_vals[t] != s_want[t]) ++nbad;
  }
  if (nbad) atomicAdd(bad, nbad);
}

}  // namespace

extern "C" int ag_div_selftest(int32_t device, int64_t pairs, uint64_t seed, int64_t *tested, int64_t *mismatches) {
  if (!mismatches || !tested || pairs < 0)
    return ag_set_error(AG_ERR_INVALID, "ag_div_selftest: pairs >= 0, non-null tested / mismatches");
  AgDeviceGuard dg(device);
  constexpr int kBlocks = 4096, kIters = 48;
  const int64_t per_launch = (int64_t)kBlocks * 256 * kIters;
  unsigned long long *cnt = nullptr;
  hipError_t e = hipMalloc(&cnt, 2 * sizeof(*cnt));
  if (e == hipSuccess) e = hipMemset(cnt, 0, 2 * sizeof(*cnt));
  for (int64_t done = 0, l = 0; e == hipSuccess && done < pairs; done += per_launch, ++l) {
    hipLaunchKernelGGL(k_div_stress, dim3(kBlocks), dim3(256), 0, nullptr, seed + (uint64_t)l * 0x100000001b3ull,
                       kIters, cnt, cnt + 1);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  unsigned long long h[2] = {0, 0};
  if (e == hipSuccess) e = hipMemcpy(h, cnt, sizeof(h), hipMemcpyDeviceToHost);
  (void)hipFree(cnt);
  if (e != hipSuccess) return ag_set_error(AG_ERR_HIP, "ag_div_selftest: %s", hipGetErrorString(e));
  *mismatches = (int64_t)h[0];
  *tested = (int64_t)h[1];
  return AG_OK;
}

extern "C" int ag_coop_selftest(int32_t device, int32_t workgroups, int32_t generations, int32_t regions,
                                int64_t *mismatches) {
  if (!mismatches) return ag_set_error(AG_ERR_INVALID, "ag_coop_selftest: null mismatches");
  if (generations < 0 || regions < 0 || regions > kStMaxRegions)
    return ag_set_error(AG_ERR_INVALID, "ag_coop_selftest: generations >= 0, regions in [0, %d]", kStMaxRegions);
  AgDeviceGuard dg(device);
  int cus = 0, per_cu = 0;
  AG_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
  const void *kern = regions == 0 ? (const void *)k_group_stress : (const void *)k_coop_stress;
  AG_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kStThreads, 0));
  const int cap = per_cu * cus;
  int G = workgroups > 0 ? workgroups : 4 * cus;
  if (G > cap)
    return ag_set_error(AG_ERR_UNSUPPORTED, "ag_coop_selftest: %d workgroups > %d co-resident", G, cap);
  int lines = regions == 0 ? agcoop::group_lines(G) : agcoop::bar_lines(G);
  if (lines < 1) lines = 1;
  const int rg = regions == 0 ? 2 : regions;  // grouped: rows [2 parities][groups][32]
  // bars: [regions][lines][32] u32; acc: [regions][lines][32] int64 (zero on entry, zero again
  // after every sum but row 0); bad: one u64
  unsigned *bars = nullptr;
  int64_t *acc = nullptr;
  unsigned long long *bad = nullptr;
  const size_t nb = (size_t)rg * lines * agcoop::kBarLineWords * sizeof(unsigned);
  const size_t na = (size_t)rg * lines * kStWords * sizeof(int64_t);
  hipError_t e = hipMalloc(&bars, nb);
  if (e == hipSuccess) e = hipMalloc(&acc, na);
  if (e == hipSuccess) e = hipMalloc(&bad, sizeof(*bad));
  if (e == hipSuccess) e = hipMemset(bars, 0, nb);
  if (e == hipSuccess) e = hipMemset(acc, 0, na);
  if (e == hipSuccess) e = hipMemset(bad, 0, sizeof(*bad));
  int nreg = regions;
  void *args[] = {&bars, &acc, &lines, &nreg, &generations, &bad};
  void *gargs[] = {&bars, &acc, &generations, &bad};
  if (e == hipSuccess)
    e = hipLaunchCooperativeKernel(kern, dim3(G), dim3(kStThreads), regions == 0 ? gargs : args, 0, nullptr);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  unsigned long long h = 0;
  if (e == hipSuccess) e = hipMemcpy(&h, bad, sizeof(h), hipMemcpyDeviceToHost);
  (void)hipFree(bars);
  (void)hipFree(acc);
  (void)hipFree(bad);
  if (e != hipSuccess) return ag_set_error(AG_ERR_HIP, "ag_coop_selftest: %s", hipGetErrorString(e));
  *mismatches = (int64_t)h;
  return AG_OK;
}
