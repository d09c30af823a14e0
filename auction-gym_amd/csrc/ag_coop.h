// ag_coop.h -- the barrier of the cooperating workgroups that train one agent (LR-TS
// allocators in ag_lrts.hip, learning bidders in ag_dr.hip; cooperative launches, so every
// workgroup is resident). Host and device: bar_lines() sizes an agent's barrier region.
#pragma once
#include <hip/hip_runtime.h>

#include <stddef.h>

#ifndef AG_BAR_SLEEP
#define AG_BAR_SLEEP 2  // s_sleep units (64 cycles) between polls of the generation word
#endif
#ifndef AG_BAR_FANIN
#define AG_BAR_FANIN 16
#endif
// AG_COOP_FENCED=1: the combining-tree sums below with the C++-model hand-off as well -- every
// thread an agent-scope fence (__threadfence: release + acquire) after its atomics and before
// the workgroup barrier that precedes an arrival, and again after the barrier that follows an
// observed arrival / generation move. The default (0) relies on gfx950's ordering of
// sc1 atomics after s_waitcnt vmcnt(0) + the workgroup barrier (see agent_allreduce_start);
// the fenced build is the A/B and the fallback if that ever proves wrong
// (tests/test_gpu_coop.py stresses both forms through ag_coop_selftest).
#ifndef AG_COOP_FENCED
#define AG_COOP_FENCED 0
#endif
#ifndef AG_COOP_GROUPED
#define AG_COOP_GROUPED 0  // 1: the learning bidders' per-epoch sums by agent_allreduce_grouped (A/B:
                           // within 1 % of the tree either way, profiles/r06k_ab_grouped_*.log)
#endif

namespace agcoop {

// Agent barrier: a combining tree of arrival counters (fan-in kBarFanIn; the last arriver at
// a node goes up a level) and a generation word the root's last arriver bumps, every word on
// its own 128-B line (same-address atomics serialise at the memory side; the waiters' polls
// stay off the counters' lines). Lines: [0] generation, then level 0's ceil(nblk / F)
// nodes, level 1's, ...
constexpr int kBarFanIn = AG_BAR_FANIN, kBarLineWords = 32;
__host__ __device__ inline int bar_lines(int nblk, int F = kBarFanIn) {
  if (nblk <= 1) return 0;
  int lines = 1;
  for (int m = nblk; m > 1; m = (m + F - 1) / F) lines += (m + F - 1) / F;
  return lines;
}

// Barrier of the workgroups of one agent (all co-resident: cooperative launch). Arrivals are
// release read-modify-writes and the waiting is relaxed polling followed by ONE acquire fence:
// on gfx950 an agent-scope acquire invalidates the XCD's L2 and a release writes it back, so
// acquire polling (an invalidation per poll, from hundreds of workgroups) stalls every XCD.
// The partials written before the barrier are visible on every XCD after it: every arrival
// RMW extends the release sequences of the earlier ones, each level's last arriver takes an
// acquire fence before it arrives one level up, and the root's release of the generation
// word is acquired by every waiter's fence.
__device__ __forceinline__ void agent_barrier(unsigned *bar, int rank, int nblk) {
  __syncthreads();
  if (nblk > 1 && threadIdx.x == 0) {
    unsigned *gen = bar;
    const unsigned g = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int idx = rank, members_prev = nblk, base = 1;
    bool last = true;
    for (;;) {
      const int nodes = (members_prev + kBarFanIn - 1) / kBarFanIn, q = idx / kBarFanIn;
      const int members = members_prev - q * kBarFanIn < kBarFanIn ? members_prev - q * kBarFanIn : kBarFanIn;
      unsigned *cnt = bar + (size_t)(base + q) * kBarLineWords;
      if (__hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT) != (unsigned)members - 1) {
        last = false;
        break;
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (nodes == 1) break;
      base += nodes;
      idx = q;
      members_prev = nodes;
    }
    if (last) {
      __hip_atomic_fetch_add(gen, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g)
        __builtin_amdgcn_s_sleep(AG_BAR_SLEEP);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
  }
  __syncthreads();
}

// agent_allreduce_i64 split in two so that a workgroup computes something else while the sum
// climbs the tree (ag_dr.hip k_bidder_pipe: the next learner's epoch): _start adds the
// workgroup's W words (LDS vals) up the tree -- the root's last arriver stores the totals to
// row 0 and bumps the generation -- and returns whether this workgroup was that root (every
// thread gets it); thread 0 keeps the generation it read before arriving in *s_gen.
// _finish waits for the generation to move (the root does not wait) and reads row 0 into
// tot. Between the two the workgroup may run other _start / _finish pairs on OTHER regions;
// on one region the calls alternate (a region's next _start follows its _finish). Every
// workgroup of the region must be resident (cooperative launch). nblk <= 1: vals is the total
// (tot must then be vals).
// Fence-free: every word that moves between workgroups is an 8-B agent-scope atomic (add,
// store, load: sc1, served by L2, never by a stale L1) on both sides, every wave's atomics are
// complete (s_waitcnt vmcnt(0), then a workgroup barrier) before its workgroup signals, and
// the wave that polled or arrived last is the one that reads (MI355X_MICROARCH.md, the
// fence-free hand-off forms): no agent release (an L2 write-back, ~1.7 us) per arrival and no
// agent acquire (an L1 invalidate, ~6.5 us at 4 workgroups per CU) per read. Nothing else may
// be handed over through these calls: a caller reading other workgroups' PLAIN stores needs
// agent_allreduce_i64's fences.
// F: the tree's fan-in (bar_lines(nblk, F) lines / rows per region).
#define AG_VMCNT0() asm volatile("s_waitcnt vmcnt(0)" ::: "memory")
#if AG_COOP_FENCED
#define AG_COOP_REL() __threadfence()
#define AG_COOP_ACQ() __threadfence()
#else
#define AG_COOP_REL() ((void)0)
#define AG_COOP_ACQ() ((void)0)
#endif
template <int F = kBarFanIn>
__device__ __forceinline__ bool agent_allreduce_start(unsigned *bar, int64_t *acc, int stride, int rank, int nblk,
                                                      const int64_t *vals, int W, unsigned *s_gen, int *s_flag) {
  const int t = threadIdx.x, nt = blockDim.x;
  __syncthreads();
  if (nblk <= 1) return true;
  for (int j = t; j < W; j += nt)
    __hip_atomic_fetch_add(acc + (size_t)(1 + rank / F) * stride + j, vals[j], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
  unsigned *gen = bar;
  if (t == 0) *s_gen = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  int idx = rank, members_prev = nblk, base = 1;
  bool root = false;
  for (;;) {
    const int nodes = (members_prev + F - 1) / F, q = idx / F;
    const int members = members_prev - q * F < F ? members_prev - q * F : F;
    AG_VMCNT0();
    AG_COOP_REL();
    __syncthreads();  // this workgroup's additions to the node are performed before it arrives
    if (t == 0) {
      unsigned *cnt = bar + (size_t)(base + q) * kBarLineWords;
      const bool last =
          __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)members - 1;
      if (last) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *s_flag = last;
    }
    __syncthreads();
    if (!*s_flag) break;
    AG_COOP_ACQ();
    int64_t *node = acc + (size_t)(base + q) * stride;
    int64_t *dst = nodes == 1 ? acc : acc + (size_t)(base + nodes + q / F) * stride;
    for (int j = t; j < W; j += nt) {  // (the arriving wave; the others after the barrier above)
      const int64_t v = __hip_atomic_load(node + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(node + j, (int64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (nodes == 1)
        __hip_atomic_store(dst + j, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else
        __hip_atomic_fetch_add(dst + j, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (nodes == 1) {
      root = true;
      break;
    }
    base += nodes;
    idx = q;
    members_prev = nodes;
  }
  AG_VMCNT0();
  AG_COOP_REL();
  __syncthreads();  // the root's totals (and every zeroed node) are stored before the generation moves
  if (t == 0 && root) __hip_atomic_fetch_add(gen, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return root;
}
__device__ __forceinline__ void agent_allreduce_finish(unsigned *bar, const int64_t *acc, int nblk, bool root,
                                                       const unsigned *s_gen, int W, int64_t *tot) {
  if (nblk <= 1) return;
  const int t = threadIdx.x, nt = blockDim.x;
  if (t == 0 && !root) {
    const unsigned g = *s_gen;
    while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g)
      __builtin_amdgcn_s_sleep(AG_BAR_SLEEP);
  }
  __syncthreads();
  AG_COOP_ACQ();
  for (int j = t; j < W; j += nt)  // (the polling wave; the others after the barrier above)
    tot[j] = __hip_atomic_load(const_cast<int64_t *>(acc) + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
}

// Exact int64 all-reduce of W words over the workgroups of one agent, summed up the same
// combining tree with integer atomics (exact in any order), every workgroup taking part:
//  - each workgroup adds its words (LDS vals [W]) to its level-0 node's accumulator row;
//  - the last arriver at a node (decided by thread 0, broadcast through LDS) moves the node's
//    row into its parent's with all its threads, zeroing the node row, and arrives one level
//    up; the root's last arriver writes the totals to row 0 and bumps the generation;
//  - everyone then reads row 0 into LDS tot [W].
// acc: the agent's rows [bar_lines(nblk)][stride] int64 (stride >= W), zero on entry and --
// row 0 aside -- zero again on return, so the next call needs no clearing. Instead of every
// workgroup reading every other workgroup's partials (nblk lines from other XCDs each), a
// workgroup reads one row. Call with every thread; nblk <= 1 copies vals to tot. Fence-free
// (agent_allreduce_start / _finish below: 8-B agent atomics both sides), so the caller may
// hand nothing else over through it.
__device__ __forceinline__ void agent_allreduce_i64(unsigned *bar, int64_t *acc, int stride, int rank, int nblk,
                                                    const int64_t *vals, int W, int64_t *tot, int *s_flag) {
  __shared__ unsigned s_gen;
  if (nblk <= 1) {
    __syncthreads();
    for (int j = threadIdx.x; j < W; j += blockDim.x) tot[j] = vals[j];
    __syncthreads();
    return;
  }
  const bool root = agent_allreduce_start(bar, acc, stride, rank, nblk, vals, W, &s_gen, s_flag);
  agent_allreduce_finish(bar, acc, nblk, root, &s_gen, W, tot);
}

// The same combining-tree sum without the wait (per-epoch launches, ag_dr.hip k_bidder_epoch):
// each workgroup adds its W words (LDS vals) up the tree and the root's last arriver stores
// the totals to `out` (a global row read by the NEXT launch: the kernel boundary orders it);
// nobody spins, so the workgroups need not be co-resident. acc / bar: as agent_allreduce_i64
// (zero on entry, zero again on return; fence-free the same way). nblk <= 1 stores vals to out.
__device__ __forceinline__ void agent_reduce_nowait(unsigned *bar, int64_t *acc, int stride, int rank, int nblk,
                                                    const int64_t *vals, int W, int64_t *out, int *s_flag) {
  const int t = threadIdx.x, nt = blockDim.x;
  __syncthreads();
  if (nblk <= 1) {
    for (int j = t; j < W; j += nt) out[j] = vals[j];
    return;
  }
  for (int j = t; j < W; j += nt)
    __hip_atomic_fetch_add(acc + (size_t)(1 + rank / kBarFanIn) * stride + j, vals[j], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
  int idx = rank, members_prev = nblk, base = 1;
  for (;;) {
    const int nodes = (members_prev + kBarFanIn - 1) / kBarFanIn, q = idx / kBarFanIn;
    const int members = members_prev - q * kBarFanIn < kBarFanIn ? members_prev - q * kBarFanIn : kBarFanIn;
    AG_VMCNT0();
    AG_COOP_REL();
    __syncthreads();  // this workgroup's additions to the node are performed before it arrives
    if (t == 0) {
      unsigned *cnt = bar + (size_t)(base + q) * kBarLineWords;
      const bool last =
          __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)members - 1;
      if (last) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *s_flag = last;
    }
    __syncthreads();
    if (!*s_flag) return;
    AG_COOP_ACQ();
    int64_t *node = acc + (size_t)(base + q) * stride;
    int64_t *dst = nodes == 1 ? out : acc + (size_t)(base + nodes + q / kBarFanIn) * stride;
    for (int j = t; j < W; j += nt) {
      const int64_t v = __hip_atomic_load(node + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(node + j, (int64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (nodes == 1)
        dst[j] = v;
      else
        __hip_atomic_fetch_add(dst + j, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (nodes == 1) return;
    base += nodes;
    idx = q;
    members_prev = nodes;
  }
}

// Grouped exact all-reduce (the trainers' per-epoch sums, AG_COOP_GROUPED): the data take one
// level instead of climbing the tree. The workgroups form ceil(nblk / F) groups of F; each adds
// its W words (LDS vals) to its group's accumulator row, waits for them to be performed, and
// arrives at its group's counter; the group's last arriver arrives at the top counter, the
// last group's bumps the generation word, and every workgroup, once the generation has moved,
// reads the group rows and sums them. Nothing is ever reset: counters and generation count
// monotonically (round r's arrivals at a counter of m members are its values m (r - 1) ..
// m r - 1), and the rows accumulate -- per round parity, since a fast workgroup adds its round
// r + 1 words while slower ones still read round r's -- so a workgroup's totals are the rows'
// sum minus the same parity's sum it read two rounds earlier (prev, LDS [2][W], zero at the
// start with the rows), exact in 2^64 arithmetic. After the last data add the critical path
// is three arrivals, one poll and one read; the tree also moved every node's row up a level
// (a load and an add per level). Fence-free as agent_allreduce_start: every word that moves is
// an agent-scope atomic, each wave's atomics are complete (s_waitcnt vmcnt(0) and a barrier)
// before its workgroup arrives, and the wave that polled reads (W <= 64).
// lines: ceil(nblk / F) group counters, then the top counter, then the generation word (each
// on its own kBarLineWords line); rows: [2][ceil(nblk / F)][stride] int64; all zero at the
// first round; rnd: 1, 2, ... (the same in every workgroup).
__host__ __device__ inline int group_lines(int nblk, int F = kBarFanIn) { return nblk > 1 ? (nblk + F - 1) / F + 2 : 0; }
template <int F = kBarFanIn>
__device__ __forceinline__ void agent_allreduce_grouped(unsigned *lines, int64_t *rows, int stride, int rank, int nblk,
                                                        const int64_t *vals, int W, int64_t *tot, unsigned rnd,
                                                        uint64_t (*prev)[32]) {
  const int t = threadIdx.x;
  const int G = (nblk + F - 1) / F, q = rank / F;
  const unsigned members = (unsigned)(nblk - q * F < F ? nblk - q * F : F);
  unsigned *top = lines + (size_t)G * kBarLineWords, *gen = top + kBarLineWords;
  int64_t *par = rows + (size_t)(rnd & 1u) * G * stride;
  __syncthreads();  // vals complete
  if (t < W)
    __hip_atomic_fetch_add(par + (size_t)q * stride + t, vals[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  AG_VMCNT0();
  AG_COOP_REL();
  __syncthreads();  // this workgroup's additions are performed before it arrives
  if (t == 0) {
    bool last = __hip_atomic_fetch_add(lines + (size_t)q * kBarLineWords, 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT) == members * rnd - 1u;
    if (last)
      last = __hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)G * rnd - 1u;
    if (last)
      __hip_atomic_fetch_add(gen, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
      while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < rnd)
        __builtin_amdgcn_s_sleep(AG_BAR_SLEEP);
  }
  if (t < 64) {  // (the polling wave)
    AG_COOP_ACQ();
    if (t < W) {
      uint64_t sum = 0;
      for (int g0 = 0; g0 < G; g0 += 8) {  // eight independent loads in flight (indices clamped)
        uint64_t v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int g = g0 + k < G ? g0 + k : G - 1;
          v[k] = (uint64_t)__hip_atomic_load(par + (size_t)g * stride + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) sum += g0 + k < G ? v[k] : 0ull;
      }
      tot[t] = (int64_t)(sum - prev[rnd & 1u][t]);
      prev[rnd & 1u][t] = sum;
    }
  }
  __syncthreads();
}

}  // namespace agcoop
