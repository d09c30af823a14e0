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

namespace agcoop {

// Agent barrier: a combining tree of arrival counters (fan-in kBarFanIn; the last arriver at
// a node goes up a level) and a generation word the root's last arriver bumps, every word on
// its own 128-B line (same-address atomics serialise at the memory side; the waiters' polls
// stay off the counters' lines). Lines: [0] generation, then level 0's ceil(nblk / F)
// nodes, level 1's, ...
constexpr int kBarFanIn = AG_BAR_FANIN, kBarLineWords = 32;
__host__ __device__ inline int bar_lines(int nblk) {
  if (nblk <= 1) return 0;
  int lines = 1;
  for (int m = nblk; m > 1; m = (m + kBarFanIn - 1) / kBarFanIn) lines += (m + kBarFanIn - 1) / kBarFanIn;
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

}  // namespace agcoop
