// ag_pop_p.hip -- k_pop / k_ts_choice instantiations for one participant count AG_P (the
// Makefile compiles this file once per P = 1..8 with -fno-slp-vectorize: the SLP vectorizer
// pairs the per-item float logits into packed ops and keeps duplicated {x_d, x_d} context
// pairs live, which spilled ~40 VGPRs of these kernels to scratch).
#include "ag_sim_pop.h"

#ifndef AG_P
#error "compile with -DAG_P=<participants>"
#endif

namespace ag {

// AUTO runs k_pop only for TruthfulBidder-only populations at P = 8 (k_simulate is faster at
// P = 2 on every population line, profiles/r03_ab_pop_vs_generic.log): the other participant
// counts are built only for A/B variants (make variant VFLAGS=-DAG_POP_ALL_P=1)
#ifndef AG_POP_ALL_P
#define AG_POP_ALL_P 0
#endif
#if AG_P >= 8 || (AG_P >= 1 && AG_POP_ALL_P)
// k_pop: the shipped catalogue shape only (K = 12, E = 5, OE = 4); mode kGenTruthful or
// kGenAll, 256- or 1024-lane workgroups
template <>
PopKernel pick_pop_for<AG_P>(int D, int K, int DO, int mode, int bt, bool tsx) {
  constexpr int P = AG_P;
  if (D != 6 || K != 12 || DO != 5) return nullptr;
  constexpr int L = kLargeThreads, S = kThreads;
  if (mode == kGenTruthful) {
    if (tsx) return bt == L ? k_pop<P, 6, 12, 5, kGenTruthful, L, true> : k_pop<P, 6, 12, 5, kGenTruthful, S, true>;
    return bt == L ? k_pop<P, 6, 12, 5, kGenTruthful, L, false> : k_pop<P, 6, 12, 5, kGenTruthful, S, false>;
  }
  if (mode == kGenAll) {
    if (tsx) return bt == L ? k_pop<P, 6, 12, 5, kGenAll, L, true> : k_pop<P, 6, 12, 5, kGenAll, S, true>;
    return bt == L ? k_pop<P, 6, 12, 5, kGenAll, L, false> : k_pop<P, 6, 12, 5, kGenAll, S, false>;
  }
  return nullptr;
}

template <>
TsChoiceKernel pick_ts_choice_for<AG_P>(int K, int DO) {
  if (K != 12 || DO != 5) return nullptr;
  return k_ts_choice<AG_P, 12, 5, kThreads>;
}

#else
template <>
PopKernel pick_pop_for<AG_P>(int, int, int, int, int, bool) { return nullptr; }
template <>
TsChoiceKernel pick_ts_choice_for<AG_P>(int, int) { return nullptr; }
#endif

}  // namespace ag
