// ag_sim_p.hip -- k_simulate instantiations for one participant count AG_P (the Makefile
// compiles this file once per P = 1..8, in parallel).
#include "ag_sim.h"
#include "ag_sim_oracle.h"

#ifndef AG_P
#error "compile with -DAG_P=<participants>"
#endif
#ifndef AG_LANE_PAIRS
#define AG_LANE_PAIRS 0
#endif

namespace ag {
namespace {

template <int P, bool PRUNE, int W, int G, int BT = kThreads>
SimKernel pick_d(int D) {
  switch (D) {
    case 2: return k_simulate<P, 2, PRUNE, W, G, BT>;
    case 3: return k_simulate<P, 3, PRUNE, W, G, BT>;
    case 4: return k_simulate<P, 4, PRUNE, W, G, BT>;
    case 5: return k_simulate<P, 5, PRUNE, W, G, BT>;
    case 6: return k_simulate<P, 6, PRUNE, W, G, BT>;
    case 7: return k_simulate<P, 7, PRUNE, W, G, BT>;
    case 8: return k_simulate<P, 8, PRUNE, W, G, BT>;
    default: return nullptr;
  }
}

}  // namespace

// prune: the f32-screened item search (D <= 8, K <= 2 kMaxKPairs), W auctions per lane
// (2 when B is even: 16-B accesses); otherwise the exact scan, one auction per lane.
// general: populations beyond OracleAllocator + TruthfulBidder (one auction per lane), in
// 256-lane workgroups or, screened, 1024-lane ones (bt; large populations' LDS images);
// kGenTruthful (TruthfulBidders only) has its own 256-lane build, otherwise the kGenAll one.
#if AG_P == 0
// P = 0: the runtime-P kernel (more than kMaxP participants), one auction per lane.
template <>
SimKernel pick_kernel_for<0>(int D, bool prune, int W, int general, int bt) {
  if (general & kGenGen) return nullptr;  // no generate-mode build of the runtime-P kernel
  general &= ~kGenShip;  // no shipped-shape build of the runtime-P kernel
  if (W != 1 || bt != kThreads || D > 8) return nullptr;
  if (general) return prune ? pick_d<0, true, 1, kGenAll>(D) : pick_d<0, false, 1, kGenAll>(D);
  return prune ? pick_d<0, true, 1, kGenOracle>(D) : pick_d<0, false, 1, kGenOracle>(D);
}

template <>
OraKernel pick_oracle_for<0>(int, bool) { return nullptr; }
#else
template <>
SimKernel pick_kernel_for<AG_P>(int D, bool prune, int W, int general, int bt) {
  constexpr int P = AG_P;
  const bool ship = (general & kGenShip) != 0;
  const bool genm = (general & kGenGen) != 0;
  general &= ~(kGenShip | kGenGen);
  if (genm) {  // generate mode (k_simulate<..., GEN>): the shipped shape's builds only
    if (!general || !ship || !prune || D != 6 || W != 1) return nullptr;
    if (bt == kLargeThreads) return k_simulate<P, 6, true, 1, kGenAll, kLargeThreads, kShipDo, true>;
    if constexpr (P >= AG_STREAM_MIN_P)
      if (bt == kMidThreads && general == kGenAll) return k_simulate<P, 6, true, 1, kGenAll, kMidThreads, kShipDo, true>;
    if (bt != kThreads) return nullptr;
    if (general == kGenTruthful) return k_simulate<P, 6, true, 1, kGenTruthful, kThreads, kShipDo, true>;
    return k_simulate<P, 6, true, 1, kGenAll, kThreads, kShipDo, true>;
  }
  if (general && ship && prune && D == 6) {  // the shipped shape: LR-TS width 5 compile-time
    if (bt == kLargeThreads) return k_simulate<P, 6, true, 1, kGenAll, kLargeThreads, kShipDo>;
    if constexpr (P >= AG_STREAM_MIN_P)  // the full mix at P >= 3: streamed, 768 lanes
      if (bt == kMidThreads && general == kGenAll) return k_simulate<P, 6, true, 1, kGenAll, kMidThreads, kShipDo>;
    if (bt != kThreads) return nullptr;
    if (general == kGenTruthful) return k_simulate<P, 6, true, 1, kGenTruthful, kThreads, kShipDo>;
    return k_simulate<P, 6, true, 1, kGenAll, kThreads, kShipDo>;
  }
  if (general) {
    if (D > 8) return nullptr;
    if (bt == kLargeThreads) return prune ? pick_d<P, true, 1, kGenAll, kLargeThreads>(D) : nullptr;
    if (bt != kThreads) return nullptr;
    if (general == kGenTruthful)
      return prune ? pick_d<P, true, 1, kGenTruthful>(D) : pick_d<P, false, 1, kGenTruthful>(D);
    return prune ? pick_d<P, true, 1, kGenAll>(D) : pick_d<P, false, 1, kGenAll>(D);
  }
  if (bt != kThreads) return nullptr;
#if AG_LANE_PAIRS
  // two auctions per lane (AG_OPT_LANE_AUCTIONS = 2): an A/B build only (a wash isolated, slower
  // sustained; k_oracle is the Oracle populations' kernel)
  if (prune && W == 2) return pick_d<P, true, 2, kGenOracle>(D);
#endif
  if (W != 1) return nullptr;
  if (prune) return pick_d<P, true, 1, kGenOracle>(D);
  if (D <= 8) return pick_d<P, false, 1, kGenOracle>(D);
  switch (D) {
    case 9: return k_simulate<P, 9, false, 1, kGenOracle>;
    case 11: return k_simulate<P, 11, false, 1, kGenOracle>;
    case 13: return k_simulate<P, 13, false, 1, kGenOracle>;
    case 16: return k_simulate<P, 16, false, 1, kGenOracle>;
    default: return nullptr;
  }
}

template <>
OraKernel pick_oracle_for<AG_P>(int D, bool gen) {
  constexpr int P = AG_P;
  switch (D) {
    case 2: return gen ? k_oracle<P, 2, true> : k_oracle<P, 2, false>;
    case 3: return gen ? k_oracle<P, 3, true> : k_oracle<P, 3, false>;
    case 4: return gen ? k_oracle<P, 4, true> : k_oracle<P, 4, false>;
    case 5: return gen ? k_oracle<P, 5, true> : k_oracle<P, 5, false>;
    case 6: return gen ? k_oracle<P, 6, true> : k_oracle<P, 6, false>;
    case 7: return gen ? k_oracle<P, 7, true> : k_oracle<P, 7, false>;
    case 8: return gen ? k_oracle<P, 8, true> : k_oracle<P, 8, false>;
    default: return nullptr;
  }
}
#endif

}  // namespace ag
