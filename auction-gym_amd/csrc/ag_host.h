// ag_host.h -- host-side state shared by the C-ABI translation units (not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "auctiongym.h"

// Sets the thread-local ag_last_error() text; returns `code`.
int ag_set_error(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));

#define AG_HIP(call)                                                                    \
  do {                                                                                  \
    hipError_t e_ = (call);                                                             \
    if (e_ != hipSuccess)                                                               \
      return ag_set_error(AG_ERR_HIP, "%s: %s (%s:%d)", #call, hipGetErrorString(e_),   \
                          __FILE__, __LINE__);                                          \
  } while (0)

// ABI structs passed by pointer start with their size (include/auctiongym.h): a binding
// compiled against another layout is refused before any other field is read.
template <typename T>
inline int ag_check_struct(const T *p, const char *who, const char *type) {
  if (p && p->struct_size != (uint64_t)sizeof(T))
    return ag_set_error(AG_ERR_INVALID,
                        "%s: %s.struct_size is %llu, this library (ABI %d) expects %llu -- the caller's "
                        "binding declares another layout of include/auctiongym.h",
                        who, type, (unsigned long long)p->struct_size, AG_ABI_VERSION,
                        (unsigned long long)sizeof(T));
  return AG_OK;
}
#define AG_CHECK_STRUCT(p, who, type) \
  do {                                \
    if (int rc_ = ag_check_struct(p, who, type)) return rc_; \
  } while (0)

// ag_batch_out of ABI 17 or of ABI 15/16 (AG_BATCH_OUT_V16_SIZE: no ABI 17 fields), read into
// a full ABI-17 struct `v` (winner_outcome NULL for the older layout).
inline int ag_read_out(const ag_batch_out *p, ag_batch_out *v, const char *who) {
  if (!p) return ag_set_error(AG_ERR_INVALID, "%s: null ag_batch_out", who);
  if (p->struct_size == (uint64_t)sizeof(ag_batch_out)) {
    *v = *p;
  } else if (p->struct_size == AG_BATCH_OUT_V16_SIZE) {
    *v = ag_batch_out{};
    __builtin_memcpy(v, p, AG_BATCH_OUT_V16_SIZE);
    v->struct_size = sizeof(ag_batch_out);
  } else {
    return ag_set_error(AG_ERR_INVALID,
                        "%s: ag_batch_out.struct_size is %llu, this library (ABI %d) expects %llu (or %llu, "
                        "the ABI 16 layout) -- the caller's binding declares another layout of include/auctiongym.h",
                        who, (unsigned long long)p->struct_size, AG_ABI_VERSION,
                        (unsigned long long)sizeof(ag_batch_out), (unsigned long long)AG_BATCH_OUT_V16_SIZE);
  }
  return AG_OK;
}
#define AG_READ_OUT(p, v, who) \
  do {                         \
    if (int rc_ = ag_read_out(p, &(v), who)) return rc_; \
  } while (0)

// LR-TS training workspace (ag_lrts.hip), grown on demand by ag_lrts_update.
struct ag_lrts_ws {
  int64_t cap = 0;            // samples the bucket arrays hold
  uint32_t *key = nullptr;    // [cap] samples bucketed by agent
  float *x = nullptr;         // [Do][cap]
  int64_t *offsets = nullptr; // [N + 1] bucket offsets, then per-agent cursors [N]
  double *adam_tab = nullptr; // [2][kLrEpochs]: 1 - 0.9^t, (1 - 0.999^t)^0.5 (host pow)
  int32_t *epochs = nullptr;  // [N]
  void *tables = nullptr;     // workgroup -> (agent, rank) tables + per-agent barriers
  int64_t *partials = nullptr;  // per-workgroup exact partial sums, 2 epoch parities
  size_t tab_cap = 0, part_cap = 0, bar_cap = 0;
  int coop_blocks = 0;        // co-resident workgroups of the training kernel
  int32_t *status = nullptr;  // [1] device-side error flags
  // resumable / record-parallel training (ag_lrts_rp_*): one launch per epoch
  struct {
    bool active = false;
    void *st = nullptr;          // LrSt [2][N], by launch parity
    int64_t *acc = nullptr;      // combining-tree accumulator rows [lines][144]
    unsigned *bar = nullptr;     // barrier lines [lines][32]
    int32_t *tables = nullptr;   // blk_agent [G], blk_rank [G], agent_nblk [N], bar_off [N], mask [N]
    size_t cap_g = 0, cap_lines = 0;
    int G = 0;
    int64_t k = 0;               // launches so far
    int64_t *totals = nullptr;   // the caller's dev int64 [2][N][144]
  } rp;
};

// Resumable / record-parallel training of the exact-sum learning bidders (ag_bidder_rp_*,
// ag_dr.hip): one launch per epoch, the training state in HBM.
struct ag_dr_rp {
  bool active = false;
  void *st = nullptr;           // FitSt [2][N], by launch parity
  int64_t *acc = nullptr;       // agents' combining-tree accumulator rows [lines][32]
  unsigned *bar = nullptr;      // agents' barrier lines [lines][32]
  int32_t *tables = nullptr;    // blk_agent [G], blk_rank [G], agent_nblk [N], bar_off [N]
  int64_t *ntot = nullptr;      // [N] records over all ranks, [N] global index of this rank's first
  size_t cap_g = 0, cap_lines = 0;
  int G = 0, lines = 0;
  int64_t k = 0;                // launches so far
  int64_t *totals = nullptr;    // the caller's dev int64 [2][N][32]
  const float *noise = nullptr; // host-drawn rsample window (ag_bidder_rp_noise)
  int64_t noise_n = 0;
  int32_t noise_e0 = 0, noise_epochs = 0;
  int32_t *mask = nullptr;      // [N] the agents under training (host copy in `agents`)
  int64_t n_local = 0;
  bool single = false;          // this rank holds every record (ag_bidder_rp_run allowed)
  // k_bidder_pipe (ag_bidder_rp_run, ag_bidder_update): slot tables, tree rows / barrier
  // lines, its own FitSt [N] for ag_bidder_update
  void *pipe = nullptr;
  size_t pipe_bytes = 0;
  void *pipe_st = nullptr;      // FitSt [N] of ag_bidder_update's pipe run
  int pipe_blocks[2] = {0, 0};  // co-resident workgroups per phase
};

// DoublyRobustBidder workspace (ag_dr.hip)
struct ag_dr_ws {
  void *buf = nullptr;          // records in log order (ctr, value, gamma, prop, util, est_util,
                                // won), sort keys / indices, hipcub temp
  size_t buf_bytes = 0;
  int64_t *counts = nullptr;    // [N] counts, [N + 1] offsets
  double *adam_tab = nullptr;   // [2][32768] Adam bias corrections (libm pow)
  float *state = nullptr;       // [N][16]: win-rate w0 w1 w2 b, policy (12)
  int32_t *init = nullptr;      // [N] AG_LEARNER_*: what the agent bids from
  int32_t *mode = nullptr;      // [N] ValueLearningBidder inference / PolicyLearningBidder loss
  int64_t *scratch = nullptr;   // [N] noise offsets + [N][4] epochs / status
  void *coop = nullptr;         // trainer workgroup tables, barriers, exchange partials
  size_t coop_bytes = 0;
  int coop_blocks = 0;          // co-resident workgroups of k_bidder_train<1>
  int coop_blocks0 = 0;         // co-resident workgroups of k_bidder_train<0>
  ag_dr_rp rp;
};

struct ag_ctx {
  int32_t device;
  ag_shape shape;
  int32_t D;
  int32_t item_search = AG_ITEM_SEARCH_AUTO;
  bool can_simulate = false;
  double *d_items = nullptr;
  double *d_values = nullptr;
  int64_t *d_partials = nullptr;
  uint32_t *d_queue = nullptr;  // k_oracle's chunk counters (AG_ORA_QUEUE): 64 x 32 words
  int32_t partial_blocks = 0;
  int32_t resident_wide[2] = {};  // the AG_SIM_KERNEL_WIDE A/B kernel's [counters]
  int32_t resident[512] = {};  // resident blocks [generate mode][768 lanes][shipped shape][truthful-only][768 / 1024 lanes][general][W][screened][counters]
  bool ship_shape = true;      // AG_OPT_SIM_SHIPPED_SHAPE: the compile-time shipped-shape general build
  bool gen_mode_all = false;   // AG_OPT_SIM_GENERAL_MODE = 1: the full general build for every population
  int64_t launch_cap = 0;  // AG_OPT_LAUNCH_AUCTIONS
  int64_t lrts_chunk = 0;  // AG_OPT_LRTS_BLOCK_SAMPLES
  bool wide = false;  // 1 auction per lane by default: higher occupancy, faster when sustained
  bool catalog = false;
  bool values_positive = false;  // every catalogue value > 0: the f32 item screens apply
  bool ora_catalog = false;  // catalogue within k_oracle's bounds (ag_sim_oracle.h)
  int32_t sim_kernel = AG_SIM_KERNEL_AUTO;  // AG_OPT_SIMULATE_KERNEL
  int32_t grid_per_cu = 0;                  // AG_OPT_SIM_BLOCKS_PER_CU (0: as many as fit)
  int32_t block_threads = 0;                // AG_OPT_SIM_BLOCK_THREADS (0: auto)
  int32_t resident_ora[4] = {};             // resident blocks of k_oracle [generate][counters]
  // general populations (anything beyond OracleAllocator + TruthfulBidder)
  bool general = false, has_lrts = false, has_shading = false, lrts_loaded = false;
  int32_t ts_sample = 1;
  int32_t *h_akind = nullptr;  // host copy of the allocator kinds [N]
  int32_t *h_bkind = nullptr;  // host copy of the bidder kinds [N]
  bool dr_loaded = false, dr_any_init = false;  // learner models loaded; some bid from a policy
  bool vl_any_search = false;                    // some ValueLearningBidder bids by search
  int64_t bidder_chunk = 0;                      // AG_OPT_BIDDER_BLOCK_SAMPLES (0: default)
  int64_t bidder_cache = -1;                     // AG_OPT_BIDDER_RECORD_CACHE (-1: default)
  uint64_t fit_noise_seed = 0;                   // AG_OPT_FIT_NOISE_SEED
  ag_dr_ws dr;
  int32_t *d_akind = nullptr, *d_bkind = nullptr;
  int32_t *d_kag = nullptr;    // [N] each agent's own item count (ag_set_agent_items); lazily allocated
  bool ragged = false;         // some agent has fewer than K items
  double *d_pg = nullptr, *d_gs = nullptr;
  float *d_tsm = nullptr, *d_tsq = nullptr, *d_tsprev = nullptr;  // LR-TS m, q, prev_iter_m
  ag_lrts_ws lrts;
  int32_t *d_status = nullptr;  // [N] per-agent update status (ag_empirical_update)
};

// Frees the LR-TS training workspace (ag_lrts.hip).
void ag_lrts_release(ag_ctx *c);
// Frees the DoublyRobustBidder workspace (ag_dr.hip).
void ag_dr_release(ag_ctx *c);

struct AgDeviceGuard {
  int prev = -1;
  explicit AgDeviceGuard(int dev) {
    if (hipGetDevice(&prev) == hipSuccess && prev != dev) (void)hipSetDevice(dev);
    else prev = -1;
  }
  ~AgDeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};
