/*
 * auctiongym.h -- C-ABI of the MI355X-native AuctionGym hot path (libauctiongym_hip.so).
 *
 * The drop-in boundary for
 *     Auction.simulate_opportunity -> Agent.bid -> {First,Second}Price.allocate -> Agent.charge
 * of the reference (soopark0221/auction-gym, src/). The reference is pure Python and has
 * no FFI; each entry point below names the reference interface it replaces, and
 * INTEGRATION.md shows the ctypes stub a maintainer would add on the reference side.
 *
 * Conventions
 *  - Every call returns AG_OK (0) or a negative ag_status; ag_last_error() describes it.
 *  - Plain pointers and sizes only. "dev" pointers are device (HBM) pointers on the ctx's
 *    device (hipMalloc or a torch tensor's data_ptr); "host" pointers are host memory.
 *  - Batched arrays are structure-of-arrays: a per-(auction, slot) array is [P][B]
 *    (slot-major, auction index fastest) so lane i of a wave touches auction i: coalesced.
 *  - Hot calls (ag_allocate, ag_simulate, ag_generate) allocate nothing, never
 *    synchronise and are stream-ordered on `stream` (a hipStream_t, NULL = default):
 *    they may be captured into a hipGraph.
 *  - One ag_ctx per process and device; a ctx is not thread-safe.
 *  - Every struct passed by pointer (ag_batch_in, ag_batch_out, ag_lrts_samples,
 *    ag_shading_samples) starts with `struct_size` = sizeof(struct) as the caller compiled
 *    it. A binding written against another layout is refused with AG_ERR_INVALID before
 *    any other field is read (AG_STRUCT_INIT sets it in C).
 */
#ifndef AUCTIONGYM_H
#define AUCTIONGYM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AG_ABI_VERSION 17

typedef enum ag_status {
  AG_OK = 0,
  AG_ERR_INVALID = -1,     /* bad argument (reference: ValueError, e.g. rng.choice with P > N) */
  AG_ERR_UNSUPPORTED = -2, /* shape / plugin kind this build does not implement */
  AG_ERR_HIP = -3,         /* HIP runtime error */
  AG_ERR_STATE = -4        /* call order (e.g. simulate before ag_load_catalog) */
} ag_status;

/* Allocation mechanisms: src/AuctionAllocation.py:11-23 (FirstPrice), :26-34 (SecondPrice). */
typedef enum ag_mechanism { AG_FIRST_PRICE = 0, AG_SECOND_PRICE = 1 } ag_mechanism;

/* Allocator plugins (src/BidderAllocation.py). */
typedef enum ag_allocator_kind {
  AG_ALLOCATOR_ORACLE = 0, /* OracleAllocator, src/BidderAllocation.py:71-82 */
  AG_ALLOCATOR_LRTS = 1    /* PyTorchLogisticRegressionAllocator (Thompson sampling),
                              src/BidderAllocation.py:21-68, src/Models.py:18-48 */
} ag_allocator_kind;

/* Bidder plugins (src/Bidder.py). */
typedef enum ag_bidder_kind {
  AG_BIDDER_TRUTHFUL = 0,         /* TruthfulBidder, src/Bidder.py:28-35 */
  AG_BIDDER_EMPIRICAL_SHADED = 1, /* EmpiricalShadedBidder, src/Bidder.py:38-58 */
  AG_BIDDER_VALUE_LEARNING = 2,   /* ValueLearningBidder, src/Bidder.py:156-333 */
  AG_BIDDER_POLICY_LEARNING = 3,  /* PolicyLearningBidder, src/Bidder.py:336-439 */
  AG_BIDDER_DOUBLY_ROBUST = 4     /* DoublyRobustBidder, src/Bidder.py:442-623 */
} ag_bidder_kind;

/* What a learning bidder (ValueLearning / PolicyLearning / DoublyRobust) bids from
 * (ag_set_dr_state `initialised`, set by ag_bidder_update): */
typedef enum ag_learner_state {
  AG_LEARNER_UNINITIALISED = 0, /* gamma ~ N(prev_gamma, gamma_sigma) (src/Bidder.py:174-179,
                                   :351-356, :458-463): gamma_raw input */
  AG_LEARNER_POLICY = 1,        /* the fitted policy's rsample (:198-203, :358-362, :464-470):
                                   policy_eps input */
  AG_LEARNER_SEARCH = 2         /* ValueLearningBidder 'search': argmax of the win-rate model's
                                   utility over 128 sorted U(0.1, 1) gammas (:180-196) */
} ag_learner_state;

/* Per-agent bidder modes (ag_set_bidder_modes): ValueLearningBidder inference ... */
typedef enum ag_vl_inference { AG_VL_SEARCH = 0, AG_VL_POLICY = 1 } ag_vl_inference;
/* ... and PolicyLearningBidder loss (src/Models.py:174-199; 'Doubly Robust' needs utility
 * estimates the PolicyLearningBidder never passes: the reference fails there). */
typedef enum ag_pl_loss {
  AG_PL_LOSS_REINFORCE = 0,
  AG_PL_LOSS_REINFORCE_OFFPOLICY = 1,
  AG_PL_LOSS_TRPO = 2,
  AG_PL_LOSS_PPO = 3
} ag_pl_loss;

/* Per-agent counters produced by ag_simulate: the quantities src/main.py:131-147 reads
 * from Agent (src/Agent.py:70-118) after each iteration, as sums over the agent's logs. */
typedef enum ag_counter {
  AG_C_NET = 0,          /* Agent.net_utility        += value*outcome - price (won)   */
  AG_C_GROSS,            /* Agent.gross_utility      += value*outcome (won)           */
  AG_C_ALLOC_REGRET,     /* get_allocation_regret:  best_ev - true_ctr*value          */
  AG_C_EST_REGRET,       /* get_estimation_regret:  est_ctr*value - true_ctr*value    */
  AG_C_OVERBID,          /* get_overbid_regret:     (price - second_price)*won        */
  AG_C_UNDERBID,         /* get_underbid_regret:    (price-bid)*!won*(price<true*val) */
  AG_C_CTR_SQERR,        /* get_CTR_RMSE numerator: (true_ctr - est_ctr)^2            */
  AG_C_CTR_BIAS,         /* get_CTR_bias numerator: est_ctr/true_ctr over won logs    */
  AG_C_BEST_EV,          /* mean best expected value numerator (src/main.py:147)      */
  AG_C_N_LOGS,           /* number of log records (participations)                   */
  AG_C_N_WON,            /* number of won log records                                 */
  AG_C_PAID,             /* sum of prices charged (revenue = sum over agents)         */
  AG_NUM_COUNTERS
} ag_counter;

/* Counters are accumulated EXACTLY as fixed-point sums: every per-record term is rounded
 * to a multiple of 2^-AG_FX_FRAC_BITS and the sum is held in AG_FX_LIMBS int64 limbs of
 * AG_FX_LIMB_BITS bits (value = sum_j limb_j * 2^(j*AG_FX_LIMB_BITS - AG_FX_FRAC_BITS)),
 * so results are independent of grid size, block order, batch split and GPU count.
 * Limb arrays can be summed across GPUs with an int64 all-reduce and then normalised.
 * AG_C_NET is held as AG_C_GROSS - AG_C_PAID (each record's net term value*outcome -
 * price is then rounded as two terms). */
#define AG_FX_FRAC_BITS 36
#define AG_FX_LIMB_BITS 42
#define AG_FX_LIMBS 3

typedef struct ag_shape {
  int32_t num_agents;         /* N: len(auction.agents)                                  */
  int32_t num_participants;   /* P: num_participants_per_round (src/Auction.py:42)       */
  int32_t num_items;          /* K: num_items per agent (one value for all agents)       */
  int32_t embedding_size;     /* E: true context dims; D = E + 1 with the intercept      */
  int32_t obs_embedding_size; /* OE: observable dims (src/Auction.py:36)                 */
  int32_t mechanism;          /* ag_mechanism                                            */
  int32_t num_slots;          /* must be 1 (max_slots is hard-coded, src/main.py:37)     */
  int32_t reserved;
  double embedding_var;       /* context ~ N(0, embedding_var) (src/Auction.py:33)       */
} ag_shape;

typedef struct ag_ctx ag_ctx;

/* C initialiser of the struct_size field: ag_batch_in in = {AG_STRUCT_INIT(ag_batch_in), ...}; */
#define AG_STRUCT_INIT(type) ((uint64_t)sizeof(type))

/* Replay inputs of B auctions (dev). The reference draws these from its numpy Generator
 * in the order src/Auction.py:33 (normal), :42 (choice), :65 (binomial's next_double). */
typedef struct ag_batch_in {
  uint64_t struct_size; /* sizeof(ag_batch_in) (ABI 16)                                   */
  const double *ctx;   /* [E][B] true context without the intercept                      */
  const int32_t *part; /* [P][B] participating agent index per slot, P distinct of N     */
  const double *u;     /* [B]    uniform in [0,1) consumed by binomial(1, CTR[winner])   */
  const double *gamma_raw; /* [P][B] raw rng.normal(prev_gamma, gamma_sigma) draw of a
                              shading bidder (src/Bidder.py:51,177,354,461); NULL if none */
  const float *ts_noise;   /* [P][T][K*(OE+1)][64], T = ceil(B/64): torch.normal(0,
                              1/sqrt(q)) of an LR-TS participant (src/Models.py:31) in tiles
                              of 64 auctions -- element (slot s, auction i, coefficient c)
                              at ((s*T + i/64)*K*(OE+1) + c)*64 + i%64, so a wave reads each
                              coefficient of its 64 auctions as one 256-B row and a tile's
                              rows are contiguous; NULL if none / no sampling */
  const float *policy_eps; /* [P][B] the rsample draw (torch, standard normal) of a
                              learning bidder bidding from its fitted policy
                              (src/Bidder.py:198-203, :358-362, :466-470); NULL if none */
  const double *gamma_grid; /* [P][128][B] the rng.uniform(0.1, 1.0, 128) grid of a
                              ValueLearningBidder bidding by search (src/Bidder.py:184-186),
                              any order; NULL if none */
  const int32_t *ts_noise_index; /* [P][B] compact Thompson-noise layout (mixed populations):
                              NULL = ts_noise is the dense tiling above; else only the
                              LR-TS pairs are stored, pair (s, i) being the j-th LR-TS pair
                              of the batch in (slot, auction) order, j = ts_noise_index[s*B+i],
                              its coefficient c at ((j/64)*K*(OE+1) + c)*64 + j%64 -- made by
                              ag_ts_noise_index over the same part (ABI 16) */
} ag_batch_in;

/* Outputs of B auctions (dev). Any pointer may be NULL to skip that array. */
typedef struct ag_batch_out {
  uint64_t struct_size;  /* sizeof(ag_batch_out) (ABI 17; AG_BATCH_OUT_V16_SIZE accepted) */
  int32_t *winner;       /* [B] winning slot (argsort(-bids)[0]; ties -> lowest slot)    */
  double *price;         /* [B] price charged (NaN when P == 1: nobody charged)          */
  double *second_price;  /* [B] second highest bid (NaN when P == 1)                     */
  uint8_t *outcome;      /* [B] click of the winner, binomial(1, true CTR)               */
  int32_t *item;         /* [P][B] item chosen by the participant (Agent.select_item)    */
  double *bid;           /* [P][B] bid submitted                                        */
  double *est_ctr;       /* [P][B] estimated CTR of the chosen item                     */
  double *true_ctr;      /* [P][B] true CTR of the chosen item (src/Auction.py:52-53)    */
  double *best_ev;       /* [P][B] max_k true_CTR_k * value_k                           */
  double *gamma;         /* [P][B] shading factor of shading bidders (NaN otherwise)     */
  double *propensity;    /* [P][B] density of gamma under the bidder's logging policy:
                            the Gaussian around prev_gamma (uninitialised learning
                            bidders) or the fitted policy's (DR); NaN otherwise          */
  /* ABI 17 (opt-in; NULL = not written): winner and outcome as one word. A byte-wide
   * outcome stream is the costliest of the per-field arrays: with this word instead of
   * `winner` + `outcome` the headline kernel runs 5-7 % faster (profiles/r05i_ab_packed.log). */
  uint32_t *winner_outcome; /* [B] winner | outcome << 31 (winner: the slot, as `winner`)    */
} ag_batch_out;
/* Size of the ABI 15/16 ag_batch_out (without winner_outcome): still accepted as struct_size,
 * winner_outcome then reads as NULL. */
#define AG_BATCH_OUT_V16_SIZE ((uint64_t)(8 + 11 * sizeof(void *)))


/* Create a context on `device` for one auction population (src/main.py:98-109
 * instantiate_auction). Validates the shape; allocates device workspace once. */
int ag_create(int32_t device, const ag_shape *shape, ag_ctx **out);
int ag_destroy(ag_ctx *ctx);

/* Per-agent plugin kinds, host [N] (src/main.py:77-95 instantiate_agents: the eval of
 * allocator/bidder class names). Default: all OracleAllocator + TruthfulBidder. */
int ag_set_agent_kinds(ag_ctx *ctx, const int32_t *allocator_kind, const int32_t *bidder_kind);

/* Per-agent plugin parameters, host [N]: kinds as above; prev_gamma / gamma_sigma of
 * shading bidders (init_gamma, gamma_sigma kwargs; may be NULL when there are none). */
int ag_set_agent_params(ag_ctx *ctx, const int32_t *allocator_kind, const int32_t *bidder_kind,
                        const double *prev_gamma, const double *gamma_sigma);

/* Each agent's own item count (src/main.py:61,66 num_items per agent config; Agent.__init__):
 * host int32 [N], each in [1, K], K = ag_shape.num_items the largest. The catalogue
 * (ag_load_catalog) and LR-TS models (ag_load_lrts) stay [N][K][...]: an agent's rows beyond
 * its count are padding, values 0 (never the first argmax of CTR * value) and LR-TS rows 0 (no
 * samples reach them: the update leaves them 0). The general kernel scores an LR-TS agent's
 * Thompson choice over its own rows (the sgemv block / remainder rows follow its count).
 * NULL: every agent has K. */
int ag_set_agent_items(ag_ctx *c, const int32_t *num_items);

/* LR-TS posterior of every AG_ALLOCATOR_LRTS agent, host float32 [N][K][OE+1] m, q and
 * prev_m (PyTorchLogisticRegression.m / .q / .prev_iter_m, src/Models.py:21-24; rows of
 * other agents ignored; prev_m NULL = m, as at construction); thompson_sampling: add the
 * batch's ts_noise to m for the item choice (src/Models.py:30-31). */
int ag_load_lrts(ag_ctx *ctx, const float *m, const float *q, const float *prev_m,
                 int32_t thompson_sampling);

/* Options (ag_set_option). */
typedef enum ag_option {
  AG_OPT_ITEM_SEARCH = 0,  /* value: ag_item_search */
  AG_OPT_LANE_AUCTIONS = 1, /* value: 1 (default) or 2 (16-B SoA accesses when B is even) */
  AG_OPT_LAUNCH_AUCTIONS = 2, /* value: cap on auctions per k_simulate launch (0 = the exact-
                                 counter capacity of the resident grid); larger batches run
                                 as consecutive launches with identical results */
  AG_OPT_LRTS_BLOCK_SAMPLES = 3, /* value: samples per workgroup of the LR-TS training kernel
                                   (0 = 16 per lane = 4096); fewer spreads an agent over more
                                   workgroups -- identical results (exact sums) */
  AG_OPT_BIDDER_BLOCK_SAMPLES = 4, /* value: records per workgroup of the learning bidders'
                                   trainer (0 = default: the exact-sum learners share the resident
                                   grid, >= 1024 records per workgroup; PolicyLearningBidder 8192);
                                   identical results for the exact-sum fits, the policy-learning
                                   fits' fixed-order sums follow the split */
  AG_OPT_FIT_NOISE_SEED = 5,      /* value: seed of the synthetic rsample noise of ag_bidder_update
                                   called with noise == NULL (default 0) */
  AG_OPT_BIDDER_RECORD_CACHE = 6, /* value: most records per workgroup the learning bidders'
                                   trainer stages in LDS (-1 = default: as many as fit; 0 = none,
                                   every epoch reads the store); identical results */
  AG_OPT_SIMULATE_KERNEL = 7,     /* value: ag_sim_kernel; identical results */
  AG_OPT_SIM_BLOCKS_PER_CU = 8,   /* value: workgroups per CU of the simulate kernels' persistent
                                     grids (0 = default: every workgroup that fits); a cap, never
                                     above what fits; identical results */
  AG_OPT_SIM_BLOCK_THREADS = 9,   /* value: lanes per workgroup of the general simulate kernel:
                                     0 = auto (1024 when the population's LDS would keep fewer than
                                     16 waves resident per CU with 256-lane workgroups), 256 or
                                     1024; identical results */
  AG_OPT_SIM_GENERAL_MODE = 10,   /* value: 0 = auto (TruthfulBidder-only populations run the
                                     general kernel built without the bid-shading code: fewer
                                     VGPRs), 1 = always the full general build; identical results */
  AG_OPT_SIM_SHIPPED_SHAPE = 11   /* value: 1 (default) = general populations of the shipped
                                     shape (E = 5, OE = 4) run a build of the general kernel
                                     with the LR-TS model width compile-time; 0 = the
                                     runtime-width build; identical results */
} ag_option;

typedef enum ag_sim_kernel {
  AG_SIM_KERNEL_AUTO = 0,   /* OracleAllocator + TruthfulBidder populations whose catalogue
                               values lie in (0, 1024): the dedicated Oracle kernel; else the
                               general one */
  AG_SIM_KERNEL_GENERIC = 1, /* always the general simulate kernel (A/B and parity tests) */
  AG_SIM_KERNEL_FUSED = 2,   /* retired (round 4): the dedicated shipped-shape population
                                kernel k_pop no longer ships -- the general kernel was as fast
                                on every line; ag_set_option refuses these two values */
  AG_SIM_KERNEL_SPLIT = 3,
  AG_SIM_KERNEL_WIDE = 4     /* general populations: the runtime-P kernel (slot results not
                                kept in registers, resolved again for the counters) at any P;
                                A/B of wide auctions, identical results */
} ag_sim_kernel;

typedef enum ag_item_search {
  AG_ITEM_SEARCH_AUTO = 0,  /* f32 screen of all K items, exact FP64 re-score of the items
                               within 2^-10 of the best (same results, bit for bit) */
  AG_ITEM_SEARCH_EXACT = 1  /* exact FP64 score of every item (the reference's loop) */
} ag_item_search;

int ag_set_option(ag_ctx *ctx, int32_t option, int64_t value);

/* Item catalogue, host: item_emb [N][K][E+1] (embeddings with the intercept column,
 * src/main.py:60-72) and item_val [N][K]; replaces OracleAllocator.update_item_embeddings
 * (src/BidderAllocation.py:78-79) and Auction.agent2items / agents2item_values. */
int ag_load_catalog(ag_ctx *ctx, const double *item_emb, const double *item_val);

/* Batched AllocationMechanism.allocate(bids, num_slots=1) (src/AuctionAllocation.py:7-8,
 * 19-22, 32-34) over B auctions: bids dev [P][B] -> winner/price/second_price dev [B].
 * FirstPrice: price = highest bid; SecondPrice: price = second highest. P == 1: FirstPrice
 * price = the bid, SecondPrice price = NaN, second_price = NaN (empty arrays). */
int ag_allocate(ag_ctx *ctx, const double *bids, int64_t B, int32_t *winner, double *price,
                double *second_price, void *stream);

/* B rounds of Auction.simulate_opportunity (src/Auction.py:28-74) in replay mode.
 * counters_fx: dev int64 [N][AG_NUM_COUNTERS][AG_FX_LIMBS], ACCUMULATED (zero it at the
 * start of an iteration, like Agent.clear_utility); may be NULL. */
int ag_simulate(ag_ctx *ctx, int64_t B, const ag_batch_in *in, ag_batch_out *out,
                int64_t *counters_fx, void *stream);

/* Generate mode: B rounds of Auction.simulate_opportunity whose inputs are drawn on the chip
 * inside the simulate kernel, the same bits ag_generate(seed, first_auction, B) -- and, for
 * general populations, ag_generate_noise(seed, first_auction, B) -- write (so the outputs and
 * counters equal ag_generate (+ ag_generate_noise) followed by ag_simulate); nothing but the
 * catalogue and the agents' parameters is read from HBM. OracleAllocator + TruthfulBidder
 * populations whose catalogue values lie in (0, 1024), P <= 8, E + 1 <= 8, K <= 16; general
 * populations (LR-TS allocators: their Thompson noise; shading and learning bidders: their
 * Gaussian or rsample draws) in the shipped shape -- E = 5, OE = 4, K <= 16, positive values,
 * P <= 8 -- except ValueLearningBidders bidding by search (their grids are not drawn);
 * otherwise AG_ERR_UNSUPPORTED. (Round 6: the general populations; ABI unchanged.) */
int ag_simulate_generated(ag_ctx *ctx, uint64_t seed, uint64_t first_auction, int64_t B, ag_batch_out *out,
                          int64_t *counters_fx, void *stream);

/* Synthetic replay inputs for auctions [first_auction, first_auction + B) (dev, SoA):
 * Philox4x32-10 keyed by seed and the GLOBAL auction index, so a sharded batch is
 * bit-identical to the unsharded one. ctx ~ N(0, embedding_var) (Box-Muller in float32 from
 * 32-bit uniforms, ABI 17), part = P distinct of N (Floyd), u ~ U[0,1) with 53 bits. */
int ag_generate(ag_ctx *ctx, uint64_t seed, uint64_t first_auction, int64_t B, double *ctx_out,
                int32_t *part_out, double *u_out, void *stream);

/* Synthetic per-participant noise for the participants `part` (dev [P][B]) of auctions
 * [first_auction, first_auction + B): gamma_raw [P][B] = prev_gamma + gamma_sigma * z for
 * shading bidders (NaN otherwise), ts_noise (tiled as in ag_batch_in) = z * (1 / sqrtf(q)) for
 * LR-TS agents (0 otherwise), policy_eps [P][B] = z for every slot; any output may be NULL.
 * Same Philox key / counter scheme; z are float32 Box-Muller normals from 32-bit uniforms, four
 * per Philox call (round 6; before, one FP64 pair per call). */
/* Synthetic search grids gamma_grid [P][128][B] (U(0.1, 1), Philox as ag_generate_noise,
 * unsorted: the search takes the smallest gamma among tied maxima) for every slot. */
int ag_generate_search_grid(ag_ctx *ctx, uint64_t seed, uint64_t first_auction, int64_t B, double *gamma_grid,
                            void *stream);

int ag_generate_noise(ag_ctx *ctx, uint64_t seed, uint64_t first_auction, int64_t B,
                      const int32_t *part, double *gamma_raw, float *ts_noise, float *policy_eps,
                      void *stream);

/* Compact Thompson-noise layout (ag_batch_in.ts_noise_index, ABI 16): index dev int32 [P][B]
 * = the rank of each LR-TS pair (slot s, auction i) among the batch's LR-TS pairs in
 * (s, i) order, -1 for other agents' pairs; *pairs (host) = their number, so the compact
 * ts_noise holds ceil(pairs/64)*64*K*(OE+1) floats. The reference draws Thompson noise only
 * for LR-TS agents (src/Models.py:30-31 via src/Agent.py:35): a mixed population then reads
 * no noise for its other slots. Synchronises (the count comes back to the host). */
int ag_ts_noise_index(ag_ctx *ctx, int64_t B, const int32_t *part, int32_t *index, int64_t *pairs,
                      void *stream);

/* ag_generate_noise's ts_noise in the compact layout of `index`: the same values for every
 * LR-TS pair, nothing written for the others. */
int ag_generate_ts_noise_compact(ag_ctx *ctx, uint64_t seed, uint64_t first_auction, int64_t B,
                                 const int32_t *part, const int32_t *index, float *ts_noise, void *stream);

/* ---- Replay-mode draws on the host (src/Auction.py:30-42, :65; src/main.py:29) -----------
 * B rounds of the reference's numpy draws in its order, without a Python round trip per
 * round: per round rng.integers(1, max_slots + 1) (nothing drawn for one slot),
 * rng.normal(0, embedding_var, E), rng.choice(N, P, replace=False), for every slot whose
 * agent is a shading bidder in its Gaussian state rng.normal(prev_gamma, gamma_sigma)
 * (src/Bidder.py:51, 177, 354, 461), then the next_double rng.binomial(1, p) consumes.
 * The generator is numpy's PCG64 bit generator: its state (bit_generator.state) goes in and
 * comes back advanced past the B rounds; the distributions are numpy's own (libnpyrandom).
 * Host arrays, SoA with leading dimension B (the ag_batch_in layout): ctx [E][B],
 * part [P][B], gamma_raw [P][B] (NaN where nothing is drawn; may be NULL when shading is
 * NULL), u [B]. shading: host uint8 [N] (NULL: none), prev_gamma / gamma_sigma host [N].
 * Draws that come from torch's generator (Thompson noise, fitted-policy rsample) are not
 * made here. AG_ERR_INVALID with numpy's message when P > N. */
typedef struct ag_pcg64_state {
  uint64_t struct_size; /* sizeof(ag_pcg64_state) (ABI 15)                                  */
  uint64_t state_hi, state_lo; /* the 128-bit LCG state                                     */
  uint64_t inc_hi, inc_lo;     /* the 128-bit increment                                     */
  int32_t has_uint32;          /* numpy's buffered upper half of a 64-bit draw ...          */
  uint32_t uinteger;           /* ... and its value                                         */
} ag_pcg64_state;

int ag_replay_draw(ag_pcg64_state *rng, int64_t B, int32_t N, int32_t P, int32_t E, double embedding_var,
                   int32_t max_slots, const uint8_t *shading, const double *prev_gamma, const double *gamma_sigma,
                   double *ctx, int32_t *part, double *gamma_raw, double *u);

/* ag_replay_draw_population -- B rounds of a general population's draws, in the reference's
 * order (src/Auction.py:30-42, :65; per participant slot, src/Agent.py:44-53: the LR-TS
 * allocator's Thompson draw torch.normal(0, 1/sqrt(q)) of src/Models.py:31, then the
 * bidder's: one rsample of a fitted policy (src/Models.py:87-88, :160-161), or the search
 * grid rng.uniform(0.1, 1, 128) sorted (src/Bidder.py:184-186), or an uninitialised shading
 * bidder's rng.normal(prev_gamma, gamma_sigma) (src/Bidder.py:51, 177, 354, 461)).
 * Replaces the per-round Python loop (auctiongym_amd/replay.py draw_round_population).
 * numpy's draws as ag_replay_draw; torch's from its CPU generator, restated: mt19937 (the
 * state blob of torch.get_rng_state(), 5056 bytes: the_initial_seed u64 @0, left i32 @8,
 * seeded i32 @12, next u64 @16, state u64[624] @24, normal_y f64 @5024, normal_is_valid i32
 * @5040, next_float_normal f32 @5048, its valid flag u8 @5052) goes in and comes back
 * advanced (hand it to torch.set_rng_state); Thompson noise = normal_fill<float> of K*Do
 * values (24-bit uniforms, Box-Muller over blocks of 16, the last 16 recomputed when
 * K*Do % 16 != 0; glibc logf / cosf / sinf) times ts_std; rsample = normal_distribution
 * <double> with its cached second value (glibc log1p / cos / sin). Per agent [N]: shading
 * (uint8, with prev_gamma / gamma_sigma), ts (uint8, with ts_std [N][KDo] = 1/sqrt(q) as
 * torch computes it; ts_kdo [N] int32: an agent's own K*Do when it has fewer items than K --
 * ag_set_agent_items -- its draws fill the first ts_kdo[a] coefficients; NULL: all KDo),
 * policy (uint8), search (uint8); each may be NULL (none). Outputs:
 * ctx, part, u, gamma_raw as ag_replay_draw; ts_noise in the kernel's tile layout
 * [P][ceil(B/64)][KDo][64] (ag_batch_in.ts_noise, zeros where nothing is drawn) when ts;
 * policy_eps [P][B] float (0 where nothing is drawn) when policy; gamma_grid [P][128][B]
 * (0 where nothing is drawn) when search. Identical numbers and generator states to the
 * Python loop (tests/test_host.py::test_replay_population_draws_match_python). */
/* `epochs` x torch.empty(n).normal_() from torch's CPU generator: the learning bidders'
 * per-epoch rsample draws of their policy fits (src/Models.py:160, :87 via src/Bidder.py:
 * 278-303, :574-595), epoch e at out[e * n + i] (host float32 [epochs][n]); torch_state: the
 * torch.get_rng_state() blob (host, 5056 B), advanced in place as the reference's draws
 * advance the global generator. Host only (no device). */
int ag_torch_normal_epochs(uint8_t *torch_state, int64_t torch_state_bytes, int64_t n, int32_t epochs, float *out);

int ag_replay_draw_population(ag_pcg64_state *rng, uint8_t *torch_state, int64_t torch_state_bytes, int64_t B,
                              int32_t N, int32_t P, int32_t E, double embedding_var, int32_t max_slots,
                              const uint8_t *shading, const double *prev_gamma, const double *gamma_sigma,
                              const uint8_t *ts, const float *ts_std, int32_t KDo, const int32_t *ts_kdo,
                              const uint8_t *policy, const uint8_t *search, double *ctx, int32_t *part,
                              double *gamma_raw, double *u, float *ts_noise, float *policy_eps, double *gamma_grid);

/* ---- LR-TS allocator update (Agent.update -> PyTorchLogisticRegressionAllocator.update,
 * src/Agent.py:79-91, src/BidderAllocation.py:29-65) ------------------------------------
 * The won samples of LR-TS agents (Agent.update's won_mask) accumulate in a caller-owned
 * device store between updates; reset *count to 0 where the reference calls
 * Agent.clear_logs. Records are unordered: the update's sums are exact, so the order
 * samples arrive in (or the rank that collected them) cannot change the result. */
#define AG_LRTS_MAX_EPOCHS 16384 /* epochs = 8192 * 2 (src/BidderAllocation.py:38) */
#define AG_LRTS_MAX_DO 8         /* OE + 1 <= 8; K * (OE + 1) <= 64 */

typedef struct ag_lrts_samples {
  uint64_t struct_size; /* sizeof(ag_lrts_samples) (ABI 15)                               */
  uint32_t *key;     /* dev [capacity]: agent << 16 | item << 1 | outcome               */
  float *x;          /* dev [OE+1][capacity]: float32(observed context), 1.0             */
  int64_t capacity;
  uint64_t *count;   /* dev [1]: records appended; > capacity = overflow (update fails)  */
} ag_lrts_samples;

/* Append the won LR-TS samples of one simulated batch (the in/out of ag_simulate; needs
 * in.ctx, in.part, out.winner, out.item, out.outcome). Hot call: stream-ordered. */
int ag_lrts_collect(ag_ctx *ctx, int64_t B, const ag_batch_in *in, const ag_batch_out *out,
                    const ag_lrts_samples *samples, void *stream);

/* Train every LR-TS agent on its samples in the store: the reference's epoch loop (Adam
 * lr 2e-3, ReduceLROnPlateau, early stop), the Laplace update of q and prev_m = m; agents
 * with < 2 samples are left unchanged. The updated posterior stays on the device for the
 * next ag_simulate. Synchronises `stream` (reads the sample count). epochs: host [N]
 * epochs run per agent (0: not trained), may be NULL; loss_trace: dev float32
 * [N][AG_LRTS_MAX_EPOCHS] per-epoch loss.item(), may be NULL. Arithmetic:
 * oracle/ag_oracle.c ora_lrts_update. */
int ag_lrts_update(ag_ctx *ctx, const ag_lrts_samples *samples, int32_t *epochs,
                   float *loss_trace, void *stream);

/* Current LR-TS posterior, host float32 [N][K][OE+1] (any may be NULL). Synchronises. */
int ag_lrts_read(ag_ctx *ctx, float *m, float *q, float *prev_m);

/* ---- Shading bidders' update (Agent.update -> EmpiricalShadedBidder.update,
 * src/Agent.py:79-94, src/Bidder.py:60-147) ------------------------------------------
 * Every participation of a shading bidder (its `gammas` and the net utilities the update
 * derives from the logs, src/Bidder.py:62-63) accumulates in a caller-owned store;
 * reset *count where the reference calls Agent.clear_logs. Records are unordered. */
typedef struct ag_shading_samples {
  uint64_t struct_size; /* sizeof(ag_shading_samples) (ABI 15)                           */
  int32_t *agent;    /* dev [capacity]                                                   */
  double *gamma;     /* dev [capacity]: the shading factor of the bid                    */
  double *utility;   /* dev [capacity]: value * outcome - price if won, else 0           */
  int64_t capacity;
  uint64_t *count;   /* dev [1]: records appended; > capacity = overflow (update fails)  */
  /* the learning bidders' update also needs (may be NULL for EmpiricalShaded only): */
  double *ctr;       /* dev [capacity]: estimated CTR of the bid                         */
  double *value;     /* dev [capacity]: value of the chosen item                         */
  double *propensity;/* dev [capacity]: logging propensity of gamma                      */
  uint8_t *won;      /* dev [capacity]                                                   */
  uint64_t *order;   /* dev [capacity]: (global auction index) * P + slot -- the record's
                        place in the agent's log order (the DR fit's noise follows it)    */
} ag_shading_samples;

/* Append the records of EmpiricalShaded and DoublyRobust bidders of one simulated batch of
 * auctions [first_auction, first_auction + B) (needs in.part, out.winner, out.item,
 * out.outcome, out.price, out.gamma; out.est_ctr and out.propensity when the store has ctr /
 * propensity). Hot call: stream-ordered. */
int ag_shading_collect(ag_ctx *ctx, int64_t first_auction, int64_t B, const ag_batch_in *in,
                       const ag_batch_out *out, const ag_shading_samples *samples, void *stream);

/* EmpiricalShadedBidder.update of every such agent from the store: the new prev_gamma is
 * written where ag_simulate reads it and, when prev_gamma (host [N]) is not NULL, copied
 * out (other agents' entries unchanged). Synchronises `stream`. AG_ERR_INVALID with the
 * reference's numpy message where the reference raises (no samples, one bucket, no bucket
 * with two samples). Arithmetic: oracle/ag_oracle.c ora_empirical_update. */
int ag_empirical_update(ag_ctx *ctx, const ag_shading_samples *samples, double *prev_gamma,
                        void *stream);
/* The same for the agents of host int32 [N] mask `agents` only (NULL: every one): the
 * reference's per-agent Agent.update (src/main.py:127-128) -- the other agents' prev_gamma and
 * errors are untouched. */
int ag_empirical_update_agents(ag_ctx *ctx, const ag_shading_samples *samples, const int32_t *agents,
                               double *prev_gamma, void *stream);

/* ---- Learning bidders: ValueLearningBidder, PolicyLearningBidder, DoublyRobustBidder ----
 * (src/Bidder.py:156-623). Per-agent model state, host float32 [N][16]:
 * PyTorchWinRateEstimator weight (3) and bias, then the policy's parameters on its forward
 * path (BidShadingContextualBandit.parameters(); for BidShadingPolicy the same layers, its
 * unused hidden layers left out): shared W 2x2, b 2; mu w 2, b; sigma w 2, b.
 * initialised [N]: ag_learner_state. */
int ag_set_dr_state(ag_ctx *ctx, const float *state, const int32_t *initialised);
int ag_get_dr_state(ag_ctx *ctx, float *state, int32_t *initialised);

/* Records per agent in a shading store (host int64 [N]); synchronises. */
int ag_shading_counts(ag_ctx *ctx, const ag_shading_samples *samples, int64_t *counts, void *stream);

/* DoublyRobustBidder.update of every DR agent from the store (Agent.update, src/Agent.py:
 * 79-94 -> src/Bidder.py:473-615): win-rate fit, imitation of the logging policy (first
 * update), doubly robust policy fit; afterwards the agents bid from their policies. The
 * store needs ctr, value, propensity, won and order; records are put in each agent's log
 * order (radix sort on agent, order). noise: dev float32, agent a's DR-fit rsample draws
 * at noise[noise_offsets[a] + e * n_a + i] for its i-th record in log order (n_a = its
 * record count, e < noise_epochs); epochs: host int32 [N][3] epochs run per fit
 * (may be NULL); traces: dev float32 [N][3][32768] per-epoch losses (may be NULL).
 * Synchronises. Arithmetic: oracle/ag_oracle_dr.c ora_dr_update. */
int ag_dr_update(ag_ctx *ctx, const ag_shading_samples *samples, const float *noise,
                 const int64_t *noise_offsets, int32_t noise_epochs, int32_t *epochs, float *traces,
                 void *stream);

/* ValueLearningBidder inference (AG_VL_*) / PolicyLearningBidder loss (AG_PL_LOSS_*) per
 * agent, host int32 [N] (entries of other agents ignored); the constructors' arguments
 * (src/Bidder.py:159-167, :339-346). Defaults: 'search', 'PPO'. */
int ag_set_bidder_modes(ag_ctx *ctx, const int32_t *modes);

/* Agent.update -> Bidder.update of EVERY learning bidder from the store, each agent on one
 * or more cooperating workgroups (AG_OPT_BIDDER_BLOCK_SAMPLES) running its fits in the
 * reference's order (src/Agent.py:79-94), in two launches (win-rate fits, then the rest):
 *  - DoublyRobustBidder (src/Bidder.py:473-615): as ag_dr_update;
 *  - ValueLearningBidder (:204-325): no won record -> the reference's fallback (nothing
 *    trained, status 1, bids revert to Gaussian shading); else the win-rate fit and, with
 *    inference 'policy', the policy fit (rsample noise as for DR, <= 16384 epochs);
 *  - PolicyLearningBidder (:364-431): imitation of the logging policy (first update), then
 *    the fit of its loss (no noise).
 * agents: host int32 [N], nonzero = update this agent (NULL: every learning bidder; the
 * reference updates agents one by one, src/main.py:127-128, and the torch draws of one
 * agent's update depend on the epochs the previous one ran). epochs host int32 [N][3] =
 * (win-rate, imitation, policy fit); status host int32 [N] (may be NULL): 0 trained, 1
 * fallback, -3 a noise-driven fit used all noise_epochs without stopping -- that agent's
 * state is left unchanged, call again with more noise epochs; traces dev float32
 * [N][3][32768] (may be NULL). AG_ERR_INVALID where the reference fails (no logs; a NaN
 * loss, where it exits). Synchronises. Arithmetic: oracle/ag_oracle_dr.c ora_dr_update /
 * ora_vl_update / ora_pl_update. */
int ag_bidder_update(ag_ctx *ctx, const ag_shading_samples *samples, const int32_t *agents, const float *noise,
                     const int64_t *noise_offsets, int32_t noise_epochs, int32_t *epochs, int32_t *status,
                     float *traces, void *stream);

/* ---- Resumable, record-parallel LR-TS allocator update ----
 * PyTorchLogisticRegressionAllocator.update (src/BidderAllocation.py:29-65: the epoch loop
 * :45-55, the Laplace q :58-63) as ONE LAUNCH PER EPOCH, each agent's state (m, Adam
 * moments, scheduler, loss history) in device memory between launches: G ranks holding shards
 * of the won samples SUM the int64 words totals[launch_index & 1] ([N][144], dev) over the
 * ranks after every ag_lrts_rp_epoch(launches = 1); every rank then ends with the posterior
 * ag_lrts_update computes in one process from all the samples, bit for bit. samples_total:
 * host int64 [N], each agent's won samples over all ranks (NULL: this process holds them
 * all); agents with < 2 of them are not trained (the reference's :33-34). totals: caller-owned
 * dev int64 [2][N][144]. The samples stay in the workspace until ag_lrts_rp_end. */
int ag_lrts_rp_begin(ag_ctx *ctx, const ag_lrts_samples *samples, const int32_t *agents, const int64_t *samples_total,
                     int64_t *totals, void *stream);
int ag_lrts_rp_epoch(ag_ctx *ctx, int32_t launches, int64_t *launch_index, void *stream);
/* Synchronises; training = agents still training (0: done). */
int ag_lrts_rp_poll(ag_ctx *ctx, int32_t *training, void *stream);
/* Every agent done: m, q, prev_m are where ag_simulate and ag_lrts_read read them; epochs host
 * int32 [N] (may be NULL). AG_ERR_STATE while an agent trains. */
int ag_lrts_rp_end(ag_ctx *ctx, int32_t *epochs, void *stream);

/* ---- Resumable, record-parallel update of the exact-sum learning bidders ----
 * ValueLearningBidder and DoublyRobustBidder (src/Bidder.py:204-325, :473-615; replaces the
 * per-epoch loops of src/Bidder.py:239-260, :278-323, :517-538, :574-595) as ONE LAUNCH PER
 * EPOCH with each learner's training state (model, Adam, scheduler, early stop, fit) in
 * device memory between launches. Two uses:
 *  - record-parallel over G ranks (one process per GPU, each holding the records of its own
 *    auction shard): after every ag_bidder_rp_epoch(launches = 1) the caller SUMs the int64
 *    words totals[launch_index & 1] ([N][32], dev) over the ranks in place (an all-reduce;
 *    the sums are exact integers) before the next call; every rank then steps to the same
 *    model, bit for bit the model ag_bidder_update fits in one process on all the records;
 *  - one process feeding a fit host-drawn rsample noise window by window (ag_bidder_rp_noise):
 *    a policy fit reaching an epoch outside the window waits (ag_bidder_rp_poll need_noise)
 *    with its state kept -- nothing is re-run.
 * records_total / records_base: host int64 [N], agent a's records over all ranks and the
 * global log-order index of this rank's first one (NULL: this process holds them all); the
 * synthetic rsample draws are keyed by that global index. agents: host int32 [N] mask (NULL:
 * every ValueLearning / DoublyRobust bidder; a PolicyLearningBidder is refused: its fits sum
 * floats in a fixed order). totals: caller-owned dev int64 [2][N][32]. The store's records
 * stay in the workspace until ag_bidder_rp_end: no other learning-bidder update in between. */
int ag_bidder_rp_begin(ag_ctx *ctx, const ag_shading_samples *samples, const int32_t *agents,
                       const int64_t *records_total, const int64_t *records_base, int64_t *totals, void *stream);
/* Queue `launches` epoch launches (stream-ordered, asynchronous); launch_index (host, may be
 * NULL) = the last launch's index: its rank totals are at totals + 32 N (launch_index & 1).
 * traces: dev float32 [N][3][32768] per-epoch losses (the rank holding global record 0), or NULL. */
int ag_bidder_rp_epoch(ag_ctx *ctx, int32_t launches, int64_t *launch_index, float *traces, void *stream);
/* One process holding every record (records_total / records_base NULL): the rest of the update
 * in persistent launches (every learner under training together, each one's per-epoch sum
 * overlapped with the others' epochs) until every learner is done or waits for noise
 * (ag_bidder_rp_poll tells which); the same state ag_bidder_rp_epoch steps, bit for bit, so the
 * two mix. Stream-ordered; AG_ERR_UNSUPPORTED on a rank holding part of the records. */
int ag_bidder_rp_run(ag_ctx *ctx, float *traces, void *stream);
/* The host-drawn rsample window of the noisy policy fits: noise dev float32, policy-fit epoch e
 * of record i (global index) at noise[(e - first_epoch) * noise_n + i], first_epoch <= e <
 * first_epoch + epochs; NULL: synthetic draws (AG_OPT_FIT_NOISE_SEED). */
int ag_bidder_rp_noise(ag_ctx *ctx, const float *noise, int64_t noise_n, int32_t first_epoch, int32_t epochs);
/* After the queued launches (synchronises): per agent, host int32 [N] each (any may be NULL):
 * fit = the fit in progress (0 win count, 1 win-rate, 2 estimated utilities, 3 imitation, 4
 * policy) or -1 done; epoch = epochs run in it; need_noise = the policy epoch waiting for
 * noise, or -1. */
int ag_bidder_rp_poll(ag_ctx *ctx, int32_t *fit, int32_t *epoch, int32_t *need_noise, void *stream);
/* Every trained agent done: its model and bidding state applied as ag_bidder_update applies
 * them; epochs host int32 [N][3], status host int32 [N] as ag_bidder_update's (may be NULL).
 * AG_ERR_INVALID on a NaN loss (the reference exits), AG_ERR_STATE while an agent trains. */
int ag_bidder_rp_end(ag_ctx *ctx, int32_t *epochs, int32_t *status, void *stream);

/* ---- Per-call plugin surface (one agent, n requests; n = 1 is the reference's call) ----
 * Allocator.estimate_CTR of agent `agent` for n contexts (dev), ctr dev [n][K]:
 *  - OracleAllocator (src/BidderAllocation.py:81-82): context [n][E+1], the TRUE context with
 *    its intercept; ctr = sigmoid(items @ context), FP64, the simulate kernels' arithmetic;
 *  - PyTorchLogisticRegressionAllocator (src/BidderAllocation.py:67-68, src/Models.py:28-33):
 *    context [n][OE+1], the OBSERVED context with its intercept; ctr = float32
 *    sigmoid(x32 . (m + noise)) widened to double; noise dev float32 [n][K][OE+1] is the
 *    Thompson draw torch.normal(0, 1/sqrt(q)) of each request (NULL: the MAP estimate,
 *    estimate_CTR(context, sample=False)). */
int ag_estimate_ctr(ag_ctx *ctx, int32_t agent, int64_t n, const double *context, const float *noise,
                    double *ctr, void *stream);

/* Bidder.bid of agent `agent` for n requests (dev [n] value and estimated CTR): bid [n], and
 * gamma / propensity [n] (may be NULL) as ag_batch_out defines them, by the agent's bidder
 * kind and state (src/Bidder.py:34-35, :47-58, :171-208, :348-367, :455-475). The draws the
 * reference makes inside bid() are inputs, as in ag_batch_in: gamma_raw [n] (the
 * rng.normal(prev_gamma, gamma_sigma) of a Gaussian-shading bid), policy_eps float32 [n] (the
 * rsample draw of a fitted policy), gamma_grid [128][n] (the 'search' grid); pass NULL for
 * what the agent's state does not draw. Synchronises for the agent's state. */
int ag_bid(ag_ctx *ctx, int32_t agent, int64_t n, const double *value, const double *est_ctr,
           const double *gamma_raw, const float *policy_eps, const double *gamma_grid, double *bid,
           double *gamma, double *propensity, void *stream);

/* Exact counters (host int64 [n][AG_FX_LIMBS], e.g. copied back or all-reduced)
 * -> doubles (host [n]), correctly rounded from the exact fixed-point sum. */
int ag_counters_to_double(const int64_t *counters_fx, int64_t n, double *out);

/* Known-answer hooks for the numerics the kernels restate (dev arrays of n):
 * src/Models.py:10-12 sigmoid with glibc-2.35-identical exp, and that exp alone. */
int ag_sigmoid(const double *z, double *out, int64_t n, void *stream);
int ag_exp(const double *x, double *out, int64_t n, void *stream);

/* Measurement hook (bench.py's measured HBM peak beside the 8 TB/s spec): copy nbytes
 * (multiple of 16, 16-B aligned dev pointers) with one 16-B non-temporal load and store per
 * lane, one 256-lane tile per workgroup, on the current device, stream-ordered. */
int ag_stream_copy(const void *src, void *dst, int64_t nbytes, void *stream);

/* Self-test of the learners' cross-workgroup exact sums (the combining-tree all-reduce every
 * trainer runs per epoch): `workgroups` cooperative workgroups on `device` (0: 4 per CU, every
 * XCD) run `generations` rounds of `regions` (1..4) interleaved 32-word int64 all-reduces and
 * compare every total with its closed form; *mismatches = the wrong totals seen (0 expected).
 * regions = 0: the grouped one-level form (csrc/ag_coop.h agent_allreduce_grouped).
 * Synchronous. Test hook, no reference counterpart. */
int ag_coop_selftest(int32_t device, int32_t workgroups, int32_t generations, int32_t regions,
                     int64_t *mismatches);

/* Self-test of the learners' split FP64 division (csrc/ag_div.h: the BCE rows share one
 * reciprocal of 1 + e between two divisions): about `pairs` random operand pairs in the split
 * form's range on `device` -- anywhere in it, and shaped as the win-rate row's and log1p's
 * divisions -- each divided both ways; *tested = the pairs in range, *mismatches = those whose
 * bits differ from the compiler's IEEE `a / b` (0 expected). Synchronous. Test hook, no
 * reference counterpart. */
int ag_div_selftest(int32_t device, int64_t pairs, uint64_t seed, int64_t *tested, int64_t *mismatches);

/* Thread-local description of the last error. */
const char *ag_last_error(void);
int32_t ag_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* AUCTIONGYM_H */
