"""ctypes binding of libauctiongym_hip.so (the C-ABI declared in include/auctiongym.h).

The library is the product path: there is no CPU fallback. If it is missing, or no GPU
is visible when a context is created, the calls raise -- they never route to the oracle.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libauctiongym_hip.so")
LIB_DEFAULT = LIB_PATH  # the product build: every entry point must be there

AG_OK, AG_ERR_INVALID, AG_ERR_UNSUPPORTED, AG_ERR_HIP, AG_ERR_STATE = 0, -1, -2, -3, -4
FIRST_PRICE, SECOND_PRICE = 0, 1
ALLOCATOR_ORACLE, ALLOCATOR_LRTS = 0, 1
BIDDER_TRUTHFUL, BIDDER_EMPIRICAL_SHADED, BIDDER_VALUE_LEARNING = 0, 1, 2
BIDDER_POLICY_LEARNING, BIDDER_DOUBLY_ROBUST = 3, 4
OPT_ITEM_SEARCH = 0
OPT_LAUNCH_AUCTIONS = 2
OPT_LRTS_BLOCK_SAMPLES = 3
OPT_LANE_AUCTIONS = 1
OPT_BIDDER_BLOCK_SAMPLES = 4
OPT_FIT_NOISE_SEED = 5
OPT_BIDDER_RECORD_CACHE = 6
OPT_SIMULATE_KERNEL = 7
OPT_SIM_BLOCKS_PER_CU = 8
OPT_SIM_BLOCK_THREADS = 9
OPT_SIM_GENERAL_MODE = 10
OPT_SIM_SHIPPED_SHAPE = 11
SIM_KERNEL_AUTO, SIM_KERNEL_GENERIC, SIM_KERNEL_FUSED, SIM_KERNEL_SPLIT, SIM_KERNEL_WIDE = 0, 1, 2, 3, 4
ITEM_SEARCH_AUTO, ITEM_SEARCH_EXACT = 0, 1

COUNTERS = ("net", "gross", "allocation_regret", "estimation_regret", "overbid_regret",
            "underbid_regret", "ctr_sqerr", "ctr_bias_sum", "best_ev_sum", "n_logs", "n_won",
            "paid")
NUM_COUNTERS = len(COUNTERS)
FX_FRAC_BITS, FX_LIMB_BITS, FX_LIMBS = 36, 42, 3

# Every symbol include/auctiongym.h declares (tests check the .so exports all of them).
EXPORTS = ("ag_create", "ag_destroy", "ag_set_agent_kinds", "ag_set_agent_params", "ag_set_agent_items",
           "ag_load_lrts",
           "ag_set_option", "ag_load_catalog", "ag_allocate", "ag_simulate", "ag_generate",
           "ag_generate_noise", "ag_lrts_collect", "ag_lrts_update", "ag_lrts_read",
           "ag_shading_collect", "ag_empirical_update", "ag_set_dr_state", "ag_get_dr_state",
           "ag_shading_counts", "ag_dr_update", "ag_set_bidder_modes", "ag_bidder_update",
           "ag_generate_search_grid", "ag_simulate_generated", "ag_stream_copy", "ag_estimate_ctr", "ag_bid",
           "ag_counters_to_double", "ag_sigmoid", "ag_exp", "ag_replay_draw", "ag_replay_draw_population",
           "ag_last_error",
           "ag_abi_version", "ag_ts_noise_index", "ag_generate_ts_noise_compact", "ag_torch_normal_epochs",
           "ag_bidder_rp_begin", "ag_bidder_rp_epoch", "ag_bidder_rp_run", "ag_bidder_rp_noise", "ag_bidder_rp_poll", "ag_bidder_rp_end",
           "ag_lrts_rp_begin", "ag_lrts_rp_epoch", "ag_lrts_rp_poll", "ag_lrts_rp_end", "ag_empirical_update_agents",
           "ag_coop_selftest", "ag_div_selftest")
ABI_VERSION = 17
LEARNER_UNINITIALISED, LEARNER_POLICY, LEARNER_SEARCH = 0, 1, 2
VL_SEARCH, VL_POLICY = 0, 1
PL_LOSSES = {"REINFORCE": 0, "REINFORCE_offpolicy": 1, "TRPO": 2, "PPO": 3}
LRTS_MAX_EPOCHS = 16384
LRTS_MAX_DO = 8


class AgShape(ctypes.Structure):
    _fields_ = [("num_agents", ctypes.c_int32), ("num_participants", ctypes.c_int32),
                ("num_items", ctypes.c_int32), ("embedding_size", ctypes.c_int32),
                ("obs_embedding_size", ctypes.c_int32), ("mechanism", ctypes.c_int32),
                ("num_slots", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("embedding_var", ctypes.c_double)]


class _Sized(ctypes.Structure):
    """ABI structs passed by pointer start with struct_size = sizeof(struct) (ABI 15): set
    here, so positional arguments start at the second field."""

    def __init__(self, *args, **kw):
        super().__init__(ctypes.sizeof(type(self)), *args, **kw)


class AgBatchIn(_Sized):
    _fields_ = [("struct_size", ctypes.c_uint64), ("ctx", ctypes.c_void_p), ("part", ctypes.c_void_p), ("u", ctypes.c_void_p),
                ("gamma_raw", ctypes.c_void_p), ("ts_noise", ctypes.c_void_p),
                ("policy_eps", ctypes.c_void_p), ("gamma_grid", ctypes.c_void_p),
                ("ts_noise_index", ctypes.c_void_p)]


class AgBatchOut(_Sized):
    _fields_ = [("struct_size", ctypes.c_uint64), ("winner", ctypes.c_void_p), ("price", ctypes.c_void_p),
                ("second_price", ctypes.c_void_p), ("outcome", ctypes.c_void_p),
                ("item", ctypes.c_void_p), ("bid", ctypes.c_void_p), ("est_ctr", ctypes.c_void_p),
                ("true_ctr", ctypes.c_void_p), ("best_ev", ctypes.c_void_p),
                ("gamma", ctypes.c_void_p), ("propensity", ctypes.c_void_p),
                ("winner_outcome", ctypes.c_void_p)]  # ABI 17


class AgLrtsSamples(_Sized):
    _fields_ = [("struct_size", ctypes.c_uint64), ("key", ctypes.c_void_p), ("x", ctypes.c_void_p), ("capacity", ctypes.c_int64),
                ("count", ctypes.c_void_p)]


class AgShadingSamples(_Sized):
    _fields_ = [("struct_size", ctypes.c_uint64), ("agent", ctypes.c_void_p), ("gamma", ctypes.c_void_p), ("utility", ctypes.c_void_p),
                ("capacity", ctypes.c_int64), ("count", ctypes.c_void_p), ("ctr", ctypes.c_void_p),
                ("value", ctypes.c_void_p), ("propensity", ctypes.c_void_p), ("won", ctypes.c_void_p),
                ("order", ctypes.c_void_p)]


class AgPcg64State(_Sized):
    _fields_ = [("struct_size", ctypes.c_uint64), ("state_hi", ctypes.c_uint64), ("state_lo", ctypes.c_uint64),
                ("inc_hi", ctypes.c_uint64), ("inc_lo", ctypes.c_uint64), ("has_uint32", ctypes.c_int32),
                ("uinteger", ctypes.c_uint32)]


class AgError(RuntimeError):
    pass


_libs = {}


def load(path=None):
    """Load the HIP library (raises if it was not built: run `make -C auction-gym_amd`).
    `path` selects another build of the same ABI (e.g. an A/B variant in tools/)."""
    path = path or LIB_PATH
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        raise AgError(f"{path} is missing: build it with `make -C auction-gym_amd` "
                      "(or __graft_entry__.build()); there is no CPU fallback")
    L = ctypes.CDLL(path)
    if L.ag_abi_version() != ABI_VERSION:
        raise AgError(f"{path}: ABI {L.ag_abi_version()} != {ABI_VERSION}; rebuild it")
    vp, i32, i64, u64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64
    sig = {
        "ag_create": (ctypes.c_int, [i32, ctypes.POINTER(AgShape), ctypes.POINTER(vp)]),
        "ag_destroy": (ctypes.c_int, [vp]),
        "ag_set_agent_kinds": (ctypes.c_int, [vp, vp, vp]),
        "ag_load_catalog": (ctypes.c_int, [vp, vp, vp]),
        "ag_set_option": (ctypes.c_int, [vp, i32, i64]),
        "ag_set_agent_params": (ctypes.c_int, [vp, vp, vp, vp, vp]),
        "ag_set_agent_items": (ctypes.c_int, [vp, vp]),
        "ag_load_lrts": (ctypes.c_int, [vp, vp, vp, vp, i32]),
        "ag_lrts_collect": (ctypes.c_int, [vp, i64, ctypes.POINTER(AgBatchIn),
                                           ctypes.POINTER(AgBatchOut), ctypes.POINTER(AgLrtsSamples), vp]),
        "ag_lrts_update": (ctypes.c_int, [vp, ctypes.POINTER(AgLrtsSamples), vp, vp, vp]),
        "ag_lrts_read": (ctypes.c_int, [vp, vp, vp, vp]),
        "ag_shading_collect": (ctypes.c_int, [vp, i64, i64, ctypes.POINTER(AgBatchIn),
                                              ctypes.POINTER(AgBatchOut), ctypes.POINTER(AgShadingSamples), vp]),
        "ag_empirical_update": (ctypes.c_int, [vp, ctypes.POINTER(AgShadingSamples), vp, vp]),
        "ag_empirical_update_agents": (ctypes.c_int, [vp, ctypes.POINTER(AgShadingSamples), vp, vp, vp]),
        "ag_set_dr_state": (ctypes.c_int, [vp, vp, vp]),
        "ag_get_dr_state": (ctypes.c_int, [vp, vp, vp]),
        "ag_shading_counts": (ctypes.c_int, [vp, ctypes.POINTER(AgShadingSamples), vp, vp]),
        "ag_dr_update": (ctypes.c_int, [vp, ctypes.POINTER(AgShadingSamples), vp, vp, i32, vp, vp, vp]),
        "ag_set_bidder_modes": (ctypes.c_int, [vp, vp]),
        "ag_bidder_update": (ctypes.c_int, [vp, ctypes.POINTER(AgShadingSamples), vp, vp, vp, i32, vp, vp, vp, vp]),
        "ag_generate_noise": (ctypes.c_int, [vp, u64, u64, i64, vp, vp, vp, vp, vp]),
        "ag_generate_search_grid": (ctypes.c_int, [vp, u64, u64, i64, vp, vp]),
        "ag_ts_noise_index": (ctypes.c_int, [vp, i64, vp, vp, ctypes.POINTER(i64), vp]),
        "ag_generate_ts_noise_compact": (ctypes.c_int, [vp, u64, u64, i64, vp, vp, vp, vp]),
        "ag_allocate": (ctypes.c_int, [vp, vp, i64, vp, vp, vp, vp]),
        "ag_simulate": (ctypes.c_int, [vp, i64, ctypes.POINTER(AgBatchIn),
                                       ctypes.POINTER(AgBatchOut), vp, vp]),
        "ag_generate": (ctypes.c_int, [vp, u64, u64, i64, vp, vp, vp, vp]),
        "ag_simulate_generated": (ctypes.c_int, [vp, u64, u64, i64, ctypes.POINTER(AgBatchOut), vp, vp]),
        "ag_counters_to_double": (ctypes.c_int, [vp, i64, vp]),
        "ag_sigmoid": (ctypes.c_int, [vp, vp, i64, vp]),
        "ag_exp": (ctypes.c_int, [vp, vp, i64, vp]),
        "ag_stream_copy": (ctypes.c_int, [vp, vp, i64, vp]),
        "ag_coop_selftest": (ctypes.c_int, [i32, i32, i32, i32, ctypes.POINTER(i64)]),
        "ag_div_selftest": (ctypes.c_int, [i32, i64, u64, ctypes.POINTER(i64), ctypes.POINTER(i64)]),
        "ag_estimate_ctr": (ctypes.c_int, [vp, i32, i64, vp, vp, vp, vp]),
        "ag_bid": (ctypes.c_int, [vp, i32, i64, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
        "ag_replay_draw": (ctypes.c_int, [ctypes.POINTER(AgPcg64State), i64, i32, i32, i32, ctypes.c_double, i32,
                                          vp, vp, vp, vp, vp, vp, vp]),
        "ag_replay_draw_population": (ctypes.c_int, [ctypes.POINTER(AgPcg64State), vp, i64, i64, i32, i32, i32,
                                                     ctypes.c_double, i32, vp, vp, vp, vp, vp, i32, vp, vp, vp,
                                                     vp, vp, vp, vp, vp, vp, vp]),
        "ag_torch_normal_epochs": (ctypes.c_int, [vp, i64, i64, i32, vp]),
        "ag_bidder_rp_begin": (ctypes.c_int, [vp, ctypes.POINTER(AgShadingSamples), vp, vp, vp, vp, vp]),
        "ag_bidder_rp_epoch": (ctypes.c_int, [vp, i32, ctypes.POINTER(i64), vp, vp]),
        "ag_bidder_rp_run": (ctypes.c_int, [vp, vp, vp]),
        "ag_bidder_rp_noise": (ctypes.c_int, [vp, vp, i64, i32, i32]),
        "ag_bidder_rp_poll": (ctypes.c_int, [vp, vp, vp, vp, vp]),
        "ag_bidder_rp_end": (ctypes.c_int, [vp, vp, vp, vp]),
        "ag_lrts_rp_begin": (ctypes.c_int, [vp, ctypes.POINTER(AgLrtsSamples), vp, vp, vp, vp]),
        "ag_lrts_rp_epoch": (ctypes.c_int, [vp, i32, ctypes.POINTER(i64), vp]),
        "ag_lrts_rp_poll": (ctypes.c_int, [vp, ctypes.POINTER(i32), vp]),
        "ag_lrts_rp_end": (ctypes.c_int, [vp, vp, vp]),
        "ag_last_error": (ctypes.c_char_p, []),
        "ag_abi_version": (i32, []),
    }
    for name, (res, args) in sig.items():
        if path != LIB_DEFAULT and not hasattr(L, name):
            continue  # an older A/B build (tools/ab_*.py) without an entry point added since
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _libs[path] = L
    return L


def check(rc, what="", lib=None):
    if rc != AG_OK:
        msg = (lib or load()).ag_last_error().decode(errors="replace")
        if rc == AG_ERR_INVALID:
            raise ValueError(msg)
        if rc == AG_ERR_UNSUPPORTED:
            raise NotImplementedError(msg)
        raise AgError(f"{what}: {msg} (status {rc})")
