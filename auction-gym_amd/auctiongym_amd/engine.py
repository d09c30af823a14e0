"""Device-resident batched engine: one ag_ctx per auction population, SoA buffers in HBM.

This is the MI355X-native core the reference-shaped classes (Auction, Agent, ...) sit on.
Torch is used only for device memory and the current HIP stream; all arithmetic runs in
the HIP kernels of libauctiongym_hip.so (auction-gym_amd/csrc/ag_kernels.hip).
"""
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import AgBatchIn, AgBatchOut, AgLrtsSamples, AgShadingSamples, AgShape
from ._lib import check as _check

COUNTERS = _lib.COUNTERS
NUM_COUNTERS = _lib.NUM_COUNTERS
FX_LIMBS = _lib.FX_LIMBS

_OUT_FIELDS = ("winner", "price", "second_price", "outcome", "item", "bid", "est_ctr",
               "true_ctr", "best_ev", "gamma", "propensity", "winner_outcome")
_CORE_FIELDS = _OUT_FIELDS[:9]
# ABI 17 (include/auctiongym.h): winner and outcome as one word. The headline's output set:
# every per-field array, winner and outcome as that word (the 1-B outcome stream alone cost
# 6 % of k_oracle's time, profiles/r05i_ab_packed.log)
HEADLINE_FIELDS = ("winner_outcome", "price", "item", "bid", "est_ctr", "true_ctr", "best_ev")


def unpack_outputs(outputs):
    """Per-field views of an output dict: winner and outcome from a winner_outcome word."""
    o = dict(outputs)
    if "winner_outcome" in o:
        wo = o["winner_outcome"].to(torch.int64) & 0xffffffff
        o["winner"] = (wo & 0x7fffffff).to(torch.int32)
        o["outcome"] = (wo >> 31).to(torch.uint8)
    return o


def _batch_out(outputs):
    return AgBatchOut(*[_ptr(outputs.get(f)).value for f in _OUT_FIELDS])


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _batch_in(inputs):
    return AgBatchIn(*[_ptr(inputs.get(k)).value for k in ("ctx", "part", "u", "gamma_raw", "ts_noise",
                                                           "policy_eps", "gamma_grid", "ts_noise_index")])


def require_gpu():
    if not torch.cuda.is_available():
        raise RuntimeError("auctiongym_amd needs a ROCm GPU (MI355X); none is visible. "
                           "There is no CPU fallback.")


class AuctionEngine:
    """Batched Auction.simulate_opportunity for N agents, P participants, K items, E dims."""

    def __init__(self, num_agents, num_participants, num_items, embedding_size,
                 obs_embedding_size, mechanism, embedding_var=1.0, device=None, lib_path=None):
        require_gpu()
        self.L = _lib.load(lib_path)
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        self.N, self.P, self.K = int(num_agents), int(num_participants), int(num_items)
        self.E, self.OE = int(embedding_size), int(obs_embedding_size)
        self.D = self.E + 1
        self.mechanism = int(mechanism)
        self.embedding_var = float(embedding_var)
        shape = AgShape(self.N, self.P, self.K, self.E, self.OE, self.mechanism, 1, 0,
                        self.embedding_var)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            self._check(self.L.ag_create(self.device.index, ctypes.byref(shape), ctypes.byref(h)),
                  "ag_create")
        self._h = h

    def _check(self, rc, what):
        _check(rc, what, self.L)

    def close(self):
        if getattr(self, "_h", None):
            self.L.ag_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------------- setup
    def set_agent_kinds(self, allocator_kinds, bidder_kinds):
        a = np.ascontiguousarray(allocator_kinds, np.int32)
        b = np.ascontiguousarray(bidder_kinds, np.int32)
        assert a.shape == (self.N,) and b.shape == (self.N,)
        self._check(self.L.ag_set_agent_kinds(self._h, a.ctypes.data, b.ctypes.data), "ag_set_agent_kinds")

    def set_agent_items(self, num_items):
        """Each agent's own item count (ag_set_agent_items; None: all K)."""
        n = None if num_items is None else np.ascontiguousarray(num_items, np.int32)
        self._check(self.L.ag_set_agent_items(self._h, None if n is None else n.ctypes.data), "ag_set_agent_items")

    def set_agent_params(self, allocator_kinds, bidder_kinds, prev_gamma=None, gamma_sigma=None):
        """Plugin kinds + shading parameters (ag_set_agent_params)."""
        a = np.ascontiguousarray(allocator_kinds, np.int32)
        b = np.ascontiguousarray(bidder_kinds, np.int32)
        pg = None if prev_gamma is None else np.ascontiguousarray(prev_gamma, np.float64)
        gs = None if gamma_sigma is None else np.ascontiguousarray(gamma_sigma, np.float64)
        self.shading = bool((b != _lib.BIDDER_TRUTHFUL).any())
        self._bkind = b.copy()
        self.dr = bool(np.isin(b, (_lib.BIDDER_VALUE_LEARNING, _lib.BIDDER_POLICY_LEARNING,
                                   _lib.BIDDER_DOUBLY_ROBUST)).any())  # learning bidders
        self.lrts = bool((a == _lib.ALLOCATOR_LRTS).any())
        self._check(self.L.ag_set_agent_params(self._h, a.ctypes.data, b.ctypes.data,
                                               None if pg is None else pg.ctypes.data,
                                               None if gs is None else gs.ctypes.data),
                    "ag_set_agent_params")

    def load_lrts(self, m, q, prev_m=None, thompson_sampling=True):
        """LR-TS posteriors m, q, prev_m float32 [N][K][OE+1] (ag_load_lrts; prev_m None = m)."""
        shape = (self.N, self.K, self.OE + 1)
        m = np.ascontiguousarray(m, np.float32)
        q = np.ascontiguousarray(q, np.float32)
        pm = None if prev_m is None else np.ascontiguousarray(prev_m, np.float32)
        if m.shape != shape or q.shape != shape or (pm is not None and pm.shape != shape):
            raise ValueError(f"LR-TS params must be [N][K][OE+1] = {shape}")
        self.ts_sample = bool(thompson_sampling)
        self._check(self.L.ag_load_lrts(self._h, m.ctypes.data, q.ctypes.data,
                                        None if pm is None else pm.ctypes.data, int(self.ts_sample)),
                    "ag_load_lrts")

    def lrts_state(self):
        """(m, q, prev_m) float32 [N][K][OE+1] as they are on the device (ag_lrts_read)."""
        shape = (self.N, self.K, self.OE + 1)
        m, q, pm = (np.empty(shape, np.float32) for _ in range(3))
        self._check(self.L.ag_lrts_read(self._h, m.ctypes.data, q.ctypes.data, pm.ctypes.data),
                    "ag_lrts_read")
        return m, q, pm

    # ---------------------------------------------------------------- LR-TS update
    def new_lrts_samples(self, capacity):
        """Device store of won LR-TS samples (ag_lrts_samples): key [cap] uint32 (as int32),
        x [OE+1][cap] float32, count [1]."""
        d = self.device
        return {"key": torch.empty((capacity,), dtype=torch.int32, device=d),
                "x": torch.empty((self.OE + 1, capacity), dtype=torch.float32, device=d),
                "count": torch.zeros((1,), dtype=torch.int64, device=d)}

    @staticmethod
    def _samples(st):
        return AgLrtsSamples(_ptr(st["key"]).value, _ptr(st["x"]).value, st["key"].shape[0],
                             _ptr(st["count"]).value)

    def lrts_collect(self, inputs, outputs, store):
        """Append the won LR-TS samples of a simulated batch (ag_lrts_collect)."""
        B = inputs["u"].shape[0]
        bi = _batch_in(inputs)
        bo = _batch_out(outputs)
        st = self._samples(store)
        self._check(self.L.ag_lrts_collect(self._h, B, ctypes.byref(bi), ctypes.byref(bo),
                                           ctypes.byref(st), _stream()), "ag_lrts_collect")

    def lrts_update(self, store, trace=False):
        """Train every LR-TS agent on the store (ag_lrts_update). Returns epochs [N] and, with
        trace=True, the per-epoch losses as a float32 [N][16384] device tensor."""
        ep = np.zeros(self.N, np.int32)
        tr = None
        if trace:
            tr = torch.zeros((self.N, _lib.LRTS_MAX_EPOCHS), dtype=torch.float32, device=self.device)
        st = self._samples(store)
        self._check(self.L.ag_lrts_update(self._h, ctypes.byref(st), ep.ctypes.data, _ptr(tr),
                                          _stream()), "ag_lrts_update")
        return (ep, tr) if trace else ep

    def lrts_rp_begin(self, store, agents=None, samples_total=None):
        """Start a resumable LR-TS update (ag_lrts_rp_begin); returns the totals tensor (int64
        [2][N][144], device) whose slot launch_index & 1 a multi-rank caller all-reduces."""
        mask = None if agents is None else np.ascontiguousarray(agents, np.int32).reshape(self.N)
        tot = np.ascontiguousarray(samples_total, np.int64) if samples_total is not None else None
        self._lrp_tot = torch.zeros((2, self.N, 144), dtype=torch.int64, device=self.device)
        self._lrp_store = self._samples(store)
        self._check(self.L.ag_lrts_rp_begin(self._h, ctypes.byref(self._lrp_store),
                                            None if mask is None else mask.ctypes.data,
                                            None if tot is None else tot.ctypes.data, _ptr(self._lrp_tot),
                                            _stream()), "ag_lrts_rp_begin")
        return self._lrp_tot

    def lrts_rp_epoch(self, launches=1):
        k = ctypes.c_int64(-1)
        self._check(self.L.ag_lrts_rp_epoch(self._h, int(launches), ctypes.byref(k), _stream()), "ag_lrts_rp_epoch")
        return k.value

    def lrts_rp_poll(self):
        """Agents still training (0: done)."""
        n = ctypes.c_int32(0)
        self._check(self.L.ag_lrts_rp_poll(self._h, ctypes.byref(n), _stream()), "ag_lrts_rp_poll")
        return n.value

    def lrts_rp_end(self):
        """Epochs [N] of the trained agents (m, q, prev_m are on the device)."""
        ep = np.zeros(self.N, np.int32)
        try:
            self._check(self.L.ag_lrts_rp_end(self._h, ep.ctypes.data, _stream()), "ag_lrts_rp_end")
        finally:
            self._lrp_store = None
        return ep

    def set_item_search(self, exact):
        """exact=True: score every item in FP64 (the reference loop); False (default): f32
        screen + exact re-score of the near-best items -- identical results."""
        mode = _lib.ITEM_SEARCH_EXACT if exact else _lib.ITEM_SEARCH_AUTO
        self._check(self.L.ag_set_option(self._h, _lib.OPT_ITEM_SEARCH, mode), "ag_set_option")

    def set_simulate_kernel(self, generic):
        """generic=True: always the general simulate kernel (k_simulate); False (default):
        k_oracle for OracleAllocator + TruthfulBidder populations, k_simulate for the others;
        "wide": the runtime-P kernel at any P (A/B variant builds only). Identical results."""
        mode = {"wide": _lib.SIM_KERNEL_WIDE}.get(generic) or (
            _lib.SIM_KERNEL_GENERIC if generic else _lib.SIM_KERNEL_AUTO)
        self._check(self.L.ag_set_option(self._h, _lib.OPT_SIMULATE_KERNEL, mode), "ag_set_option")

    def set_blocks_per_cu(self, n):
        """Resident workgroups per CU of the Oracle kernel's persistent grid (0: as many as
        fit); same results."""
        self._check(self.L.ag_set_option(self._h, _lib.OPT_SIM_BLOCKS_PER_CU, int(n)), "ag_set_option")

    def set_lane_auctions(self, n):
        """Auctions per lane in the screened kernel: 1 (default) or 2 (16-B SoA accesses when
        B is even; lower occupancy, slower under sustained load). Same results either way."""
        self._check(self.L.ag_set_option(self._h, _lib.OPT_LANE_AUCTIONS, int(n)), "ag_set_option")

    def set_launch_auctions(self, n):
        """Cap on auctions per k_simulate launch (0: the resident grid's exact-counter
        capacity); larger batches run as consecutive launches, same results."""
        self._check(self.L.ag_set_option(self._h, _lib.OPT_LAUNCH_AUCTIONS, int(n)), "ag_set_option")

    def set_bidder_block_samples(self, n):
        """Records per workgroup of the learning bidders' trainer (0: the default split)."""
        self._check(self.L.ag_set_option(self._h, _lib.OPT_BIDDER_BLOCK_SAMPLES, int(n)), "ag_set_option")

    def set_bidder_record_cache(self, n):
        """Most records per workgroup the learning bidders' trainer keeps in LDS (-1: as many
        as fit, 0: none); results are identical."""
        self._check(self.L.ag_set_option(self._h, _lib.OPT_BIDDER_RECORD_CACHE, int(n)), "ag_set_option")

    def set_fit_noise_seed(self, seed):
        """Seed of the synthetic rsample noise of bidder_update(noise=None)."""
        self._check(self.L.ag_set_option(self._h, _lib.OPT_FIT_NOISE_SEED, int(seed)), "ag_set_option")

    def set_lrts_block_samples(self, n):
        """Samples per workgroup of the LR-TS training kernel (0: 4096); same results."""
        self._check(self.L.ag_set_option(self._h, _lib.OPT_LRTS_BLOCK_SAMPLES, int(n)), "ag_set_option")

    def load_catalog(self, items, values):
        items = np.ascontiguousarray(items, np.float64)
        values = np.ascontiguousarray(values, np.float64)
        if items.shape != (self.N, self.K, self.D) or values.shape != (self.N, self.K):
            raise ValueError(f"catalogue shapes {items.shape}/{values.shape} != "
                             f"({self.N},{self.K},{self.D})/({self.N},{self.K})")
        self._check(self.L.ag_load_catalog(self._h, items.ctypes.data, values.ctypes.data),
              "ag_load_catalog")

    # ---------------------------------------------------------------- buffers
    def alloc_inputs(self, B):
        d = self.device
        inp = {"ctx": torch.empty((self.E, B), dtype=torch.float64, device=d),
               "part": torch.empty((self.P, B), dtype=torch.int32, device=d),
               "u": torch.empty((B,), dtype=torch.float64, device=d)}
        if getattr(self, "shading", False):
            inp["gamma_raw"] = torch.empty((self.P, B), dtype=torch.float64, device=d)
        if getattr(self, "dr", False):
            inp["policy_eps"] = torch.empty((self.P, B), dtype=torch.float32, device=d)
        if getattr(self, "vl_search", False):
            inp["gamma_grid"] = torch.empty((self.P, 128, B), dtype=torch.float64, device=d)
        if getattr(self, "lrts", False) and getattr(self, "ts_sample", True):
            inp["ts_noise"] = torch.empty((self.P, (B + 63) // 64, self.K * (self.OE + 1), 64),
                                          dtype=torch.float32, device=d)
        return inp

    @staticmethod
    def tile_ts_noise(noise):
        """Thompson noise per (auction, slot) [B][P][K*Do] (or [B][P][K][Do]) -> the kernel's
        64-auction tiles [P][T][K*Do][64] (include/auctiongym.h ag_batch_in.ts_noise)."""
        z = np.asarray(noise, np.float32)
        B, P = z.shape[:2]
        z = z.reshape(B, P, -1)
        T = (B + 63) // 64
        pad = np.zeros((T * 64, P, z.shape[2]), np.float32)
        pad[:B] = z
        return np.ascontiguousarray(pad.reshape(T, 64, P, -1).transpose(2, 0, 3, 1))

    @staticmethod
    def untile_ts_noise(tiles, B):
        """Inverse of tile_ts_noise: [P][T][K*Do][64] -> [B][P][K*Do]."""
        t = tiles.detach().cpu().numpy() if torch.is_tensor(tiles) else np.asarray(tiles)
        P, T, KDo, _ = t.shape
        return np.ascontiguousarray(t.transpose(1, 3, 0, 2).reshape(T * 64, P, KDo)[:B])

    def alloc_outputs(self, B, fields=None, packed=False):
        """Device output arrays (ag_batch_out) of B auctions; packed: the ABI 17 word
        winner_outcome (winner | outcome << 31) instead of the winner and outcome arrays."""
        if fields is None:
            fields = _OUT_FIELDS[:11] if getattr(self, "shading", False) else _CORE_FIELDS
        if packed:
            fields = [f for f in fields if f not in ("winner", "outcome")] + ["winner_outcome"]
        d, P = self.device, self.P
        spec = {"winner": ((B,), torch.int32), "price": ((B,), torch.float64),
                "second_price": ((B,), torch.float64), "outcome": ((B,), torch.uint8),
                "item": ((P, B), torch.int32), "bid": ((P, B), torch.float64),
                "est_ctr": ((P, B), torch.float64), "true_ctr": ((P, B), torch.float64),
                "best_ev": ((P, B), torch.float64), "gamma": ((P, B), torch.float64),
                "propensity": ((P, B), torch.float64),
                "winner_outcome": ((B,), torch.int32)}
        return {k: torch.empty(spec[k][0], dtype=spec[k][1], device=d) for k in fields}

    def new_counters(self):
        return torch.zeros((self.N, NUM_COUNTERS, FX_LIMBS), dtype=torch.int64, device=self.device)

    # ---------------------------------------------------------------- hot calls
    def simulate(self, inputs, outputs, counters=None):
        B = inputs["u"].shape[0]
        for k, t in inputs.items():
            if not t.is_contiguous() or t.device != self.device:
                raise ValueError(f"input {k} must be a contiguous tensor on {self.device}")
        if inputs["ctx"].shape != (self.E, B) or inputs["part"].shape != (self.P, B):
            raise ValueError("inputs must be SoA: ctx [E][B], part [P][B], u [B]")
        bi = _batch_in(inputs)
        bo = _batch_out(outputs)
        self._check(self.L.ag_simulate(self._h, B, ctypes.byref(bi), ctypes.byref(bo),
                                 _ptr(counters), _stream()), "ag_simulate")

    def simulate_generated(self, seed, first_auction, outputs, counters=None):
        """Generate mode (ag_simulate_generated): B = outputs["winner"].shape[0] rounds whose
        inputs are drawn inside the kernel -- the same bits generate(seed, first_auction)
        writes -- so only the outputs touch HBM."""
        B = (outputs["winner"] if "winner" in outputs else outputs["winner_outcome"]).shape[0]
        bo = _batch_out(outputs)
        self._check(self.L.ag_simulate_generated(self._h, int(seed), int(first_auction), B, ctypes.byref(bo),
                                                 _ptr(counters), _stream()), "ag_simulate_generated")

    def generate(self, seed, first_auction, inputs):
        B = inputs["u"].shape[0]
        self._check(self.L.ag_generate(self._h, int(seed), int(first_auction), B, _ptr(inputs["ctx"]),
                                 _ptr(inputs["part"]), _ptr(inputs["u"]), _stream()), "ag_generate")

    def generate_search_grid(self, seed, first_auction, inputs):
        """Synthetic ValueLearningBidder search grids into inputs["gamma_grid"] (ag_generate_search_grid)."""
        B = inputs["u"].shape[0]
        self._check(self.L.ag_generate_search_grid(self._h, int(seed), int(first_auction), B,
                                                   _ptr(inputs["gamma_grid"]), _stream()), "ag_generate_search_grid")

    def generate_noise(self, seed, first_auction, inputs, compact=False):
        """Synthetic gamma_raw / ts_noise for the participants already in inputs["part"].
        compact=True: the Thompson noise in the compact layout (ag_ts_noise_index) -- the same
        values, stored for the LR-TS pairs only; inputs["ts_noise"] is reallocated to fit and
        inputs["ts_noise_index"] set."""
        B = inputs["u"].shape[0]
        if compact and "ts_noise" in inputs:
            self.compact_ts_noise(seed, first_auction, inputs)
            self._check(self.L.ag_generate_noise(self._h, int(seed), int(first_auction), B,
                                                 _ptr(inputs["part"]), _ptr(inputs.get("gamma_raw")),
                                                 None, _ptr(inputs.get("policy_eps")), _stream()),
                        "ag_generate_noise")
            return
        self._check(self.L.ag_generate_noise(self._h, int(seed), int(first_auction), B,
                                             _ptr(inputs["part"]), _ptr(inputs.get("gamma_raw")),
                                             _ptr(inputs.get("ts_noise")), _ptr(inputs.get("policy_eps")),
                                             _stream()),
                    "ag_generate_noise")

    def ts_noise_index(self, part):
        """(index int32 [P][B] dev, pairs): the compact Thompson-noise layout of `part`
        (ag_ts_noise_index)."""
        B = part.shape[1]
        idx = torch.empty((self.P, B), dtype=torch.int32, device=self.device)
        n = ctypes.c_int64()
        self._check(self.L.ag_ts_noise_index(self._h, B, _ptr(part), _ptr(idx), ctypes.byref(n), _stream()),
                    "ag_ts_noise_index")
        return idx, int(n.value)

    def compact_ts_noise(self, seed, first_auction, inputs):
        """Replace inputs["ts_noise"] by the compact layout of the same synthetic draws."""
        B = inputs["u"].shape[0]
        idx, n = self.ts_noise_index(inputs["part"])
        inputs.pop("ts_noise", None)
        inputs["ts_noise_index"] = idx
        inputs["ts_noise"] = torch.empty((max(1, (n + 63) // 64), self.K * (self.OE + 1), 64),
                                         dtype=torch.float32, device=self.device)
        self._check(self.L.ag_generate_ts_noise_compact(self._h, int(seed), int(first_auction), B,
                                                        _ptr(inputs["part"]), _ptr(idx), _ptr(inputs["ts_noise"]),
                                                        _stream()), "ag_generate_ts_noise_compact")
        return n

    @staticmethod
    def compact_to_dense_ts_noise(compact, index, P, B):
        """The dense tiles [P][T][K*Do][64] of a compact layout (zeros for non-LR-TS pairs)."""
        c = compact.detach().cpu().numpy() if torch.is_tensor(compact) else np.asarray(compact)
        ix = index.detach().cpu().numpy() if torch.is_tensor(index) else np.asarray(index)
        KDo = c.shape[1]
        flat = c.transpose(0, 2, 1).reshape(-1, KDo)  # pair j -> its K*Do coefficients
        T = (B + 63) // 64
        dense = np.zeros((P, T * 64, KDo), np.float32)
        m = ix >= 0
        dense[:, :B][m] = flat[ix[m]]
        return np.ascontiguousarray(dense.reshape(P, T, 64, KDo).transpose(0, 1, 3, 2))

    # ---------------------------------------------------------------- per-call plugin surface
    def _dev(self, a, dtype):
        if a is None:
            return None
        t = a if torch.is_tensor(a) else torch.from_numpy(np.ascontiguousarray(a))
        return t.to(device=self.device, dtype=dtype).contiguous()

    def estimate_ctr(self, agent, contexts, noise=None):
        """Allocator.estimate_CTR of `agent` for n contexts [n][E+1] (OracleAllocator: true
        context with intercept) or [n][OE+1] (LR-TS: observed context with intercept); noise
        [n][K][OE+1] float32 Thompson draws or None (MAP). Returns float64 [n][K] (device)."""
        x = self._dev(contexts, torch.float64)
        n = x.shape[0]
        nz = self._dev(noise, torch.float32)
        out = torch.empty((n, self.K), dtype=torch.float64, device=self.device)
        self._check(self.L.ag_estimate_ctr(self._h, int(agent), n, _ptr(x), _ptr(nz), _ptr(out), _stream()),
                    "ag_estimate_ctr")
        return out

    def bid(self, agent, values, ctrs, gamma_raw=None, policy_eps=None, gamma_grid=None):
        """Bidder.bid of `agent` for n requests (ag_bid): values, estimated CTRs [n]; the
        draws its state makes: gamma_raw [n], policy_eps [n], gamma_grid [n][128]. Returns
        (bid, gamma, propensity) float64 [n] device tensors."""
        v = self._dev(values, torch.float64).reshape(-1)
        c = self._dev(ctrs, torch.float64).reshape(-1)
        n = v.numel()
        g = self._dev(gamma_raw, torch.float64)
        e = self._dev(policy_eps, torch.float32)
        gr = None if gamma_grid is None else self._dev(gamma_grid, torch.float64).reshape(n, 128).t().contiguous()
        b, gm, pr = (torch.empty(n, dtype=torch.float64, device=self.device) for _ in range(3))
        self._check(self.L.ag_bid(self._h, int(agent), n, _ptr(v), _ptr(c), _ptr(g), _ptr(e), _ptr(gr), _ptr(b),
                                  _ptr(gm), _ptr(pr), _stream()), "ag_bid")
        return b, gm, pr

    def allocate(self, bids):
        """Batched allocate: bids [P][B] (device, float64) -> winner, price, second_price."""
        if bids.dim() != 2 or bids.shape[0] != self.P or bids.dtype != torch.float64:
            raise ValueError("bids must be a float64 [P][B] tensor")
        bids = bids.contiguous()
        B = bids.shape[1]
        w = torch.empty(B, dtype=torch.int32, device=self.device)
        p = torch.empty(B, dtype=torch.float64, device=self.device)
        s = torch.empty(B, dtype=torch.float64, device=self.device)
        self._check(self.L.ag_allocate(self._h, _ptr(bids), B, _ptr(w), _ptr(p), _ptr(s), _stream()),
              "ag_allocate")
        return w, p, s

    # ---------------------------------------------------------------- shading update
    def new_shading_samples(self, capacity, learning=False):
        """Device store of shading-bidder records (ag_shading_samples); learning=True adds
        the fields the DoublyRobustBidder update needs (ctr, value, propensity, won)."""
        d = self.device
        st = {"agent": torch.empty((capacity,), dtype=torch.int32, device=d),
              "gamma": torch.empty((capacity,), dtype=torch.float64, device=d),
              "utility": torch.empty((capacity,), dtype=torch.float64, device=d),
              "count": torch.zeros((1,), dtype=torch.int64, device=d)}
        if learning:
            for k in ("ctr", "value", "propensity"):
                st[k] = torch.empty((capacity,), dtype=torch.float64, device=d)
            st["won"] = torch.empty((capacity,), dtype=torch.uint8, device=d)
            st["order"] = torch.empty((capacity,), dtype=torch.int64, device=d)  # uint64 bits
        return st

    @staticmethod
    def _shading(st):
        return AgShadingSamples(_ptr(st["agent"]).value, _ptr(st["gamma"]).value,
                                _ptr(st["utility"]).value, st["agent"].shape[0], _ptr(st["count"]).value,
                                _ptr(st.get("ctr")).value, _ptr(st.get("value")).value,
                                _ptr(st.get("propensity")).value, _ptr(st.get("won")).value,
                                _ptr(st.get("order")).value)

    def shading_counts(self, store):
        """Records per agent in a shading store (ag_shading_counts)."""
        c = np.zeros(self.N, np.int64)
        self._check(self.L.ag_shading_counts(self._h, ctypes.byref(self._shading(store)), c.ctypes.data,
                                             _stream()), "ag_shading_counts")
        return c

    def set_dr_state(self, state, initialised):
        """Learning bidders' models, float32 [N][16] (win-rate w0 w1 w2 b, policy 12), and what
        each bids from (LEARNER_*)."""
        st = np.ascontiguousarray(state, np.float32).reshape(self.N, 16)
        ini = np.ascontiguousarray(initialised, np.int32).reshape(self.N)
        self._check(self.L.ag_set_dr_state(self._h, st.ctypes.data, ini.ctypes.data), "ag_set_dr_state")

    def dr_state(self):
        st = np.zeros((self.N, 16), np.float32)
        ini = np.zeros(self.N, np.int32)
        self._check(self.L.ag_get_dr_state(self._h, st.ctypes.data, ini.ctypes.data), "ag_get_dr_state")
        return st, ini

    def dr_update(self, store, noise, noise_offsets, noise_epochs, trace=False):
        """DoublyRobustBidder.update of every DR agent (ag_dr_update). noise: float32 device
        tensor holding agent a's per-epoch rsample draws at noise_offsets[a] (rows of its
        record count). Returns epochs [N][3] (and traces [N][3][32768] with trace=True)."""
        ep = np.zeros((self.N, 3), np.int32)
        off = np.ascontiguousarray(noise_offsets, np.int64)
        tr = torch.zeros((self.N, 3, 32768), dtype=torch.float32, device=self.device) if trace else None
        self._check(self.L.ag_dr_update(self._h, ctypes.byref(self._shading(store)), _ptr(noise),
                                        off.ctypes.data, int(noise_epochs), ep.ctypes.data, _ptr(tr),
                                        _stream()), "ag_dr_update")
        return (ep, tr) if trace else ep

    def set_bidder_modes(self, modes):
        """ValueLearningBidder inference (VL_SEARCH / VL_POLICY) / PolicyLearningBidder loss
        (PL_LOSSES) per agent, int32 [N] (ag_set_bidder_modes)."""
        m = np.ascontiguousarray(modes, np.int32).reshape(self.N)
        self._check(self.L.ag_set_bidder_modes(self._h, m.ctypes.data), "ag_set_bidder_modes")
        self.vl_search = bool(((self._bkind == _lib.BIDDER_VALUE_LEARNING) & (m == _lib.VL_SEARCH)).any())

    def bidder_update(self, store, noise=None, noise_offsets=None, noise_epochs=0, trace=False, agents=None):
        """Bidder.update of the learning bidders (ag_bidder_update; agents: [N] mask, None =
        all). noise: float32 device tensor with agent a's per-epoch rsample draws at
        noise_offsets[a] (rows of its record count), for DoublyRobust / ValueLearning 'policy'
        agents. Returns (epochs [N][3], status [N]) and, with trace=True, the traces
        [N][3][32768]. status -3: the agent needs more noise epochs (left unchanged)."""
        mask = None if agents is None else np.ascontiguousarray(agents, np.int32).reshape(self.N)
        ep = np.zeros((self.N, 3), np.int32)
        stat = np.zeros(self.N, np.int32)
        off = np.ascontiguousarray(noise_offsets if noise_offsets is not None else np.zeros(self.N), np.int64)
        tr = torch.zeros((self.N, 3, 32768), dtype=torch.float32, device=self.device) if trace else None
        self._check(self.L.ag_bidder_update(self._h, ctypes.byref(self._shading(store)),
                                            None if mask is None else mask.ctypes.data, _ptr(noise),
                                            off.ctypes.data, int(noise_epochs), ep.ctypes.data, stat.ctypes.data,
                                            _ptr(tr), _stream()), "ag_bidder_update")
        return (ep, stat, tr) if trace else (ep, stat)

    # ---- resumable / record-parallel learning-bidder training (ag_bidder_rp_*) ----
    def bidder_rp_begin(self, store, agents=None, records_total=None, records_base=None):
        """Start a resumable update of the exact-sum learning bidders (ag_bidder_rp_begin):
        agents [N] mask (None: every ValueLearning / DoublyRobust bidder); records_total /
        records_base [N]: the agents' records over all ranks and the global index of this
        rank's first one (None: this process holds them all). Returns the totals tensor
        (int64 [2][N][32] on the device) whose slot launch_index & 1 a multi-rank caller
        all-reduces (SUM) after every epoch launch."""
        mask = None if agents is None else np.ascontiguousarray(agents, np.int32).reshape(self.N)
        tot = np.ascontiguousarray(records_total, np.int64) if records_total is not None else None
        base = np.ascontiguousarray(records_base, np.int64) if records_base is not None else None
        self._rp_tot = torch.zeros((2, self.N, 32), dtype=torch.int64, device=self.device)
        self._rp_store = self._shading(store)
        self._check(self.L.ag_bidder_rp_begin(self._h, ctypes.byref(self._rp_store),
                                              None if mask is None else mask.ctypes.data,
                                              None if tot is None else tot.ctypes.data,
                                              None if base is None else base.ctypes.data,
                                              _ptr(self._rp_tot), _stream()), "ag_bidder_rp_begin")
        self._rp_noise = None
        return self._rp_tot

    def bidder_rp_epoch(self, launches=1, traces=None):
        """Queue `launches` epoch launches; returns the last launch's index (its totals:
        totals[index & 1])."""
        k = ctypes.c_int64(-1)
        self._check(self.L.ag_bidder_rp_epoch(self._h, int(launches), ctypes.byref(k), _ptr(traces), _stream()),
                    "ag_bidder_rp_epoch")
        return k.value

    def bidder_rp_run(self, traces=None):
        """One process holding every record: run the learners in persistent launches until each
        is done or waits for noise (ag_bidder_rp_run; the same state bidder_rp_epoch steps)."""
        self._check(self.L.ag_bidder_rp_run(self._h, _ptr(traces), _stream()), "ag_bidder_rp_run")

    def bidder_rp_noise(self, noise, noise_n, first_epoch, epochs):
        """The host-drawn rsample window (device float32 [epochs][noise_n]) of the policy fits."""
        self._rp_noise = noise  # kept alive while the launches read it
        self._check(self.L.ag_bidder_rp_noise(self._h, _ptr(noise), int(noise_n), int(first_epoch), int(epochs)),
                    "ag_bidder_rp_noise")

    def bidder_rp_poll(self):
        """(fit [N] (-1 done), epoch [N], need_noise [N] (-1 or the policy epoch waiting))."""
        fit, ep, nn = (np.zeros(self.N, np.int32) for _ in range(3))
        self._check(self.L.ag_bidder_rp_poll(self._h, fit.ctypes.data, ep.ctypes.data, nn.ctypes.data, _stream()),
                    "ag_bidder_rp_poll")
        return fit, ep, nn

    def bidder_rp_end(self):
        """Apply the trained states; returns (epochs [N][3], status [N])."""
        ep = np.zeros((self.N, 3), np.int32)
        stat = np.zeros(self.N, np.int32)
        try:
            self._check(self.L.ag_bidder_rp_end(self._h, ep.ctypes.data, stat.ctypes.data, _stream()),
                        "ag_bidder_rp_end")
        finally:
            self._rp_noise = self._rp_store = None
        return ep, stat

    def shading_collect(self, inputs, outputs, store, first_auction=0):
        """Append the shading-bidder records of a simulated batch of auctions
        [first_auction, first_auction + B) (ag_shading_collect)."""
        B = inputs["u"].shape[0]
        bi = _batch_in(inputs)
        bo = _batch_out(outputs)
        st = self._shading(store)
        self._check(self.L.ag_shading_collect(self._h, int(first_auction), B, ctypes.byref(bi), ctypes.byref(bo),
                                              ctypes.byref(st), _stream()), "ag_shading_collect")

    def empirical_update(self, store, agents=None):
        """EmpiricalShadedBidder.update of every such agent, or of the agents of the [N] mask
        `agents` (ag_empirical_update_agents); returns the prev_gamma of all agents [N] after it."""
        pg = np.zeros(self.N, np.float64)
        st = self._shading(store)
        mask = None if agents is None else np.ascontiguousarray(agents, np.int32).reshape(self.N)
        self._check(self.L.ag_empirical_update_agents(self._h, ctypes.byref(st),
                                                      None if mask is None else mask.ctypes.data, pg.ctypes.data,
                                                      _stream()), "ag_empirical_update")
        return pg

    # ---------------------------------------------------------------- counters
    @staticmethod
    def counters_to_numpy(counters):
        """Exact fixed-point limbs [N][C][3] (tensor or array) -> float64 [N][C]."""
        fx = counters.detach().cpu().numpy() if torch.is_tensor(counters) else np.asarray(counters)
        fx = np.ascontiguousarray(fx, np.int64)
        n = fx.size // FX_LIMBS
        out = np.empty(n, np.float64)
        _check(_lib.load().ag_counters_to_double(fx.ctypes.data, n, out.ctypes.data),
               "ag_counters_to_double")
        return out.reshape(fx.shape[:-1])


# torch CPU builds whose float normal_ of >= 16 elements runs normal_fill_16_AVX2 (the kernel
# ag_replay.cpp restates: compiled under __AVX2__, which the AVX512 build defines too); the
# DEFAULT build takes the scalar normal_fill with libm logf / cosf over the whole tensor
TORCH_NORMAL_AVX2 = ("AVX2", "AVX512")


def torch_normal_epochs(state, n, epochs):
    """`epochs` x torch.empty(n).normal_() from the torch CPU generator state blob `state`
    (numpy uint8 [5056], advanced in place): float32 [epochs][n] (ag_torch_normal_epochs, the C
    restatement of torch's normal kernels; the same numbers as the calls themselves). On a torch
    build without the vectorised kernel the C restatement does not apply to n >= 16: the draws
    are then torch's own calls from `state` (the caller's generator state is left as it was)."""
    from . import _lib
    if n >= 16 and torch.backends.cpu.get_cpu_capability() not in TORCH_NORMAL_AVX2:
        saved = torch.get_rng_state()
        try:
            torch.set_rng_state(torch.from_numpy(state.copy()))
            out = np.empty((int(epochs), int(n)), np.float32)
            for e in range(int(epochs)):
                out[e] = torch.empty(int(n)).normal_().numpy()
            state[:] = torch.get_rng_state().numpy()
        finally:
            torch.set_rng_state(saved)
        return out
    L = _lib.load()
    out = np.empty((int(epochs), int(n)), np.float32)
    rc = L.ag_torch_normal_epochs(state.ctypes.data, state.nbytes, int(n), int(epochs), out.ctypes.data)
    _lib.check(rc, "ag_torch_normal_epochs", L)
    return out


def device_exp(x, sigmoid=False):
    """The kernels' exp (or sigmoid) on a float64 device tensor (known-answer hook)."""
    require_gpu()
    L = _lib.load()
    x = x.contiguous()
    y = torch.empty_like(x)
    f = L.ag_sigmoid if sigmoid else L.ag_exp
    _check(f(_ptr(x), _ptr(y), x.numel(), _stream()), "ag_exp")
    return y


def stream_copy(src, dst):
    """ag_stream_copy of src into dst (contiguous device tensors of the same byte size):
    the measured HBM peak of bench.py's roofline."""
    require_gpu()
    L = _lib.load()
    n = src.numel() * src.element_size()
    if dst.numel() * dst.element_size() != n or not (src.is_contiguous() and dst.is_contiguous()):
        raise ValueError("stream_copy: contiguous tensors of equal byte size")
    _check(L.ag_stream_copy(_ptr(src), _ptr(dst), n, _stream()), "ag_stream_copy")
