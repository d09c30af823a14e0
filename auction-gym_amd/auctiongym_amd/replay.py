"""Replay-mode inputs: the reference's per-round random draws, in its order.

src/Auction.py draws, per round, from the ONE numpy Generator shared by everything
(src/main.py:29): integers(1, max_slots + 1) (:30; consumes nothing when max_slots == 1),
normal(0, embedding_var, E) (:33), choice(N, P, replace=False) (:42), then, after the
bids, binomial(1, CTR[winner]) (:65), which for n = 1 consumes exactly one next_double U.
TruthfulBidder / OracleAllocator draw nothing in between. Drawing U with rng.random()
leaves the Generator in the same state as the reference after every round
(tests/golden/make_golden.py asserts that on every captured round), so a batch of
rounds can be drawn up front and resolved on the GPU.

Populations with shading bidders or Thompson-sampling allocators draw more per round, in
slot order after the participants (src/Agent.py:44-53): a shading bidder in its
uninitialised state draws rng.normal(prev_gamma, gamma_sigma) (src/Bidder.py:51, 177, 354,
461); an LR-TS allocator draws torch.normal(0, 1/sqrt(q)) from torch's own global
generator (src/Models.py:31). draw_round_population makes the same calls in the same order.

(The one exception: numpy's binomial draws nothing when p == 0.0 exactly, i.e. when a
winner's sigmoid underflows to 0, which needs items . ctx < -745.)
"""
import numpy as np
import torch


def draw_round(rng, num_agents, num_participants, embedding_size, embedding_var, max_slots=1):
    rng.integers(1, max_slots + 1)
    ctx = rng.normal(0, embedding_var, size=embedding_size)
    part = rng.choice(num_agents, num_participants, replace=False)
    u = rng.random()
    return ctx, part, u


def draw_rounds(rng, B, num_agents, num_participants, embedding_size, embedding_var, max_slots=1):
    """B rounds -> SoA host arrays ctx [E][B] float64, part [P][B] int32, u [B] float64."""
    ctx = np.empty((embedding_size, B))
    part = np.empty((num_participants, B), np.int32)
    u = np.empty(B)
    for r in range(B):
        c, p, uu = draw_round(rng, num_agents, num_participants, embedding_size, embedding_var,
                              max_slots)
        ctx[:, r] = c
        part[:, r] = p
        u[r] = uu
    return ctx, part, u


M128 = (1 << 128) - 1
M64 = (1 << 64) - 1


def draw_rounds_native(rng, B, num_agents, num_participants, embedding_size, embedding_var, max_slots=1,
                       shading=None, out=None):
    """B rounds of draw_round (and, with `shading` [N] of (prev_gamma, gamma_sigma) or None,
    of draw_round_population's numpy-only draws: the shading bidders' Gaussian gammas) in C
    (ag_replay_draw), the same numbers and the same generator state afterwards as the Python
    loop. rng must be a numpy Generator on PCG64. Returns SoA host arrays ctx [E][B], part
    [P][B] int32, u [B] and gamma_raw [P][B] (NaN where nothing is drawn; None without
    shading). `out` may supply the arrays (e.g. pinned host tensors' numpy views)."""
    import ctypes

    from . import _lib
    bg = rng.bit_generator
    st = bg.state
    if st.get("bit_generator") != "PCG64":
        raise NotImplementedError("ag_replay_draw restates numpy's PCG64 only")
    s, inc = int(st["state"]["state"]), int(st["state"]["inc"])
    c = _lib.AgPcg64State(s >> 64, s & M64, inc >> 64, inc & M64, int(st["has_uint32"]), int(st["uinteger"]))
    B, N, P, E = int(B), int(num_agents), int(num_participants), int(embedding_size)
    o = out or {}
    ctx = o.get("ctx") if o.get("ctx") is not None else np.empty((E, B))
    part = o.get("part") if o.get("part") is not None else np.empty((P, B), np.int32)
    u = o.get("u") if o.get("u") is not None else np.empty(B)
    g = None
    sh = pg = gs = None
    if shading is not None:
        g = o.get("gamma_raw") if o.get("gamma_raw") is not None else np.empty((P, B))
        sh = np.array([x is not None for x in shading], np.uint8)
        pg = np.array([x[0] if x is not None else 0.0 for x in shading], np.float64)
        gs = np.array([x[1] if x is not None else 1.0 for x in shading], np.float64)
    for a in (ctx, part, u) + ((g,) if g is not None else ()):
        if not a.flags.c_contiguous:
            raise ValueError("replay arrays must be C-contiguous")
    ptr = lambda a: None if a is None else a.ctypes.data  # noqa: E731
    L = _lib.load()
    _lib.check(L.ag_replay_draw(ctypes.byref(c), B, N, P, E, float(embedding_var), int(max_slots), ptr(sh), ptr(pg),
                                ptr(gs), ptr(ctx), ptr(part), ptr(g), ptr(u)), "ag_replay_draw", L)
    st["state"]["state"] = (int(c.state_hi) << 64) | int(c.state_lo)
    st["state"]["inc"] = (int(c.inc_hi) << 64) | int(c.inc_lo)
    st["has_uint32"] = int(c.has_uint32)
    st["uinteger"] = int(c.uinteger)
    bg.state = st
    return ctx, part, u, g


def _pcg_in(rng):
    from . import _lib
    st = rng.bit_generator.state
    if st.get("bit_generator") != "PCG64":
        raise NotImplementedError("ag_replay_draw restates numpy's PCG64 only")
    s, inc = int(st["state"]["state"]), int(st["state"]["inc"])
    return st, _lib.AgPcg64State(s >> 64, s & M64, inc >> 64, inc & M64, int(st["has_uint32"]), int(st["uinteger"]))


def _pcg_out(rng, st, c):
    st["state"]["state"] = (int(c.state_hi) << 64) | int(c.state_lo)
    st["state"]["inc"] = (int(c.inc_hi) << 64) | int(c.inc_lo)
    st["has_uint32"] = int(c.has_uint32)
    st["uinteger"] = int(c.uinteger)
    rng.bit_generator.state = st


def draw_rounds_native_population(rng, B, num_agents, num_participants, embedding_size, embedding_var,
                                  shading, ts_models, max_slots=1, policy=None, search=None, kdo_max=None):
    """B rounds of draw_round_population in C (ag_replay_draw_population): numpy's draws and
    torch's (the LR-TS Thompson draws of src/Models.py:31, the fitted policies' rsample draws of
    src/Models.py:87-88 / :160-161) in the same order, with the same numbers, leaving both
    generators (rng and torch's global CPU generator) exactly where the Python loop leaves
    them. Returns ctx [E][B], part [P][B] int32, gamma_raw [P][B] (NaN where nothing is drawn)
    or None, u [B], ts_noise in the kernel's tile layout [P][ceil(B/64)][K*Do][64] or None,
    policy_eps [P][B] float32 or None, gamma_grid [P][128][B] or None. kdo_max: the noise rows'
    width K*Do (default: the largest model's)."""
    import ctypes

    from . import _lib
    B, N, P, E = int(B), int(num_agents), int(num_participants), int(embedding_size)
    st, c = _pcg_in(rng)
    u8 = lambda flags: None if flags is None or not any(flags) else np.array([bool(x) for x in flags], np.uint8)  # noqa: E731
    sh, ts, pol, sea = u8(None if shading is None else [x is not None for x in shading]), \
        u8(None if ts_models is None else [m is not None for m in ts_models]), u8(policy), u8(search)
    pg = gs = std = None
    KDo = 0
    ctx, part, u = np.empty((E, B)), np.empty((P, B), np.int32), np.empty(B)
    g = noise = eps = grid = None
    if sh is not None:
        pg = np.array([x[0] if x is not None else 0.0 for x in shading], np.float64)
        gs = np.array([x[1] if x is not None else 1.0 for x in shading], np.float64)
        g = np.empty((P, B))
    kdo = None
    if ts is not None:
        # an agent's own K*Do (src/main.py:61,66: per-agent num_items); the noise rows of the
        # largest model's width, an agent's draws in its first K_a*Do coefficients
        kdo = np.array([int(m.q.numel()) if m is not None else 0 for m in ts_models], np.int32)
        KDo = int(kdo_max) if kdo_max else int(kdo.max())
        std = np.zeros((N, KDo), np.float32)
        for a, m in enumerate(ts_models):
            if m is not None:
                std[a, :kdo[a]] = (1.0 / torch.sqrt(m.q)).numpy().ravel()  # as src/Models.py:31 computes it
        noise = np.empty((P, (B + 63) // 64, KDo, 64), np.float32)
    if pol is not None:
        eps = np.empty((P, B), np.float32)
    if sea is not None:
        grid = np.empty((P, 128, B))
    blob = None
    if ts is not None or pol is not None:
        blob = torch.get_rng_state().numpy().copy()
    ptr = lambda a: None if a is None else a.ctypes.data  # noqa: E731
    L = _lib.load()
    _lib.check(L.ag_replay_draw_population(ctypes.byref(c), ptr(blob), 0 if blob is None else blob.size, B, N, P, E,
                                           float(embedding_var), int(max_slots), ptr(sh), ptr(pg), ptr(gs), ptr(ts),
                                           ptr(std), KDo, ptr(kdo), ptr(pol), ptr(sea), ptr(ctx), ptr(part), ptr(g), ptr(u),
                                           ptr(noise), ptr(eps), ptr(grid)), "ag_replay_draw_population", L)
    _pcg_out(rng, st, c)
    if blob is not None:
        torch.set_rng_state(torch.from_numpy(blob))
    return ctx, part, g, u, noise, eps, grid


def draw_round_population(rng, num_agents, num_participants, embedding_size, embedding_var,
                          shading, ts_models, max_slots=1, policy=None, search=None, kdo_max=None):
    """One round of a general population. shading[a] = (prev_gamma, gamma_sigma) of a shading
    bidder in its uninitialised state (else None); ts_models[a] = the LR-TS model whose
    Thompson draw the round makes (else None); policy[a] = True for a learning bidder bidding
    from its fitted policy, whose rsample draws one standard normal from torch's generator
    (src/Models.py:87-88 / :160-161, via torch.distributions.Normal.rsample); search[a] = True
    for a ValueLearningBidder bidding by search, which draws rng.uniform(0.1, 1.0, 128) and
    sorts it (src/Bidder.py:184-186). Returns ctx [E], part [P], gamma_raw [P] (NaN where
    nothing is drawn), u, ts_noise [P][K*Do] float32 or None, policy_eps [P] float32 (0
    where nothing is drawn) or None, gamma_grid [P][128] (0 where nothing is drawn) or
    None."""
    rng.integers(1, max_slots + 1)
    ctx = rng.normal(0, embedding_var, size=embedding_size)
    part = rng.choice(num_agents, num_participants, replace=False)
    gamma_raw = np.full(num_participants, np.nan)
    noise = None
    eps = None
    grid = None
    for s, a in enumerate(part):
        m = ts_models[a]
        if m is not None:  # Agent.select_item: the allocator's Thompson draw first
            z = m.sample_noise().numpy().ravel()
            if noise is None:
                noise = np.zeros((num_participants, kdo_max or z.size), np.float32)
            noise[s, :z.size] = z  # an agent with fewer items: its rows first, zeros after
        if policy is not None and policy[a]:  # then the bidder's
            if eps is None:
                eps = np.zeros(num_participants, np.float32)
            eps[s] = torch.empty(1).normal_().item()
            continue
        if search is not None and search[a]:
            if grid is None:
                grid = np.zeros((num_participants, 128))
            gg = rng.uniform(0.1, 1.0, size=128)
            gg.sort()
            grid[s] = gg
            continue
        sh = shading[a]
        if sh is not None:
            gamma_raw[s] = rng.normal(sh[0], sh[1])
    u = rng.random()
    return ctx, part, gamma_raw, u, noise, eps, grid
