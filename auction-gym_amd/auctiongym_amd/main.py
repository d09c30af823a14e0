"""Experiment driver: the drop-in for src/main.py (parse_config / instantiate_agents /
instantiate_auction / the run x iteration x round loop / CSV outputs).

    python -m auctiongym_amd.main config/SP_Oracle.json      (from auction-gym_amd/)

Same JSON keys (CONFIG.md), same seeded catalogue draws, same plugin factory semantics
(class names from JSON evaluated with the rng, string kwargs quoted as in the reference
configs), same per-iteration prints and CSV files. The round loop of each iteration runs
as one batched GPU launch. Plots (src/main.py:239-326) are not produced.
"""
import argparse
import json
import os
from collections import defaultdict
from copy import deepcopy

import numpy as np

from .Agent import Agent
from .Auction import Auction
from .AuctionAllocation import FirstPrice, SecondPrice  # noqa: F401  (plugin registry)
from .Bidder import (DoublyRobustBidder, EmpiricalShadedBidder, PolicyLearningBidder,  # noqa: F401
                     TruthfulBidder, ValueLearningBidder)
from .BidderAllocation import OracleAllocator, PyTorchLogisticRegressionAllocator  # noqa: F401

PLUGINS = {c.__name__: c for c in (FirstPrice, SecondPrice, TruthfulBidder, EmpiricalShadedBidder,
                                   ValueLearningBidder, PolicyLearningBidder, DoublyRobustBidder,
                                   OracleAllocator, PyTorchLogisticRegressionAllocator)}


def parse_kwargs(kwargs):
    """src/main.py:19-21: ',k=v,...' appended to the constructor call string."""
    parsed = ",".join(f"{key}={value}" for key, value in kwargs.items())
    return "," + parsed if parsed else ""


def make_plugin(type_name, rng, kwargs, pass_rng=True):
    """The reference builds plugins with eval(f"{type}(rng=rng{kwargs})") (mechanisms with
    eval(f"{type}()")); the same call string is evaluated here against the plugin registry
    only."""
    if type_name not in PLUGINS:
        raise ValueError(f"unknown plugin type {type_name!r}")
    call = f"{type_name}(rng=rng{parse_kwargs(kwargs)})" if pass_rng else f"{type_name}()"
    return eval(call, {"__builtins__": {}}, dict(PLUGINS, rng=rng))


def parse_config(path):
    """src/main.py:24-74. Returns the reference's 10-tuple; the catalogue is drawn from the
    config's seeded Generator in the reference order: all embeddings, all values, then all
    intercepts -3 - U[0,1)."""
    with open(path) as f:
        config = json.load(f)
    rng = np.random.default_rng(config["random_seed"])
    np.random.seed(config["random_seed"])
    num_runs = config["num_runs"] if "num_runs" in config else 1
    max_slots = 1
    embedding_size = config["embedding_size"]
    embedding_var = config["embedding_var"]
    obs_embedding_size = config["obs_embedding_size"]

    agent_configs = []
    for agent_config in config["agents"]:
        copies = agent_config.get("num_copies")
        if copies is None:
            agent_configs.append(agent_config)
            continue
        for _ in range(copies):
            c = deepcopy(agent_config)
            c["name"] += f" {len(agent_configs) + 1}"
            agent_configs.append(c)

    emb = {c["name"]: rng.normal(0.0, embedding_var, size=(c["num_items"], embedding_size))
           for c in agent_configs}
    vals = {c["name"]: rng.lognormal(0.1, 0.2, c["num_items"]) for c in agent_configs}
    agents2items = {name: np.hstack((e, -3.0 - 1.0 * rng.random((e.shape[0], 1))))
                    for name, e in emb.items()}
    return (rng, config, agent_configs, agents2items, vals, num_runs, max_slots, embedding_size,
            embedding_var, obs_embedding_size)


def instantiate_agents(rng, agent_configs, agents2item_values, agents2items):
    """src/main.py:77-95."""
    agents = [Agent(rng=rng, name=c["name"], num_items=c["num_items"],
                    item_values=agents2item_values[c["name"]],
                    allocator=make_plugin(c["allocator"]["type"], rng, c["allocator"]["kwargs"]),
                    bidder=make_plugin(c["bidder"]["type"], rng, c["bidder"]["kwargs"]),
                    memory=c.get("memory", 0))
              for c in agent_configs]
    for agent in agents:
        if isinstance(agent.allocator, OracleAllocator):
            agent.allocator.update_item_embeddings(agents2items[agent.name])
    return agents


def instantiate_auction(rng, config, agents2items, agents2item_values, agents, max_slots,
                        embedding_size, embedding_var, obs_embedding_size):
    """src/main.py:98-109."""
    allocation = make_plugin(config["allocation"], rng, {}, pass_rng=False)
    auction = Auction(rng, allocation, agents, agents2items, agents2item_values, max_slots,
                      embedding_size, embedding_var, obs_embedding_size,
                      config["num_participants_per_round"])
    return auction, config["num_iter"], config["rounds_per_iter"], config["output_dir"]


MEASURES = ("net_utility", "gross_utility", "allocation_regret", "estimation_regret",
            "overbid_regret", "underbid_regret", "CTR_RMSE", "CTR_bias", "best_expected_value")


def simulation_run(auction, num_iter, rounds_per_iter, verbose=True):
    """src/main.py:112-155 for one run: per iteration, the rounds as one batch, then the
    per-agent metrics, update, clear. Returns (agent -> measure -> [per iteration], revenue)."""
    stats = {m: defaultdict(list) for m in MEASURES}
    revenue = []
    for i in range(num_iter):
        if verbose:
            print(f"==== ITERATION {i} ====")
        auction.simulate_batch(rounds_per_iter)
        if verbose:
            import pandas as pd
            print(pd.DataFrame({"Name": [a.name for a in auction.agents],
                                "Net": [a.net_utility for a in auction.agents],
                                "Gross": [a.gross_utility for a in auction.agents]}))
            print(f"\tAuction revenue: \t {auction.revenue}")
        for agent in auction.agents:
            agent.update(iteration=i, plot=False)
            s = agent.name
            stats["net_utility"][s].append(agent.net_utility)
            stats["gross_utility"][s].append(agent.gross_utility)
            stats["allocation_regret"][s].append(agent.get_allocation_regret())
            stats["estimation_regret"][s].append(agent.get_estimation_regret())
            stats["overbid_regret"][s].append(agent.get_overbid_regret())
            stats["underbid_regret"][s].append(agent.get_underbid_regret())
            stats["CTR_RMSE"][s].append(agent.get_CTR_RMSE())
            stats["CTR_bias"][s].append(agent.get_CTR_bias())
            stats["best_expected_value"][s].append(agent.get_mean_best_expected_value())
            agent.clear_utility()
            agent.clear_logs()
        revenue.append(auction.revenue)
        auction.clear_revenue()
    return stats, revenue


def _per_agent_rows(run2stats, measure, column):
    rows = {"Run": [], "Agent": [], "Iteration": [], column: []}
    for run, stats in run2stats.items():
        for agent, vals in stats[measure].items():
            for it, v in enumerate(vals):
                rows["Run"].append(run)
                rows["Agent"].append(agent)
                rows["Iteration"].append(it)
                rows[column].append(v)
    return rows


def write_csvs(output_dir, run2stats, run2revenue, rounds_per_iter, num_iter, num_runs,
               obs_embedding_size, embedding_size):
    """The CSV files of src/main.py:271,277,287,289,345 (same names and columns)."""
    import pandas as pd
    os.makedirs(output_dir, exist_ok=True)
    tag = (f"{rounds_per_iter}_rounds_{num_iter}_iters_{num_runs}_runs_"
           f"{obs_embedding_size}_emb_of_{embedding_size}")
    dfs = {}
    for measure, column, fname in (("net_utility", "Net Utility", "net_utility"),
                                   ("gross_utility", "Gross Utility", "gross_utility"),
                                   ("overbid_regret", "Overbid Regret", "overbid_regret"),
                                   ("underbid_regret", "Underbid Regret", "underbid_regret")):
        df = pd.DataFrame(_per_agent_rows(run2stats, measure, column))
        if measure in ("net_utility", "gross_utility"):
            df = df.sort_values(["Agent", "Run", "Iteration"])
        df.to_csv(f"{output_dir}/{fname}_{tag}.csv", index=False)
        dfs[measure] = (df, column)
    rev = pd.DataFrame({"Run": [r for r, v in run2revenue.items() for _ in v],
                        "Iteration": [i for v in run2revenue.values() for i in range(len(v))],
                        "Measure": [x for v in run2revenue.values() for x in v]})
    rev["Measure Name"] = "Auction Revenue"
    parts = [rev]
    for measure, name in (("net_utility", "Social Surplus"), ("gross_utility", "Social Welfare")):
        df, column = dfs[measure]
        g = df.groupby(["Run", "Iteration"])[column].sum().reset_index()
        g.columns = ["Run", "Iteration", "Measure"]
        g["Measure Name"] = name
        parts.append(g)
    pd.concat(parts).to_csv(f"{output_dir}/results_{tag}.csv", index=False)


def main(argv=None):
    parser = argparse.ArgumentParser()
    parser.add_argument("config", type=str, help="Path to experiment configuration file")
    parser.add_argument("--quiet", action="store_true")
    args = parser.parse_args(argv)
    (rng, config, agent_configs, agents2items, agents2item_values, num_runs, max_slots,
     embedding_size, embedding_var, obs_embedding_size) = parse_config(args.config)
    run2stats, run2revenue = {}, {}
    for run in range(num_runs):
        agents = instantiate_agents(rng, agent_configs, agents2item_values, agents2items)
        auction, num_iter, rounds_per_iter, output_dir = instantiate_auction(
            rng, config, agents2items, agents2item_values, agents, max_slots, embedding_size,
            embedding_var, obs_embedding_size)
        run2stats[run], run2revenue[run] = simulation_run(auction, num_iter, rounds_per_iter,
                                                          verbose=not args.quiet)
    write_csvs(output_dir, run2stats, run2revenue, rounds_per_iter, num_iter, num_runs,
               obs_embedding_size, embedding_size)
    return run2stats, run2revenue


if __name__ == "__main__":
    main()
