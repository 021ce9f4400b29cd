#!/usr/bin/env python3
"""Reference-fitted models of the SURVEY §8(d) benchmark workloads (build container only).

For each benchmark config (cfg2, cfg3, cfg4, cfg5, anchor64) this script builds the §8(d)
random DAG and linear-Gaussian SEM data (``vectorizedbayesiannetwork_amd.synthetic``), has the
reference (imported by path from ``/root/reference``; nothing of it is copied) fit every node
with the YAML hyper-parameters of its CPD kind and ``fit={"epochs": 1, "batch_size": 4096}``
(reference ``vbn/learning/node_wise.py:105-191``, ``cpds/gaussian_nn.py:121-192``, kde
``max_points`` per config), saves the model with the reference's own ``VBN.save`` and keeps the
checkpoint dict (tensors and builtins only, ``torch.load(weights_only=True)``) under
``tests/golden/models/<cfg>.pt``.

cfg4's KDE nodes store their training rows unchanged (M = 10,000 rows = ``max_points``, so
``kde.py:70-76`` keeps them in order and ``fit`` trains nothing): the script checks that the
fitted point sets equal the SEM data columns bit for bit and saves a 1-KiB marker instead of
6 MB of copies; :func:`vectorizedbayesiannetwork_amd.synthetic.fitted_model` rebuilds that
model from the data.

Usage: python tests/golden/make_golden_models.py [--out tests/golden/models] [--configs cfg2,...]
"""
from __future__ import annotations

import argparse
import os
import sys

# one OpenMP / MKL thread, fixed before torch loads: the reference's fits (linear_gaussian's
# lstsq, the NN epochs) then reproduce bit for bit from run to run (under the default thread
# pool the ridge weights drifted by up to 2.4e-7 between regenerations)
os.environ["OMP_NUM_THREADS"] = "1"
os.environ["MKL_NUM_THREADS"] = "1"

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

import make_golden as G  # noqa: E402
from vectorizedbayesiannetwork_amd import synthetic  # noqa: E402

CONFIGS = ("cfg2", "cfg3", "cfg4", "cfg5", "anchor64")


def fit_reference(cfg_name: str):
    from vbn import VBN, defaults
    G.deterministic_fits()
    cfg = synthetic.CONFIGS[cfg_name]
    g = synthetic.random_dag(cfg["n_nodes"], seed=0)
    data = synthetic.sem_data(g, cfg.get("rows", 2048), seed=0)
    kinds = synthetic.round_robin_kinds(g, cfg["kinds"])
    torch.manual_seed(0)                      # kde _limit_points draws a randperm from the global RNG
    vbn = VBN(g, seed=0, device="cpu")
    conf = {}
    for node in g.nodes:
        c = defaults.cpd(kinds[node])
        c["fit"] = {**c["fit"], "epochs": 1, "batch_size": 4096}
        if kinds[node] == "kde" and "kde_max_points" in cfg:
            c["max_points"] = cfg["kde_max_points"]
        conf[node] = c
    vbn.set_learning_method(defaults.learning("node_wise"), nodes_cpds=conf)
    vbn.fit({k: v for k, v in data.items()}, verbosity=0)
    return g, data, kinds, G.checkpoint_dict(vbn)


def kde_points_are_data(ck, g, data) -> bool:
    for node, info in ck["nodes"].items():
        ex = info.get("extra_state") or info["state_dict"].get("_extra_state")
        par = [data[p] for p in g.predecessors(node)]
        want_p = torch.cat(par, dim=-1) if par else torch.zeros(data[node].shape[0], 0)
        if not (torch.equal(ex["targets"], data[node]) and torch.equal(ex["parents"], want_p)):
            return False
    return True


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(HERE, "models"))
    ap.add_argument("--configs", default=",".join(CONFIGS))
    args = ap.parse_args()
    if not os.path.isdir(os.path.join(G.REF, "vbn")):
        print(f"reference not found at {G.REF}; nothing to do")
        return 0
    sys.path.insert(0, G.REF)
    os.environ.setdefault("CI", "1")
    os.makedirs(args.out, exist_ok=True)
    total = 0
    for name in args.configs.split(","):
        g, data, kinds, ck = fit_reference(name)
        if name == "cfg4":
            assert kde_points_are_data(ck, g, data), "cfg4's fitted KDE points differ from the SEM data"
            node0 = next(iter(ck["nodes"]))
            ck = {"kde_points_are_sem_data": True, "meta": ck["meta"],
                  "init_kwargs": dict(ck["nodes"][node0]["init_kwargs"])}
        ck["fit"] = {"epochs": 1, "batch_size": 4096, "config": name}
        path = os.path.join(args.out, f"{name}.pt")
        torch.save(ck, path)
        torch.load(path, weights_only=True)
        total += os.path.getsize(path)
        print(f"{name}: {os.path.getsize(path) / 1024:.1f} KiB -> {path}", flush=True)
    print(f"total {total / 1024:.1f} KiB")
    return 0


if __name__ == "__main__":
    sys.exit(main())
