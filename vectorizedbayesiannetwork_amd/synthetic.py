"""Synthetic workloads of SURVEY.md §8(d): random DAG, linear-Gaussian SEM data, queries.

These generators are shared by the golden-fixture script (which fits models with the
reference), the tests and ``bench.py`` (which builds random-init models of the same
architecture, see :mod:`vectorizedbayesiannetwork_amd.model`).

* DAG: nodes ``x0..x{N-1}``; for i >= 1 draw ``k = rng.randint(0, min(3, i))`` parents
  with ``rng.sample(range(i), k)`` (``rng = random.Random(seed)``), edges inserted in
  that order (the order fixes the parent-concat order, reference ``core/dags.py:31-33``).
* Data: ``x = 0.3 * N(0,1) + 0.5 * sum(parents)`` over ``nx.topological_sort`` with a
  ``torch.Generator().manual_seed(seed)``.
* Query: target = last node of the topological order; evidence =
  ``random.Random(seed).sample(topo[:-1], N // 4)``.
"""
from __future__ import annotations

import random
from typing import Dict, List, Sequence, Tuple

import networkx as nx
import torch

__all__ = [
    "random_dag",
    "sem_data",
    "round_robin_kinds",
    "default_query_nodes",
    "CONFIGS",
]


def random_dag(n_nodes: int, seed: int = 0, max_parents: int = 3) -> nx.DiGraph:
    rng = random.Random(seed)
    g = nx.DiGraph()
    names = [f"x{i}" for i in range(n_nodes)]
    g.add_nodes_from(names)
    for i in range(1, n_nodes):
        k = rng.randint(0, min(max_parents, i))
        for j in rng.sample(range(i), k):
            g.add_edge(names[j], names[i])
    return g


def sem_data(g: nx.DiGraph, n_rows: int, seed: int = 0) -> Dict[str, torch.Tensor]:
    gen = torch.Generator().manual_seed(seed)
    out: Dict[str, torch.Tensor] = {}
    for node in nx.topological_sort(g):
        x = 0.3 * torch.randn(n_rows, generator=gen)
        for p in g.predecessors(node):
            x = x + 0.5 * out[p][:, 0]
        out[node] = x.unsqueeze(-1)
    return out


def round_robin_kinds(g: nx.DiGraph, kinds: Sequence[str]) -> Dict[str, str]:
    return {node: kinds[i % len(kinds)] for i, node in enumerate(g.nodes)}


def fitted_model(cfg_name: str, models_dir: str):
    """The reference-fitted model of ``cfg_name`` (YAML hyper-parameters,
    ``fit={"epochs": 1, "batch_size": 4096}``, fitted by the reference in the build container,
    ``tests/golden/make_golden_models.py``), or None when ``models_dir`` has no fixture for it.

    cfg4's fixture is a marker: its KDE nodes keep their 10,000 training rows unchanged
    (M = ``max_points``), which the script checked bit for bit against the SEM data, so the
    model is rebuilt from the data with the recorded init kwargs."""
    import os

    from .model import model_from_checkpoint, random_init_model
    path = os.path.join(models_dir, f"{cfg_name}.pt")
    if not os.path.exists(path):
        return None
    ck = torch.load(path, weights_only=True)
    if ck.get("kde_points_are_sem_data"):
        cfg = CONFIGS[cfg_name]
        assert tuple(cfg["kinds"]) == ("kde",), f"{cfg_name}: the data marker is for KDE-only models"
        g = random_dag(cfg["n_nodes"], seed=0)
        data = sem_data(g, cfg.get("rows", 2048), seed=0)
        model = random_init_model(g, round_robin_kinds(g, cfg["kinds"]), data, seed=0,
                                  overrides={"kde": dict(ck["init_kwargs"])})
        for rec in model.cpds.values():
            assert rec.extra["targets"].shape[0] == int(ck["init_kwargs"]["max_points"])
        return model
    return model_from_checkpoint(ck)


def default_query_nodes(g: nx.DiGraph, seed: int = 1) -> Tuple[str, List[str]]:
    topo = list(nx.topological_sort(g))
    target = topo[-1]
    evidence = random.Random(seed).sample(topo[:-1], len(g.nodes) // 4)
    return target, evidence


# BASELINE.json "configs" (index 0..4). B = queries, S = samples per query.
CONFIGS = {
    "cfg1": dict(name="readme-3node-gaussian_nn-mcm", n_nodes=3, kinds=("gaussian_nn",),
                 engine="monte_carlo_marginalization", B=1, S=200),
    "cfg2": dict(name="32node-gaussian_nn-mcm", n_nodes=32, kinds=("gaussian_nn",),
                 engine="monte_carlo_marginalization", B=4096, S=1024, rows=2048),
    "cfg3": dict(name="32node-mdn+softmax_nn-is", n_nodes=32, kinds=("mdn", "softmax_nn"),
                 engine="importance_sampling", B=4096, S=1024, rows=2048),
    "cfg4": dict(name="64node-kde10k-mcm", n_nodes=64, kinds=("kde",),
                 engine="monte_carlo_marginalization", B=4096, S=1024, rows=10000,
                 kde_max_points=10000),
    "cfg5": dict(name="128node-mixed-mcm", n_nodes=128,
                 kinds=("gaussian_nn", "linear_gaussian", "mdn", "kde", "softmax_nn"),
                 engine="monte_carlo_marginalization", B=8192, S=2048, rows=8192,
                 kde_max_points=4096),           # B per GPU: 65,536 queries over 8 MI355X
    # §8(f) row on the cfg2 DAG: Rao-Blackwellized target (P = S = 1024)
    "rb32": dict(name="32node-gaussian_nn-rb", n_nodes=32, kinds=("gaussian_nn",),
                 engine="rao_blackwellized_marginalization", B=4096, S=1024, rows=2048),
    "ris32": dict(name="32node-gaussian_nn-ris", n_nodes=32, kinds=("gaussian_nn",),
                  engine="resampled_importance_sampling", B=4096, S=1024, rows=2048),
    "anchor64": dict(name="64node-gaussian_nn-mcm", n_nodes=64, kinds=("gaussian_nn",),
                     engine="monte_carlo_marginalization", B=4096, S=1024, rows=2048),
}
