"""SURVEY §8(d) synthetic workloads for the GPU tests: the reference-fitted models of
``tests/golden/models`` (make_golden_models.py; random-init CPDs of the reference
architectures for a config without one), on-manifold evidence from the oracle's own
ancestral pass."""
from __future__ import annotations

import os

import torch

from oracle import vbn_oracle as O


MODELS_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "models")


def synthetic_workload(cfg_name: str, n_queries: int, device: str = "cuda"):
    """(model, vbn, target, evidence [n_queries, 1] per node on CPU) of config ``cfg_name``."""
    from vectorizedbayesiannetwork_amd import VBN, synthetic
    from vectorizedbayesiannetwork_amd.model import random_init_model
    cfg = synthetic.CONFIGS[cfg_name]
    g = synthetic.random_dag(cfg["n_nodes"], seed=0)
    model = synthetic.fitted_model(cfg_name, MODELS_DIR)
    if model is None:
        data = synthetic.sem_data(g, cfg.get("rows", 2048), seed=0)
        kinds = synthetic.round_robin_kinds(g, cfg["kinds"])
        overrides = {"kde": {"max_points": cfg["kde_max_points"]}} if "kde_max_points" in cfg else None
        model = random_init_model(g, kinds, data, seed=0, overrides=overrides)
    vbn = VBN.from_model(model, device=device)
    target, ev_nodes = synthetic.default_query_nodes(g, seed=1)
    torch.manual_seed(2)                         # on-manifold evidence: the model's own draw
    joint = O.ancestral(model, None, {}, {}, n_queries, O.TorchDraws())
    evidence = {n: joint[n][0].clone() for n in ev_nodes}
    return model, vbn, target, evidence
