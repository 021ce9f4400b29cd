#!/usr/bin/env python3
"""Golden fixtures for the Gibbs sampler (build container only).

Same recorder as ``make_golden.py``.  The initial ancestral draw of ``GibbsSampler.sample``
(gibbs.py:29) is phase 0; every sweep's draws are phase 1, in call order: per latent node
its 8-candidate draws (tagged with the node), then the chain choice (a ``cat`` record,
node None, gibbs.py:80).  Writes ``tests/golden/ext_gibbs.pt``.

Cases: a 10-node gaussian_nn / softmax_nn / linear_gaussian / mdn mix and a 6-node mix with
a kde node; B = 1 with latent roots (the reference indexes root candidates ``[1, 8, D]`` by
``arange(b)`` at gibbs.py:81, so latent roots need B = 1), and B = 3 with every root
observed; burn-in 0 / 3, thinning 1 / 2, a fixed target, a do node.

Usage: python tests/golden/make_golden_gibbs.py [--out tests/golden]
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
sys.path.insert(0, HERE)

import make_golden as G  # noqa: E402


def run_gibbs(vbn, seed, query, n_samples, burn_in, n_steps):
    import vbn.sampling.gibbs as gmod
    rec = G.Recorder(seed)
    out = {"engine": "gibbs", "params": {"burn_in": int(burn_in), "n_steps": int(n_steps)},
           "n_samples": int(n_samples),
           "query": {"target": query["target"],
                     "evidence": {k: v.clone() for k, v in query.get("evidence", {}).items()},
                     "do": {k: v.clone() for k, v in query.get("do", {}).items()}},
           "seed": seed}
    G.tag_nodes(vbn, rec)
    orig = gmod._ancestral_sample_tensor

    def anc(*a, **k):                               # initial state: phase 0, sweeps: phase 1
        rec.phase = 0
        try:
            return orig(*a, **k)
        finally:
            rec.phase = 1
    gmod._ancestral_sample_tensor = anc
    try:
        with rec:
            vbn.set_sampling_method("gibbs", n_samples=n_samples, burn_in=burn_in, n_steps=n_steps)
            s = vbn.sample(query, n_samples=n_samples)
            out["outputs"] = {"samples": s.detach().clone()}
    finally:
        gmod._ancestral_sample_tensor = orig
        G.untag_nodes(vbn)
    out["draws"] = rec.records
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=HERE)
    args = ap.parse_args()
    if not os.path.isdir(os.path.join(G.REF, "vbn")):
        print(f"reference not found at {G.REF}; nothing to do")
        return 0
    sys.path.insert(0, G.REF)
    os.environ.setdefault("CI", "1")
    import networkx as nx
    import vbn as vbn_mod  # noqa: F401
    G.deterministic_fits()
    from vectorizedbayesiannetwork_amd import synthetic

    torch.manual_seed(0)
    fixtures = {}

    g10 = synthetic.random_dag(10, seed=7)
    d10 = synthetic.sem_data(g10, 512, seed=0)
    kinds = synthetic.round_robin_kinds(g10, ["gaussian_nn", "softmax_nn", "linear_gaussian", "mdn"])
    vbn = G.fit_model(vbn_mod, g10, kinds, d10)
    topo = list(nx.topological_sort(g10))
    roots = [n for n in topo if g10.in_degree(n) == 0]
    rows = torch.arange(3) * 7 + 1
    r1 = rows[:1]
    mid = topo[len(topo) // 2]
    cases = [
        run_gibbs(vbn, 301, {"target": topo[-1], "evidence": {topo[3]: d10[topo[3]][r1]}}, 5, 2, 1),
        run_gibbs(vbn, 302, {"target": mid, "evidence": {topo[-1]: d10[topo[-1]][r1]}}, 4, 0, 2),
        run_gibbs(vbn, 303, {"target": topo[-1], "evidence": {r: d10[r][rows] for r in roots}}, 4, 3, 1),
        run_gibbs(vbn, 304, {"target": mid, "evidence": {**{r: d10[r][rows] for r in roots},
                                                          topo[-1]: d10[topo[-1]][rows]}}, 3, 1, 2),
        run_gibbs(vbn, 305, {"target": roots[0], "evidence": {r: d10[r][rows] for r in roots}}, 3, 1, 1),
        run_gibbs(vbn, 306, {"target": topo[-1], "evidence": {r: d10[r][rows] for r in roots[1:]},
                             "do": {roots[0]: d10[roots[0]][rows]}}, 3, 2, 1),
    ]
    fixtures["ext_gibbs_mix10"] = {"model": G.checkpoint_dict(vbn), "cases": cases}

    g6 = synthetic.random_dag(6, seed=5)
    d6 = synthetic.sem_data(g6, 512, seed=0)
    kinds = synthetic.round_robin_kinds(g6, ["kde", "gaussian_nn", "softmax_nn"])
    extra = {nd: {"max_points": 40} for nd in g6.nodes if kinds[nd] == "kde"}
    vbn = G.fit_model(vbn_mod, g6, kinds, d6, extra_kwargs=extra)
    topo = list(nx.topological_sort(g6))
    roots = [n for n in topo if g6.in_degree(n) == 0]
    cases = [
        run_gibbs(vbn, 311, {"target": topo[-1], "evidence": {topo[1]: d6[topo[1]][r1]}}, 4, 1, 1),
        run_gibbs(vbn, 312, {"target": topo[-1], "evidence": {r: d6[r][rows] for r in roots}}, 3, 2, 1),
    ]
    fixtures["ext_gibbs_kde6"] = {"model": G.checkpoint_dict(vbn), "cases": cases}

    os.makedirs(args.out, exist_ok=True)
    for name, fx in fixtures.items():
        path = os.path.join(args.out, f"{name}.pt")
        torch.save(fx, path)
        torch.load(path, weights_only=True)
        print(f"{name}: {len(fx['cases'])} cases -> {path} ({os.path.getsize(path) / 1024:.1f} KiB)")
    return 0


if __name__ == "__main__":
    sys.exit(main())
