#!/usr/bin/env python3
"""Golden fixtures at the sizes the benchmark configs run (build container only).

The first fixtures keep every KDE at <= 64 points, so all points sit in the first of the
kernel's 16 inverse-CDF chunks.  These cover the realistic sizes:

* ``large_kde``: the 8-node random DAG (seed 3), kde CPDs fitted on 10,000 SEM rows with the
  YAML default ``max_points: 4096`` (vbn/configs/cpds/kde.yaml:4) and with ``max_points:
  10000`` (cfg4), B = 2 queries x S = 64 samples: MCM, IS, LW, ancestral, per-CPD cases for
  every parent count, and off-manifold evidence that underflows every kernel weight of a
  latent child (kde.py:105-182; chunking at 39, subsampling at 68-75);
* ``large_mix``: the 12-node five-family mix (seed 5) with kde ``max_points: 4096`` at
  S = 2048, B = 1 (cfg5's sample count).

Same recorder as ``make_golden.py``; categorical records also carry the width of the chosen
CDF interval (``width``) so a consumer can tell which choices are within fp32 rounding of a
boundary.  Usage: python tests/golden/make_golden_large.py [--out tests/golden]
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


class WidthRecorder(G.Recorder):
    def multinomial(self, probs, num_samples, replacement=False, *a, **k):
        out = super().multinomial(probs, num_samples, replacement, *a, **k)
        p = probs.detach().double()
        p = p / p.sum(-1, keepdim=True)
        cdf = p.cumsum(-1)
        cdf[:, -1] = 1.0
        idx = self.records[-1]["index"].view(p.shape[0], -1)
        hi = cdf.gather(1, idx)
        lo = torch.where(idx > 0, cdf.gather(1, (idx - 1).clamp(min=0)), torch.zeros_like(hi))
        self.records[-1]["width"] = (hi - lo).reshape(-1).float()
        return out


def _with_width_recorder(fn, *args, **kw):
    saved = G.Recorder
    G.Recorder = WidthRecorder
    try:
        return fn(*args, **kw)
    finally:
        G.Recorder = saved


def cases_for(vbn, g, data, seed0, B, S, far=None):
    import networkx as nx
    target, ev_nodes = G.synthetic.default_query_nodes(g, seed=1)
    parents_t = list(g.predecessors(target))
    ev_nodes = [n for n in ev_nodes if n != target]
    if parents_t and all(p in ev_nodes for p in parents_t):
        ev_nodes = [n for n in ev_nodes if n != parents_t[0]]
    rows = torch.arange(B) * 7 + 3
    q = {"target": target, "evidence": G.query_rows(data, ev_nodes, rows)}
    run = lambda *a, **k: _with_width_recorder(G.run_case, *a, **k)   # noqa: E731
    out = [run(vbn, seed0 + 1, "monte_carlo_marginalization", q, S),
           run(vbn, seed0 + 2, "importance_sampling", q, S, ess_threshold=0.0),
           run(vbn, seed0 + 3, "likelihood_weighting", q, S),
           run(vbn, seed0 + 4, "ancestral", q, S)]
    if far is not None:
        # every kernel weight of a latent child underflows in fp32 (the rescue path)
        node, value = far
        qf = {"target": target, "evidence": {node: torch.full((B, 1), float(value))}}
        out.append(run(vbn, seed0 + 5, "monte_carlo_marginalization", qf, S))
    seen = set()
    for node in nx.topological_sort(g):
        k = (type(vbn.nodes[node]).__name__, g.in_degree(node))
        if k in seen:
            continue
        seen.add(k)
        par = None if k[1] == 0 else torch.cat([data[p][rows] for p in g.predecessors(node)], dim=-1)
        out.append(_with_width_recorder(G.run_cpd_case, vbn, node, seed0 + 50 + len(seen), par, S,
                                        x=data[node][rows]))
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
    import vbn as vbn_mod
    G.deterministic_fits()

    torch.manual_seed(0)
    fixtures = {}
    g8 = G.synthetic.random_dag(8, seed=3)
    d8 = G.synthetic.sem_data(g8, 10000, seed=0)
    kinds = G.synthetic.round_robin_kinds(g8, ["kde"])
    # off-manifold value for the first root with a child: its children's kernel weights underflow
    root = next(n for n in g8.nodes if g8.in_degree(n) == 0 and g8.out_degree(n) > 0)
    cases, model = [], None
    for m, base in ((4096, 100), (10000, 200)):
        vbn = G.fit_model(vbn_mod, g8, kinds, d8, extra_kwargs={n: {"max_points": m} for n in g8.nodes})
        fixtures[f"large_kde{m}"] = {"model": G.checkpoint_dict(vbn),
                                     "cases": cases_for(vbn, g8, d8, 9000 + base, B=2, S=64, far=(root, 40.0))}

    g12 = G.synthetic.random_dag(12, seed=5)
    d12 = G.synthetic.sem_data(g12, 8192, seed=0)
    kinds = G.synthetic.round_robin_kinds(g12, ["gaussian_nn", "linear_gaussian", "mdn", "kde", "softmax_nn"])
    extra = {nd: {"max_points": 4096} for nd in g12.nodes if kinds[nd] == "kde"}
    vbn = G.fit_model(vbn_mod, g12, kinds, d12, extra_kwargs=extra)
    fixtures["large_mix12"] = {"model": G.checkpoint_dict(vbn),
                               "cases": cases_for(vbn, g12, d12, 9500, B=1, S=2048)}

    os.makedirs(args.out, exist_ok=True)
    total = 0
    for name, fx in fixtures.items():
        path = os.path.join(args.out, f"{name}.pt")
        torch.save(fx, path)
        torch.load(path, weights_only=True)
        total += os.path.getsize(path)
        print(f"{name}: {len(fx['cases'])} cases -> {path} ({os.path.getsize(path) / 1024:.1f} KiB)")
    print(f"total {total / 1024:.1f} KiB")
    return 0


if __name__ == "__main__":
    sys.exit(main())
