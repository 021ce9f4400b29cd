#!/usr/bin/env python3
"""Golden fixtures for CPD shapes beyond the YAML defaults (build container only).

A 10-node DAG fitted by the reference with
* gaussian_nn ``hidden_dims=(64, 64)`` on 4 parent dims, a single-layer net ``hidden_dims=()``,
* mdn ``hidden_dims=(16,)`` (K = 3) and a root mdn (K = 4),
* softmax_nn ``hidden_dims=(32, 32, 32)``,
* a 3-dimensional linear_gaussian node,
* kde with 5 parent dims and kde with 5 target dims,
* a default (32, 32) gaussian_nn whose W2 is scaled by 1e6 (and W3 by 1e-6, the same
  function) -- beyond the f16 split range, so the walk takes its exact f32 chain,
and, for every node, per-CPD sample / log_prob, ``CPDHandle.conditional`` and
``BaseCPD.forward``, plus MCM / IS / LW / ancestral queries (reference
vbn/cpds/gaussian_nn.py:16-34 ``_build_mlp``; kde.py:105-182).
Writes ``tests/golden/shapes.pt``.  Usage: python tests/golden/make_golden_shapes.py
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
import make_golden_handle as H  # noqa: E402


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
    import vbn as vbn_mod
    G.deterministic_fits()

    g = nx.DiGraph()
    g.add_edges_from([("a", "b"), ("a", "c"), ("b", "c"), ("c", "d"), ("c", "e"), ("d", "e"), ("e", "f"),
                      ("r", "f"), ("b", "k5p"), ("c", "k5p"), ("d", "k5p"), ("a", "k5y"), ("c", "w")])
    gen = torch.Generator().manual_seed(17)
    n = 600
    nz = lambda *s: 0.3 * torch.randn(*s, generator=gen)   # noqa: E731
    d = {"a": torch.randn(n, 1, generator=gen)}
    d["r"] = torch.randn(n, 1, generator=gen) * 0.7 + 0.2
    d["b"] = d["a"] * torch.tensor([[0.5, -0.3, 0.8]]) + nz(n, 3)
    d["c"] = 0.4 * d["a"] + d["b"] @ torch.tensor([[0.3], [0.2], [-0.4]]) + nz(n, 1)
    d["d"] = torch.tanh(d["c"]) + nz(n, 1)
    d["e"] = 0.5 * d["c"] - 0.4 * d["d"] + nz(n, 1)
    d["f"] = 0.6 * d["e"] + 0.3 * d["r"] + nz(n, 1)
    d["k5p"] = 0.3 * d["b"].sum(1, keepdim=True) + 0.2 * d["c"] - 0.2 * d["d"] + nz(n, 1)
    d["k5y"] = d["a"] * torch.tensor([[0.5, -0.5, 0.2, 0.9, -0.1]]) + nz(n, 5)
    d["w"] = 0.7 * d["c"] + nz(n, 1)
    kinds = {"a": "gaussian_nn", "r": "mdn", "b": "linear_gaussian", "c": "gaussian_nn", "d": "mdn",
             "e": "softmax_nn", "f": "gaussian_nn", "k5p": "kde", "k5y": "kde", "w": "gaussian_nn"}
    extra = {"c": {"hidden_dims": (64, 64)}, "d": {"hidden_dims": (16,), "n_components": 3},
             "r": {"n_components": 4}, "e": {"hidden_dims": (32, 32, 32)}, "f": {"hidden_dims": ()},
             "k5p": {"max_points": 200}, "k5y": {"max_points": 150, "bandwidth": 0.6}}
    vbn = G.fit_model(vbn_mod, g, kinds, d, extra_kwargs=extra, epochs=3)
    with torch.no_grad():                     # W2 beyond the f16 split range, same function
        net = vbn.nodes["w"].net
        net[2].weight.mul_(1e6)
        net[2].bias.mul_(1e6)
        net[4].weight.mul_(1e-6)
    assert float(vbn.nodes["w"].net[2].weight.abs().max()) > 32768
    cases = G.model_cases(vbn, g, d, 12000, B=3, S=48)
    rows = torch.arange(3) * 5 + 1
    for i, node in enumerate(nx.topological_sort(g)):
        par_nodes = list(g.predecessors(node))
        par = None if not par_nodes else torch.cat([d[p][rows] for p in par_nodes], dim=-1)
        cases.append(G.run_cpd_case(vbn, node, 12500 + i, par, 24, x=d[node][rows]))
        rec = G.Recorder(12600 + i)
        rec.node = node
        with rec, torch.no_grad():
            out = vbn.cpd(node).conditional(par, n_samples=24)
        o = {k: H._as_tensor(out[k]) for k in H.TENSOR_FIELDS if k in out}
        o["format"] = out["format"]
        if "k" in out:
            o["k"] = int(out["k"])
        cases.append({"engine": "conditional", "node": node, "parents": par, "n_samples": 24, "seed": 12600 + i,
                      "draws": rec.records, "outputs": o})
        rec = G.Recorder(12700 + i)
        rec.node = node
        with rec, torch.no_grad():
            fo = vbn.nodes[node].forward(par, 16)
        cases.append({"engine": "forward", "node": node, "parents": par, "n_samples": 16, "seed": 12700 + i,
                      "draws": rec.records, "outputs": {"samples": fo.samples.detach().clone(),
                                                        "log_prob": fo.log_prob.detach().clone(),
                                                        "pdf": fo.pdf.detach().clone()}})
    fx = {"model": G.checkpoint_dict(vbn), "cases": cases}
    path = os.path.join(args.out, "shapes.pt")
    torch.save(fx, path)
    torch.load(path, weights_only=True)
    print(f"shapes: {len(cases)} cases -> {path} ({os.path.getsize(path) / 1024:.1f} KiB)")
    return 0


if __name__ == "__main__":
    sys.exit(main())
