#!/usr/bin/env python3
"""Golden fixtures for the per-node CPD surface (build container only).

Loads the ``mix12`` and ``variants`` fixture models into the reference (``VBN.load`` of the
recorded checkpoint) and records, for every node:

* ``CPDHandle.conditional(parents)`` (vbn/core/cpd_handle.py:348-404): the normal / mixture /
  categorical parameters, or -- for kde -- the empirical summary of recorded draws;
* ``BaseCPD.forward(parents, n)`` (vbn/core/base.py:55-59): samples, log_prob, pdf.

Writes ``tests/golden/ext_handle.pt`` (tensors and builtins only).
Usage: python tests/golden/make_golden_handle.py [--out tests/golden]
"""
from __future__ import annotations

import argparse
import os
import sys
import tempfile

# one OpenMP / MKL thread, fixed before torch loads: the reference's fits (linear_gaussian's
# lstsq, the NN epochs) then reproduce bit for bit from run to run (under the default thread
# pool the ridge weights drifted by up to 2.4e-7 between regenerations)
os.environ["OMP_NUM_THREADS"] = "1"
os.environ["MKL_NUM_THREADS"] = "1"

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import make_golden as G  # noqa: E402

TENSOR_FIELDS = ("mean", "std", "weights", "loc", "scale", "probs", "support", "samples")


def _as_tensor(v):
    return torch.tensor(v, dtype=torch.float32) if isinstance(v, list) else v


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

    cases = []
    models = {}
    for src in ("mix12", "variants"):
        ck = torch.load(os.path.join(HERE, f"{src}.pt"), weights_only=True)["model"]
        with tempfile.TemporaryDirectory() as d:
            p = os.path.join(d, "m.pt")
            torch.save(ck, p)
            v = vbn_mod.VBN.load(p, map_location="cpu")
        models[src] = ck
        g = torch.Generator().manual_seed(11)
        for i, node in enumerate(ck["dag"]["topological_order"]):
            cpd = v.nodes[node]
            d_in = int(cpd.input_dim)
            par = None if d_in == 0 else torch.randn(3, d_in, generator=g) * 0.8
            seed = 40000 + 100 * len(models) + i
            # conditional (draws recorded: kde's empirical branch samples)
            rec = G.Recorder(seed)
            rec.node = node
            with rec, torch.no_grad():
                out = v.cpd(node).conditional(par, n_samples=32)
            o = {k: _as_tensor(out[k]) for k in TENSOR_FIELDS if k in out}
            o["format"] = out["format"]
            if "k" in out:
                o["k"] = int(out["k"])
            cases.append({"engine": "conditional", "source": src, "node": node, "parents": par,
                          "n_samples": 32, "seed": seed, "draws": rec.records, "outputs": o})
            # BaseCPD.forward
            rec = G.Recorder(seed + 50)
            rec.node = node
            with rec, torch.no_grad():
                fo = cpd.forward(par, 16)
            cases.append({"engine": "forward", "source": src, "node": node, "parents": par, "n_samples": 16,
                          "seed": seed + 50, "draws": rec.records,
                          "outputs": {"samples": fo.samples.detach().clone(), "log_prob": fo.log_prob.detach().clone(),
                                      "pdf": fo.pdf.detach().clone()}})
    # one fixture per source model (golden fixtures carry exactly one model)
    os.makedirs(args.out, exist_ok=True)
    for src, ck in models.items():
        fx = {"model": ck, "cases": [c for c in cases if c["source"] == src]}
        path = os.path.join(args.out, f"ext_handle_{src}.pt")
        torch.save(fx, path)
        torch.load(path, weights_only=True)
        print(f"ext_handle_{src}: {len(fx['cases'])} cases -> {path} ({os.path.getsize(path) / 1024:.1f} KiB)")
    return 0


if __name__ == "__main__":
    sys.exit(main())
