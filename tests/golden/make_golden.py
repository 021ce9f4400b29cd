#!/usr/bin/env python3
"""Generate golden fixtures from the Python reference (build container only).

Runs the reference (imported by path from ``/root/reference``; nothing of it is copied) on
small fitted models and records, for each case, every RNG draw the reference makes together
with its outputs.  RNG calls are routed through a recorder that keeps each draw's
distribution exactly:

* ``torch.randn_like`` / ``Normal.sample``  -> standard normal ``z`` (Normal.sample returns
  ``z*scale+loc``, bit-identical to ``torch.normal``);
* ``torch.rand_like``                       -> uniform ``u``;
* ``torch.multinomial(p, k)``               -> k inverse-CDF draws per row in fp64; the fixture
  stores the chosen index AND the midpoint of its CDF interval (``u_mid``), so a consumer that
  recomputes the probabilities in fp32 picks the same index from ``u_mid``;
* ``torch.randint(0, n, (k,))``             -> ``floor(u*n)``, stored as index and
  ``u_mid = (idx + 0.5) / n``.

Every saved object is a tensor or a builtin, so fixtures load with
``torch.load(weights_only=True)``.  The script exits 0 without writing when the reference
is not present (as on the GPU box).

Usage: python tests/golden/make_golden.py [--out tests/golden]
"""
from __future__ import annotations

import argparse
import contextlib
import math
import os
import sys
import tempfile

# one OpenMP / MKL thread, fixed before torch loads: the reference's fits (linear_gaussian's
# lstsq, the NN epochs) then reproduce bit for bit from run to run (under the default thread
# pool the ridge weights drifted by up to 2.4e-7 between regenerations)
os.environ["OMP_NUM_THREADS"] = "1"
os.environ["MKL_NUM_THREADS"] = "1"

import torch

REF = os.environ.get("VBN_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from vectorizedbayesiannetwork_amd import synthetic  # noqa: E402


class Recorder:
    """Context manager that replaces the reference's RNG entry points."""

    def __init__(self, seed: int):
        self.g = torch.Generator().manual_seed(seed)
        self.records = []
        self.node = None
        self.phase = 0
        self._saved = {}

    def _rec(self, kind, value, index=None):
        self.records.append({
            "kind": kind, "node": self.node, "phase": self.phase,
            "value": value.detach().to(torch.float32).reshape(-1).clone(),
            "index": None if index is None else index.detach().reshape(-1).clone(),
            "shape": list(value.shape),
        })

    def randn_like(self, t, *a, **k):
        z = torch.randn(t.shape, generator=self.g, dtype=torch.float32)
        self._rec("normal", z)
        return z.to(t.dtype)

    def rand_like(self, t, *a, **k):
        u = torch.rand(t.shape, generator=self.g, dtype=torch.float32)
        self._rec("uniform", u)
        return u.to(t.dtype)

    def randint(self, *args, **kw):
        if len(args) == 3:
            low, high, size = args
        elif len(args) == 2:
            low, high, size = 0, args[0], args[1]
        else:
            raise RuntimeError(f"unexpected randint signature {args} {kw}")
        n = int(high) - int(low)
        cnt = int(torch.Size(size).numel())
        u = torch.rand(cnt, generator=self.g, dtype=torch.float64)
        idx = torch.floor(u * n).long().clamp(max=n - 1)
        umid = (idx.double() + 0.5) / n
        self._rec("randint", umid, idx)
        return (idx + int(low)).reshape(tuple(size))

    def multinomial(self, probs, num_samples, replacement=False, *a, **k):
        if num_samples != 1:
            return self._multinomial_n(probs, int(num_samples), replacement)
        p = probs.detach().double()
        p = p / p.sum(-1, keepdim=True)
        cdf = p.cumsum(-1)
        cdf[:, -1] = 1.0
        u = torch.rand(p.shape[0], generator=self.g, dtype=torch.float64)
        idx = (cdf <= u.unsqueeze(-1)).sum(-1).clamp(max=p.shape[1] - 1)
        hi = cdf.gather(1, idx.unsqueeze(1)).squeeze(1)
        lo = torch.where(idx > 0, cdf.gather(1, (idx - 1).clamp(min=0).unsqueeze(1)).squeeze(1),
                         torch.zeros_like(hi))
        self._rec("cat", 0.5 * (lo + hi), idx)
        return idx.unsqueeze(1)

    def _multinomial_n(self, probs, n, replacement):
        """multinomial(p, n, replacement=True) (resampled_importance_sampling.py:38): n inverse-
        CDF draws per row, recorded as index + CDF-interval midpoint like the 1-draw case."""
        if not replacement:
            raise RuntimeError("recorder supports num_samples > 1 with replacement only")
        p = probs.detach().double()
        p = p / p.sum(-1, keepdim=True)
        cdf = p.cumsum(-1)
        cdf[:, -1] = 1.0
        u = torch.rand(p.shape[0], n, generator=self.g, dtype=torch.float64)
        idx = (cdf.unsqueeze(1) <= u.unsqueeze(-1)).sum(-1).clamp(max=p.shape[1] - 1)     # [b, n]
        hi = cdf.gather(1, idx)
        lo = torch.where(idx > 0, cdf.gather(1, (idx - 1).clamp(min=0)), torch.zeros_like(hi))
        self._rec("cat", 0.5 * (lo + hi), idx)
        return idx

    def normal_sample(self, dist, sample_shape=torch.Size()):
        shape = dist._extended_shape(torch.Size(sample_shape))
        with torch.no_grad():
            z = torch.randn(shape, generator=self.g, dtype=torch.float32)
            self._rec("normal", z)
            return z * dist.scale.expand(shape) + dist.loc.expand(shape)

    def __enter__(self):
        rec = self
        self._saved = {
            "randn_like": torch.randn_like, "rand_like": torch.rand_like,
            "randint": torch.randint, "multinomial": torch.multinomial,
            "Normal.sample": torch.distributions.Normal.sample,
        }
        torch.randn_like = self.randn_like
        torch.rand_like = self.rand_like
        torch.randint = self.randint
        torch.multinomial = self.multinomial
        torch.distributions.Normal.sample = lambda d, sample_shape=torch.Size(): rec.normal_sample(d, sample_shape)
        return self

    def __exit__(self, *exc):
        torch.randn_like = self._saved["randn_like"]
        torch.rand_like = self._saved["rand_like"]
        torch.randint = self._saved["randint"]
        torch.multinomial = self._saved["multinomial"]
        torch.distributions.Normal.sample = self._saved["Normal.sample"]


def tag_nodes(vbn, rec: Recorder):
    """Wrap each CPD's ``sample`` at instance level so draws carry their node name."""
    for name, cpd in vbn.nodes.items():
        orig = cpd.sample

        def wrapped(parents, n_samples, _orig=orig, _name=name):
            prev, rec.node = rec.node, _name
            try:
                return _orig(parents, n_samples)
            finally:
                rec.node = prev
        cpd.sample = wrapped


def untag_nodes(vbn):
    for cpd in vbn.nodes.values():
        cpd.__dict__.pop("sample", None)


# ------------------------------------------------------------------------------------------

def deterministic_fits():
    """Make the reference's linear_gaussian closed-form fit reproducible bit for bit (in this
    generator process only; the reference's files are untouched).  Its lstsq on the float32
    ridge system (linear_gaussian.py:79-126) drifts by up to ~1e-6 between runs even on one
    thread, which made regenerated fixtures differ in the fitted weights.  The same ridge
    least-squares problem -- weights and bias of [parents, 1], ridge on the weight block only,
    residual variance with Bessel's correction, clamped at 1e-6 -- is solved here in float64
    (normal equations) and rounded to float32 once.  The fixtures record the fitted model
    together with the reference's inference outputs ON that model, so how the weights were
    obtained does not enter any parity check."""
    import numpy as np
    from vbn.cpds.linear_gaussian import LinearGaussianCPD
    if getattr(LinearGaussianCPD, "_vbn_deterministic", False):
        return
    orig = LinearGaussianCPD._fit_closed_form

    def fit(self, parents, x, ridge):
        if parents.shape[0] == 0 or self.input_dim == 0:
            return orig(self, parents, x, ridge)
        reg = float(ridge)
        if reg < 0:
            raise ValueError("ridge must be >= 0")
        p64 = parents.detach().cpu().double().numpy()
        x64 = x.detach().cpu().double().numpy()
        a = np.concatenate([p64, np.ones((p64.shape[0], 1))], axis=1)
        d = p64.shape[1]
        g = a.T @ a
        g[np.arange(d), np.arange(d)] += reg
        theta = np.linalg.solve(g, a.T @ x64)
        var = (x64 - a @ theta).var(axis=0, ddof=1)
        t = torch.from_numpy(theta).to(device=self.device, dtype=x.dtype)
        s2 = torch.from_numpy(var).to(device=self.device, dtype=x.dtype).clamp_min(1e-6)
        return t[:-1], t[-1], s2

    LinearGaussianCPD._fit_closed_form = fit
    LinearGaussianCPD._vbn_deterministic = True


def fit_model(vbn_mod, g, kinds, data, extra_kwargs=None, epochs=3):
    from vbn import VBN, defaults
    vbn = VBN(g, seed=0, device="cpu")
    conf = {}
    for node in g.nodes:
        kind = kinds[node]
        c = defaults.cpd(kind)
        c["fit"] = {**c["fit"], "epochs": epochs, "batch_size": 256}
        if extra_kwargs and node in extra_kwargs:
            c.update(extra_kwargs[node])
        conf[node] = c
    vbn.set_learning_method(defaults.learning("node_wise"), nodes_cpds=conf)
    vbn.fit({k: v for k, v in data.items()}, verbosity=0)
    return vbn


def checkpoint_dict(vbn):
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "m.pt")
        vbn.save(path)
        ck = torch.load(path, map_location="cpu", weights_only=True)
    ck.pop("config", None)
    ck.pop("update_state", None)
    ck["meta"] = {"seed": ck["meta"].get("seed")}
    return ck


def run_case(vbn, seed, kind, query, n_samples, **params):
    from vbn.core.base import Query
    rec = Recorder(seed)
    out = {"engine": kind, "params": dict(params), "n_samples": int(n_samples),
           "query": {"target": query["target"],
                     "evidence": {k: v.clone() for k, v in query.get("evidence", {}).items()},
                     "do": {k: v.clone() for k, v in query.get("do", {}).items()}},
           "seed": seed}
    tag_nodes(vbn, rec)
    try:
        with rec:
            if kind == "ancestral":
                vbn.set_sampling_method("ancestral", n_samples=n_samples)
                s = vbn.sample(query, n_samples=n_samples)
                out["outputs"] = {"samples": s.clone()}
            else:
                vbn.set_inference_method(kind, n_samples=n_samples, **{k: v for k, v in params.items()
                                                                      if k != "ess_threshold"})
                eng = vbn._inference
                if "ess_threshold" in params:
                    eng.ess_threshold = params["ess_threshold"]
                if kind == "importance_sampling":
                    # LW fallback runs inside; mark its draws as phase 1
                    lw = eng._lw
                    orig = lw.infer_posterior

                    def lw_wrapped(*a, _o=orig, **k):
                        rec.phase = 1
                        return _o(*a, **k)
                    lw.infer_posterior = lw_wrapped
                pdf, samples = vbn.infer_posterior(query)
                out["outputs"] = {"pdf": pdf.clone(), "samples": samples.clone()}
                if kind == "importance_sampling":
                    out["outputs"]["ess"] = eng._last_ess.detach().clone()
                    out["outputs"]["fallback"] = bool(eng._last_fallback)
    finally:
        untag_nodes(vbn)
    out["draws"] = rec.records
    return out


def run_cpd_case(vbn, node, seed, parents, n_samples, x=None):
    cpd = vbn.nodes[node]
    rec = Recorder(seed)
    rec.node = node
    with rec:
        s = cpd.sample(parents, n_samples)
    out = {"engine": "cpd", "node": node, "n_samples": n_samples, "seed": seed,
           "parents": None if parents is None else parents.clone(),
           "draws": rec.records, "outputs": {"sample": s.detach().clone()}}
    with torch.no_grad():
        out["outputs"]["log_prob_sampled"] = cpd.log_prob(s, parents).detach().clone()
        if x is not None:
            out["x"] = x.clone()
            out["outputs"]["log_prob_x"] = cpd.log_prob(x, parents).detach().clone()
    return out


def query_rows(data, nodes, rows):
    return {n: data[n][rows].clone() for n in nodes}


def model_cases(vbn, g, data, seed0, B=3, S=16, extra=None):
    import networkx as nx
    topo = list(nx.topological_sort(g))
    cases = []
    target, ev_nodes = synthetic.default_query_nodes(g, seed=1)
    parents_t = list(g.predecessors(target))
    # make sure the full pass is exercised: not all target parents observed
    ev_nodes = [n for n in ev_nodes if n != target]
    if parents_t and all(p in ev_nodes for p in parents_t):
        ev_nodes = [n for n in ev_nodes if n != parents_t[0]]
    rows = torch.arange(B) * 7 + 3
    ev = query_rows(data, ev_nodes, rows)
    q = {"target": target, "evidence": ev}
    s = seed0
    cases.append(run_case(vbn, s + 1, "monte_carlo_marginalization", q, S))
    cases.append(run_case(vbn, s + 2, "importance_sampling", q, S, ess_threshold=0.0))
    cases.append(run_case(vbn, s + 3, "importance_sampling", q, S))
    cases.append(run_case(vbn, s + 4, "importance_sampling", q, S, ess_threshold=1.1))
    cases.append(run_case(vbn, s + 5, "likelihood_weighting", q, S))
    cases.append(run_case(vbn, s + 6, "likelihood_weighting", q, S, normalize=False))
    cases.append(run_case(vbn, s + 7, "ancestral", q, S))
    # parents-observed shortcut (Q2)
    nonroot = [n for n in topo if list(g.predecessors(n))]
    if nonroot:
        t2 = nonroot[-1]
        q2 = {"target": t2, "evidence": query_rows(data, list(g.predecessors(t2)), rows)}
        cases.append(run_case(vbn, s + 8, "monte_carlo_marginalization", q2, S))
        # target is evidence as well (Q17), full pass when some parent is latent
        q3 = {"target": t2, "evidence": query_rows(data, [t2], rows)}
        cases.append(run_case(vbn, s + 9, "monte_carlo_marginalization", q3, S))
    # root target (Q4): pdf (1,S)
    roots = [n for n in topo if not list(g.predecessors(n))]
    q4 = {"target": roots[0], "evidence": query_rows(data, [n for n in ev_nodes if n != roots[0]][:2], rows)}
    cases.append(run_case(vbn, s + 10, "monte_carlo_marginalization", q4, S))
    # do-target (Q3) and do on an ancestor
    q5 = {"target": target, "do": {target: data[target][rows].clone()}}
    cases.append(run_case(vbn, s + 11, "monte_carlo_marginalization", q5, S))
    anc = [n for n in topo if n != target and n not in ev_nodes]
    if anc:
        q6 = {"target": target, "evidence": ev, "do": {anc[0]: data[anc[0]][rows].clone()}}
        cases.append(run_case(vbn, s + 12, "monte_carlo_marginalization", q6, S))
        cases.append(run_case(vbn, s + 13, "likelihood_weighting", q6, S))
        cases.append(run_case(vbn, s + 14, "ancestral", q6, S))
    # single query (B=1) batch paths
    q7 = {"target": target, "evidence": {k: v[:1] for k, v in ev.items()}}
    cases.append(run_case(vbn, s + 15, "importance_sampling", q7, S, ess_threshold=0.0))
    cases.append(run_case(vbn, s + 16, "monte_carlo_marginalization", q7, S))
    # direct CPD cases (root and non-root) for every node kind present
    seen = set()
    for node in topo:
        kind = type(vbn.nodes[node]).__name__
        root = not list(g.predecessors(node))
        if (kind, root) in seen:
            continue
        seen.add((kind, root))
        par = None if root else torch.cat([data[p][rows] for p in g.predecessors(node)], dim=-1)
        x = data[node][rows]
        cases.append(run_cpd_case(vbn, node, s + 100 + len(seen), par, S, x=x))
    if extra:
        cases.extend(extra(vbn, g, data, rows, s))
    return cases


def softmax_edge_cases(vbn, g, data, rows, s):
    """Bin-boundary and off-manifold evidence for softmax_nn nodes (tests/test_cpds.py:66-82, Q6)."""
    out = []
    topo = [n for n in g.nodes]
    for node in topo:
        cpd = vbn.nodes[node]
        if type(cpd).__name__ != "SoftmaxNNCPD" or bool(cpd._is_discrete.any()):
            continue
        edges = cpd._bin_edges[0].detach().clone()
        par = None if not list(g.predecessors(node)) else torch.cat(
            [data[p][rows[:1]].expand(len(edges) + 2, -1) for p in g.predecessors(node)], dim=-1)
        xs = torch.cat([edges, edges[:1] - 1.0, edges[-1:] + 1.0]).unsqueeze(-1)
        c = run_cpd_case(vbn, node, s + 300, par if par is not None else None, 4, x=xs)
        out.append(c)
        # NaN-weight IS rows: evidence far outside the bins of a softmax_nn evidence node
        ch = list(g.successors(node))
        if ch:
            t = ch[0]
            q = {"target": t, "evidence": {node: torch.tensor([[float(edges[-1]) + 5.0], [float(edges[0]) - 5.0]])}}
            out.append(run_case(vbn, s + 301, "importance_sampling", q, 8))
        break
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=HERE)
    args = ap.parse_args()
    if not os.path.isdir(os.path.join(REF, "vbn")):
        print(f"reference not found at {REF}; nothing to do")
        return 0
    sys.path.insert(0, REF)
    os.environ.setdefault("CI", "1")
    import networkx as nx
    import vbn as vbn_mod  # noqa: F401
    deterministic_fits()

    torch.manual_seed(0)
    fixtures = {}

    # 1) README 3-node graph (README.md:84-127): gaussian_nn x2 + mdn(K=3)
    gen = torch.Generator().manual_seed(0)
    n = 1000
    x0 = torch.randn(n, generator=gen)
    x1 = torch.randn(n, generator=gen)
    x2 = 0.5 * x0 - 0.2 * x1 + 0.1 * torch.randn(n, generator=gen)
    g = nx.DiGraph()
    g.add_edges_from([("feature_0", "feature_2"), ("feature_1", "feature_2")])
    data = {"feature_0": x0.unsqueeze(-1), "feature_1": x1.unsqueeze(-1), "feature_2": x2.unsqueeze(-1)}
    kinds = {"feature_0": "gaussian_nn", "feature_1": "gaussian_nn", "feature_2": "mdn"}
    vbn = fit_model(vbn_mod, g, kinds, data, extra_kwargs={"feature_2": {"n_components": 3}}, epochs=20)
    cases = [run_case(vbn, 11, "monte_carlo_marginalization",
                      {"target": "feature_2", "evidence": {"feature_0": torch.tensor([[0.3]]),
                                                           "feature_1": torch.tensor([[-0.2]])}}, 200)]
    cases += model_cases(vbn, g, data, 20)
    fixtures["readme"] = {"model": checkpoint_dict(vbn), "cases": cases}

    # 2) per-family 8-node random DAGs (SURVEY §8(d) generator)
    g8 = synthetic.random_dag(8, seed=3)
    d8 = synthetic.sem_data(g8, 512, seed=0)
    for fam in ["gaussian_nn", "linear_gaussian", "mdn", "kde", "softmax_nn"]:
        kinds = synthetic.round_robin_kinds(g8, [fam])
        extra = {nd: {"max_points": 64} for nd in g8.nodes} if fam == "kde" else None
        vbn = fit_model(vbn_mod, g8, kinds, d8, extra_kwargs=extra)
        cases = model_cases(vbn, g8, d8, 1000 + 100 * len(fixtures),
                            extra=softmax_edge_cases if fam == "softmax_nn" else None)
        fixtures[f"family_{fam}"] = {"model": checkpoint_dict(vbn), "cases": cases}

    # 3) 12-node five-family mix (round robin)
    g12 = synthetic.random_dag(12, seed=5)
    d12 = synthetic.sem_data(g12, 512, seed=0)
    kinds = synthetic.round_robin_kinds(g12, ["gaussian_nn", "linear_gaussian", "mdn", "kde", "softmax_nn"])
    extra = {nd: {"max_points": 48} for nd in g12.nodes if kinds[nd] == "kde"}
    vbn = fit_model(vbn_mod, g12, kinds, d12, extra_kwargs=extra)
    fixtures["mix12"] = {"model": checkpoint_dict(vbn),
                         "cases": model_cases(vbn, g12, d12, 5000, extra=softmax_edge_cases)}

    # 4) variants: activations, within-bin modes, discrete softmax root, multi-dim nodes
    gv = nx.DiGraph()
    gv.add_edges_from([("c", "t"), ("t", "u"), ("c", "u"), ("u", "gl"), ("gl", "w"), ("w", "e"),
                       ("e", "v2"), ("t", "v2"), ("v2", "m2"), ("v2", "k2"), ("k2", "s2"), ("m2", "s2")])
    gen = torch.Generator().manual_seed(7)
    rows_v = 400
    dv = {"c": torch.randint(0, 3, (rows_v, 1), generator=gen).float()}
    dv["t"] = 0.4 * dv["c"] + 0.3 * torch.randn(rows_v, 1, generator=gen)
    dv["u"] = 0.5 * dv["t"] - 0.2 * dv["c"] + 0.3 * torch.randn(rows_v, 1, generator=gen)
    dv["gl"] = 0.7 * dv["u"] + 0.3 * torch.randn(rows_v, 1, generator=gen)
    dv["w"] = 0.5 * dv["gl"] + 0.3 * torch.randn(rows_v, 1, generator=gen)
    dv["e"] = -0.5 * dv["w"] + 0.3 * torch.randn(rows_v, 1, generator=gen)
    dv["v2"] = torch.cat([dv["e"] + dv["t"], dv["e"] - dv["t"]], 1) * 0.5 + 0.3 * torch.randn(rows_v, 2, generator=gen)
    dv["m2"] = dv["v2"] @ torch.tensor([[0.5, 0.1], [-0.3, 0.4]]) + 0.3 * torch.randn(rows_v, 2, generator=gen)
    dv["k2"] = dv["v2"].flip(1) * 0.6 + 0.3 * torch.randn(rows_v, 2, generator=gen)
    dv["s2"] = torch.cat([dv["k2"][:, :1] + dv["m2"][:, 1:], dv["m2"][:, :1]], 1) + 0.3 * torch.randn(rows_v, 2, generator=gen)
    kinds = {"c": "softmax_nn", "t": "gaussian_nn", "u": "softmax_nn", "gl": "gaussian_nn", "w": "softmax_nn",
             "e": "gaussian_nn", "v2": "linear_gaussian", "m2": "mdn", "k2": "kde", "s2": "softmax_nn"}
    extra = {"c": {"n_classes": 3}, "t": {"activation": "tanh"}, "u": {"within_bin": "uniform", "binning": "uniform"},
             "gl": {"activation": "gelu"}, "w": {"within_bin": "gaussian"}, "e": {"activation": "elu"},
             "m2": {"n_components": 3}, "k2": {"max_points": 40, "bandwidth": 0.4, "parent_bandwidth": 0.3},
             "s2": {"n_classes": 5}}
    vbn = fit_model(vbn_mod, gv, kinds, dv, extra_kwargs=extra)
    fixtures["variants"] = {"model": checkpoint_dict(vbn), "cases": model_cases(vbn, gv, dv, 7000)}

    os.makedirs(args.out, exist_ok=True)
    total = 0
    for name, fx in fixtures.items():
        path = os.path.join(args.out, f"{name}.pt")
        torch.save(fx, path)
        torch.load(path, weights_only=True)        # must be loadable without unpickling code
        total += os.path.getsize(path)
        print(f"{name}: {len(fx['cases'])} cases -> {path} ({os.path.getsize(path) / 1024:.1f} KiB)")
    print(f"total {total / 1024:.1f} KiB")
    return 0


if __name__ == "__main__":
    sys.exit(main())
