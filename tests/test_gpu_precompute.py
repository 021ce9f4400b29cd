"""Per-sample and per-query precompute on the GPU (plan.precompute_plans, engines.run_walk):
the walk that reads the per-sample quantities of nodes with shared-root parents (one-query
pre-pass) and the per-query quantities of nodes with evidence parents (one-wave-per-query
pre-pass) must give outputs bit-identical to the walk that recomputes them per particle -- for
MCM, IS, LW and ancestral, gaussian_nn / mdn / softmax_nn / KDE nodes, interpreter and
plan-specialised kernels.  The plain walk is pinned to the oracle per particle
(test_gpu_lean_parity.py), so this pins the precompute path."""
from __future__ import annotations

import pytest
import torch

from workloads import synthetic_workload

pytestmark = pytest.mark.gpu

B, S = 8, 1024


def _run(engine, vbn, q, precompute, plan_jit, seed, n=S):
    from vectorizedbayesiannetwork_amd import engines as E
    cls = {"mcm": E.MonteCarloMarginalization, "lw": E.LikelihoodWeighting, "ancestral": E.AncestralSampler,
           "is": E.ImportanceSampling}[engine]
    eng = cls(n_samples=n, plan_jit=plan_jit)
    old = E.PRECOMPUTE
    E.PRECOMPUTE = precompute
    try:
        out = eng.sample(vbn, q, n, seed=seed) if engine == "ancestral" else eng.infer_posterior(vbn, q, seed=seed)
        torch.cuda.synchronize()
    finally:
        E.PRECOMPUTE = old
    out = out if isinstance(out, tuple) else (out,)
    return [o.clone() for o in out], bool(E.LAST_LAUNCH.get("precomputed"))


def _same(a, b):
    return all(x.shape == y.shape and torch.equal(torch.nan_to_num(x, 7.0, 8.0, 9.0), torch.nan_to_num(y, 7.0, 8.0, 9.0))
               and torch.equal(torch.isnan(x), torch.isnan(y)) for x, y in zip(a, b))


@pytest.mark.parametrize("cfg_name,engine", [("cfg2", "mcm"), ("cfg2", "lw"), ("cfg2", "is"), ("anchor64", "mcm"),
                                             ("cfg3", "is"), ("cfg3", "lw"), ("cfg4", "mcm"), ("cfg4", "lw"),
                                             ("cfg5", "mcm"), ("cfg5", "lw"), ("cfg5", "ancestral")])
@pytest.mark.parametrize("plan_jit", [False, True])
def test_precompute_bit_identical(cfg_name, engine, plan_jit):
    from vectorizedbayesiannetwork_amd import jit
    from vectorizedbayesiannetwork_amd.engines import Query
    if plan_jit and not jit.enabled():
        pytest.skip("VBN_PLAN_JIT=0")
    model, vbn, target, ev = synthetic_workload(cfg_name, B, "cuda")
    q = Query(target, {k: v.cuda() for k, v in ev.items()})
    ref, p0 = _run(engine, vbn, q, False, plan_jit, seed=321)
    got, p1 = _run(engine, vbn, q, True, plan_jit, seed=321)
    from vectorizedbayesiannetwork_amd import engines as E
    plan = E.LAST_LAUNCH["plan"]
    assert not p0 and p1, "the precompute path did not run"
    assert plan.pre_q is not None, "every §8(d) query has nodes whose parents are all evidence"
    assert _same(got, ref)
    assert all(torch.isfinite(g).any() for g in got)


def test_precompute_needs_whole_waves_per_query():
    """S not a multiple of 64: waves straddle queries, so the walk recomputes every node."""
    from vectorizedbayesiannetwork_amd.engines import Query
    model, vbn, target, ev = synthetic_workload("cfg2", B, "cuda")
    q = Query(target, {k: v.cuda() for k, v in ev.items()})
    _, used = _run("mcm", vbn, q, True, False, seed=5, n=200)
    assert not used
