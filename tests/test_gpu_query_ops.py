"""Query-level custom ops (``torch.ops.vbn_hip.pack_plan / mcm / is_lw /
ancestral``, ops.py): an out-of-tree caller packs a query signature once (VBN.pack_query) and
runs the whole engine body in one op call.  Their outputs must equal the Python engines'
bit for bit (same plan, same walk, same seed), with and without the precompute sections."""
from __future__ import annotations

import pytest
import torch

from workloads import synthetic_workload

pytestmark = pytest.mark.gpu

B, S = 8, 1024


def _fixed(packed, ev, b, clamp=False):
    """the [b, fixed_ld] buffer in the plan's column order"""
    cols = []
    for n in packed["fixed_nodes"]:
        v = ev[n][:b].cuda().float().view(b, -1)
        if clamp:                            # clamp_evidence (inference/_core.py:112-114)
            v = torch.nan_to_num(v, nan=0.0, posinf=1e6, neginf=-1e6).clamp(-1e6, 1e6)
        cols.append(v)
    return torch.cat(cols, 1).contiguous()


@pytest.mark.parametrize("cfg_name", ["cfg2", "cfg3", "cfg5"])
@pytest.mark.parametrize("method", ["monte_carlo_marginalization", "importance_sampling", "likelihood_weighting",
                                    "ancestral"])
def test_query_ops_equal_engines(cfg_name, method):
    from vectorizedbayesiannetwork_amd.engines import Query
    from vectorizedbayesiannetwork_amd.registry import INFERENCE_REGISTRY, SAMPLING_REGISTRY
    b, s = B, S
    if cfg_name == "cfg5":
        b = 2
    model, vbn, target, ev = synthetic_workload(cfg_name, B, "cuda")
    sig = {"target": target, "evidence": list(ev)}
    packed = vbn.pack_query(sig, method, n_samples=s)
    assert packed["plan"].dtype == torch.int32 and packed["plan"].device.type == "cpu"
    q = Query(target, {k: v[:b].cuda() for k, v in ev.items()})
    seed = 8080
    fixed = _fixed(packed, ev, b, clamp=method == "likelihood_weighting")
    ops = torch.ops.vbn_hip
    if method == "monte_carlo_marginalization":
        ref = INFERENCE_REGISTRY[method](n_samples=s).infer_posterior(vbn, q, seed=seed)
        got = ops.mcm(packed["plan"], packed["params"], fixed, s, seed)
    elif method == "ancestral":
        ref = (SAMPLING_REGISTRY[method](n_samples=s).sample(vbn, q, s, seed=seed),)
        got = (ops.ancestral(packed["plan"], packed["params"], fixed, s, seed),)
    elif method == "likelihood_weighting":
        ref = INFERENCE_REGISTRY[method](n_samples=s).infer_posterior(vbn, q, seed=seed)
        w, x, ess, flag = ops.is_lw(packed["plan"], packed["params"], fixed, s, seed, lw_mode=True)
        got = (w, x)
    else:
        _check_is_op(vbn, sig, packed, q, ev, b, s, seed)
        return
    _equal(got, ref)


def _equal(got, ref):
    torch.cuda.synchronize()
    for g, r in zip(got, ref):
        assert g.shape == r.shape, (g.shape, r.shape)
        assert torch.equal(torch.nan_to_num(g, 7.0, 8.0, 9.0), torch.nan_to_num(r, 7.0, 8.0, 9.0))


def _check_is_op(vbn, sig, packed, q, ev, b, s, seed, expect_fallback=None):
    """vbn_hip::is_lw against the engine: the op's IS weights / samples / ESS equal the engine's
    walk before its fallback decision, its flag equals the engine's decision, and when the
    fallback fired, the caller's re-draw -- is_lw(lw_mode=True) on the likelihood-weighting
    signature with the engine's RNG offset 1 and clamped evidence -- equals the engine's final
    output (importance_sampling.py:82-88)."""
    from vectorizedbayesiannetwork_amd.registry import INFERENCE_REGISTRY
    ops = torch.ops.vbn_hip
    eng = INFERENCE_REGISTRY["importance_sampling"](n_samples=s)
    ref = eng.infer_posterior(vbn, q, seed=seed)
    w, x, ess, flag = ops.is_lw(packed["plan"], packed["params"], _fixed(packed, ev, b), s, seed)
    assert bool(flag) == eng._last_fallback
    if expect_fallback is not None:
        assert eng._last_fallback == expect_fallback
    assert torch.equal(torch.nan_to_num(ess, 7.0), torch.nan_to_num(eng._last_ess, 7.0))
    # the engine's IS walk and normalisation before the decision
    log_w, px = eng._walk(vbn, q, s, clamp=False, shared_roots=False, kwargs={"_seed_value": seed})
    pw, _ = ops.normalize_weights(log_w, True, 0.0)
    _equal((w, x), (pw, px))
    if not eng._last_fallback:
        _equal((w, x), ref)
        return
    pl = vbn.pack_query(sig, "likelihood_weighting", n_samples=s)
    lw_w, lw_x, _, lw_flag = ops.is_lw(pl["plan"], pl["params"], _fixed(pl, ev, b, clamp=True), s, seed, 1,
                                       lw_mode=True)
    assert not bool(lw_flag)
    _equal((lw_w, lw_x), ref)


def test_query_op_is_fallback_redraw():
    """The IS -> LW fallback through the query ops: off-manifold evidence in one query (an
    evidence node with latent parents, so its log-weight varies over the particles) collapses
    that query's ESS and fires the batch-global fallback."""
    from vectorizedbayesiannetwork_amd.engines import Query
    model, vbn, target, ev = synthetic_workload("cfg2", B, "cuda")
    par = model.parents
    k0 = next(k for k in sorted(ev) if par[k] and not any(p in ev for p in par[k]))
    ev = {k: v.clone() for k, v in ev.items()}
    ev[k0][B - 1, 0] = 50.0
    sig = {"target": target, "evidence": list(ev)}
    packed = vbn.pack_query(sig, "importance_sampling", n_samples=S)
    q = Query(target, {k: v.cuda() for k, v in ev.items()})
    _check_is_op(vbn, sig, packed, q, ev, B, S, 8181, expect_fallback=True)


def test_pack_plan_round_trip_and_errors():
    from vectorizedbayesiannetwork_amd import engines as E, ops
    model, vbn, target, ev = synthetic_workload("cfg2", B, "cuda")
    packed = vbn.pack_query({"target": target, "evidence": list(ev)}, "monte_carlo_marginalization")
    secs = ops._unpack(packed["plan"], torch.device("cuda", 0))
    assert secs[0] is not None and secs[1] is not None        # cfg2 MCM: walk + precompute variant
    assert secs[2] is not None                                # the per-sample pre-pass
    assert (secs[3] is not None) == E.PRECOMPUTE_Q            # the per-query pre-pass
    with pytest.raises(ValueError):
        torch.ops.vbn_hip.mcm(packed["plan"][:4].clone(), packed["params"], torch.zeros(B, 1, device="cuda"), S, 1)
    with pytest.raises(ValueError):
        torch.ops.vbn_hip.ancestral(packed["plan"], packed["params"],
                                    torch.zeros(B, len(packed["fixed_nodes"]), device="cuda"), S, 1)
