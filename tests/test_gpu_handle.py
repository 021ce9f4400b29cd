"""CPD handles, wide-fan-in walks and op argument checks on the GPU.

* ``VBN.cpd(node)`` returns the reference ``CPDHandle`` surface (core/cpd_handle.py); its
  ``conditional`` dicts are the reference's formats after ``to_serializable`` (the values
  themselves are pinned against the reference in tests/test_gpu_parity.py, ext_handle_*).
* A gaussian_nn node with 510 parent dims: the two LDS weight buffers cannot fit next to the
  value slots, so the launch falls back to an unstaged kind set that reads the weights from
  the blob (csrc vbn_hip_walk) -- checked against the oracle on the production Philox draws.
* ``torch.ops.vbn_hip.walk`` rejects a ``wbuf`` smaller than the step table's weight blocks.
"""
from __future__ import annotations

import networkx as nx
import pytest
import torch

from oracle import vbn_oracle as O
from philox_draws import PhiloxDraws

pytestmark = pytest.mark.gpu


def _mix12():
    from conftest import load_golden
    from vectorizedbayesiannetwork_amd import VBN
    from vectorizedbayesiannetwork_amd.model import model_from_checkpoint
    model = model_from_checkpoint(load_golden("mix12")["model"])
    return model, VBN.from_model(model, device="cuda")


def test_handle_surface_formats():
    model, vbn = _mix12()
    handles = vbn.get_cpds()
    assert set(handles) == set(model.nodes)
    want = {"gaussian_nn": "normal_params", "linear_gaussian": "normal_params", "mdn": "mixture_params",
            "softmax_nn": "categorical_probs", "kde": "empirical_samples"}
    g = torch.Generator().manual_seed(0)
    for node, h in handles.items():
        rec = model.cpds[node]
        assert h.cpd_name == rec.kind and h.parents == model.parents[node] and h.is_fitted
        par = None if rec.input_dim == 0 else {p: torch.randn(4, 1, generator=g) for p in model.parents[node]}
        out = h.conditional(par, n_samples=16)
        assert out["format"] == want[rec.kind] and out["node"] == node
        assert isinstance(out.get("mean", out.get("weights", out.get("probs"))), list)
        fo = h.forward(par, 8)
        b = 1 if par is None else 4
        assert fo.samples.shape == (b, 8, rec.output_dim) and fo.log_prob.shape == (b, 8)
        assert torch.allclose(fo.pdf, fo.log_prob.exp())
        s = h.summary()
        assert s["cpd_type"] == h.cpd_type and s["input_dim"] == rec.input_dim
    with pytest.raises(ValueError, match="Unknown node"):
        vbn.cpd("nope")
    nonroot = next(n for n in model.topo if model.parents[n])
    with pytest.raises(ValueError, match="Parents required"):
        vbn.cpd(nonroot).conditional(None)


def test_wide_fan_in_runs_unstaged_and_matches_oracle():
    from vectorizedbayesiannetwork_amd import VBN
    from vectorizedbayesiannetwork_amd import engines as E
    from vectorizedbayesiannetwork_amd.engines import MonteCarloMarginalization, Query
    from vectorizedbayesiannetwork_amd.model import random_init_model
    g = nx.DiGraph()
    g.add_edges_from([("a", "c"), ("b", "c")])
    gen = torch.Generator().manual_seed(3)
    data = {"a": torch.randn(512, 255, generator=gen), "b": torch.randn(512, 255, generator=gen)}
    data["c"] = 0.01 * (data["a"].sum(1, keepdim=True) - data["b"].sum(1, keepdim=True)) + \
        0.3 * torch.randn(512, 1, generator=gen)
    model = random_init_model(g, {"a": "linear_gaussian", "b": "linear_gaussian", "c": "gaussian_nn"}, data, seed=0)
    vbn = VBN.from_model(model, device="cuda")
    B, S, seed = 2, 128, 4242
    pdf, xs = MonteCarloMarginalization(n_samples=S).infer_posterior(vbn, Query("c", {}), seed=seed)
    torch.cuda.synchronize()
    last = E.LAST_LAUNCH
    assert last["plan"].n_slots >= 511 and last["plan"].wbuf > 0
    draws = PhiloxDraws(last["plan"].steps, last["pk"].node_id, seed=seed, n_queries=1, n_samples=S)
    rpdf, rxs = O.monte_carlo_marginalization(model, "c", {}, {}, S, draws)
    assert torch.allclose(xs.cpu(), rxs, atol=1e-5, rtol=1e-5)
    assert torch.allclose(pdf.cpu(), rpdf, atol=1e-30, rtol=1e-4)


def test_walk_op_rejects_short_wbuf():
    from vectorizedbayesiannetwork_amd import engines as E
    from vectorizedbayesiannetwork_amd import ops
    from vectorizedbayesiannetwork_amd.engines import MonteCarloMarginalization, Query
    model, vbn = _mix12()
    MonteCarloMarginalization(n_samples=8).infer_posterior(vbn, Query(model.topo[-1], {}), seed=1)
    last = E.LAST_LAUNCH
    plan, pk = last["plan"], last["pk"]
    assert plan.wbuf > 0
    args = (plan.steps, plan.in_cols, pk.params, last["fixed"], None, plan.out_cols, 1, 8, plan.n_slots,
            plan.max_out, plan.fixed_ld, False, 1, len(plan.noise_nodes), pk.dmax, int(plan.out_cols.numel()),
            plan.mode, 0, 1, 0, True, plan.kind_mask)
    with pytest.raises(ValueError, match="wbuf"):
        ops.walk(*args, 0)
    ops.walk(*args, plan.wbuf)
    torch.cuda.synchronize()
