"""The posterior summary fused into the reductions (reference vbn/vbn.py:483-504
behind infer_relative 519-568): the MCM walk's epilogue partials + vbn_hip_posterior_stats_merge,
and the IS / LW normalisation with the summary in the same pass (vbn_hip_normalize_weights_stats).
Each is compared with the oracle's _posterior_stats (oracle/vbn_oracle.py posterior_stats, pinned
to the reference by tests/golden/ext_stats.pt) on the pdf / samples the same call returned.

Tolerance: the reference sums in float32 (torch order), the fused MCM form in float64 over 64-particle
waves merged pairwise, the fused normalisation in float32 with vbn_posterior_stats_kernel's tree; all
three agree to float32 accumulation error -- rtol 1e-4, atol 1e-6 (means / std of O(1) values over
<= 4096 samples)."""
import pytest
import torch

from conftest import load_golden
from oracle import vbn_oracle as O

pytestmark = pytest.mark.gpu

RTOL, ATOL = 1e-4, 1e-6


def _vbn(name):
    from vectorizedbayesiannetwork_amd import VBN
    from vectorizedbayesiannetwork_amd.model import model_from_checkpoint
    return VBN.from_model(model_from_checkpoint(load_golden(name)["model"]), device="cuda")


def _check(st, pdf, xs, eps=1e-12):
    assert "mean" in st, "the fused summary did not run"
    ref = O.posterior_stats(pdf.detach().cpu().double(), xs.detach().cpu().double(), eps)
    for k in ("mean", "std", "ess"):
        got = st[k].cpu()
        assert got.shape == ref[k].shape, k
        torch.testing.assert_close(got.double(), ref[k], rtol=RTOL, atol=ATOL, equal_nan=True,
                                   msg=lambda m, k=k: f"{k}: {m}")


def _query(vbn, target, ev_nodes, b, seed=0):
    g = torch.Generator().manual_seed(seed)
    ev = {n: torch.randn(b, vbn.model.out_dim(n), generator=g) * 0.5 for n in ev_nodes}
    return vbn._normalize_query({"target": target, "evidence": ev})


@pytest.mark.parametrize("fixture,target,ev", [
    ("readme", None, None),
    ("variants", "v2", None),       # gaussian_nn, 2 output columns
    ("variants", "k2", None),       # kde, 2 columns
    ("variants", "m2", None),       # mdn, 2 columns
    ("shapes", "k5y", None),        # 5 columns
])
def test_mcm_walk_epilogue_summary(fixture, target, ev):
    from vectorizedbayesiannetwork_amd.engines import MonteCarloMarginalization
    vbn = _vbn(fixture)
    topo = vbn.model.topo
    target = target or topo[-1]
    ev_nodes = [n for n in topo if n != target and vbn.model.out_dim(n) == 1
                and n not in vbn.model.parents.get(target, [])][:1]
    q = _query(vbn, target, ev_nodes, 3)
    for n in (64, 256, 1024):
        st = {"eps": 1e-12}
        pdf, xs = MonteCarloMarginalization(n_samples=n, seed=7).infer_posterior(vbn, q, _stats=st)
        torch.cuda.synchronize()
        _check(st, pdf, xs)


def test_mcm_summary_needs_whole_waves():
    """n_samples % 64 != 0: no fused summary (the facade runs the separate pass)."""
    from vectorizedbayesiannetwork_amd.engines import MonteCarloMarginalization
    vbn = _vbn("readme")
    q = _query(vbn, vbn.model.topo[-1], [], 2)
    st = {"eps": 1e-12}
    MonteCarloMarginalization(n_samples=100, seed=1).infer_posterior(vbn, q, _stats=st)
    assert "mean" not in st


def test_mcm_summary_across_kde_generations(monkeypatch):
    """cfg4 (KDE, M = 10,000) at 512 queries in generation launches (engines._generations,
    VBN_GEN_WAVES): each launch writes its own queries' partial rows."""
    from workloads import synthetic_workload
    from vectorizedbayesiannetwork_amd import engines as E
    from vectorizedbayesiannetwork_amd.engines import MonteCarloMarginalization
    monkeypatch.setattr(E, "GEN_WAVES", 2048)
    model, vbn, target, evidence = synthetic_workload("cfg4", 512)
    q = vbn._normalize_query({"target": target, "evidence": evidence})
    st = {"eps": 1e-12}
    eng = MonteCarloMarginalization(n_samples=1024, seed=3)
    pdf, xs = eng.infer_posterior(vbn, q, _stats=st)
    torch.cuda.synchronize()
    plan = E.LAST_LAUNCH["plan"]
    assert E._generations(plan.pc if plan.pc is not None else plan, 512, 1024) > 1
    _check(st, pdf, xs)


@pytest.mark.parametrize("engine", ["importance_sampling", "likelihood_weighting"])
@pytest.mark.parametrize("n", [200, 1024])
def test_weighted_normalisation_summary(engine, n):
    from vectorizedbayesiannetwork_amd.registry import INFERENCE_REGISTRY
    vbn = _vbn("mix12")
    topo = vbn.model.topo
    q = _query(vbn, topo[0], [topo[-1], topo[-2]], 4, seed=1)
    st = {"eps": 1e-12}
    eng = INFERENCE_REGISTRY[engine](n_samples=n, seed=11)
    pdf, xs = eng.infer_posterior(vbn, q, _stats=st)
    torch.cuda.synchronize()
    _check(st, pdf, xs)


def test_is_fallback_overwrites_the_summary():
    """ess_threshold above 1: every call falls back to likelihood weighting, and the summary is
    the one of the re-drawn outputs (the predicated normalisation rewrites it)."""
    from vectorizedbayesiannetwork_amd.engines import ImportanceSampling
    vbn = _vbn("mix12")
    topo = vbn.model.topo
    q = _query(vbn, topo[0], [topo[-1]], 3, seed=2)
    eng = ImportanceSampling(n_samples=256, seed=5)
    eng.ess_threshold = 2.0
    st = {"eps": 1e-12}
    pdf, xs = eng.infer_posterior(vbn, q, _stats=st)
    torch.cuda.synchronize()
    assert eng._last_fallback is True
    _check(st, pdf, xs)


def test_lw_unnormalised_summary():
    from vectorizedbayesiannetwork_amd.engines import LikelihoodWeighting
    vbn = _vbn("mix12")
    topo = vbn.model.topo
    q = _query(vbn, topo[1], [topo[-1]], 2, seed=3)
    st = {"eps": 1e-12}
    pdf, xs = LikelihoodWeighting(n_samples=512, seed=2, normalize=False).infer_posterior(vbn, q, _stats=st)
    torch.cuda.synchronize()
    _check(st, pdf, xs)


@pytest.mark.parametrize("s", [64, 1000, 4096])
def test_normalisation_summary_edge_rows(s):
    """Crafted log-weights: an ordinary row, an all -inf row (softmax NaN -> uniform weights), a
    row with a NaN weight, a one-hot row; samples with 2 columns, one NaN sample in the last row."""
    from vectorizedbayesiannetwork_amd import ops
    g = torch.Generator().manual_seed(s)
    lw = torch.randn(5, s, generator=g) * 3
    lw[1] = -float("inf")
    lw[2, s // 3] = float("nan")
    lw[3] = -float("inf")
    lw[3, 5] = 0.0
    x = torch.randn(5, s, 2, generator=g)
    x[4, 7, 1] = float("nan")
    lw, x = lw.cuda(), x.cuda()
    for normalize in (True, False):
        st = {"x": x, "eps": 1e-12}
        w, _, _ = ops.normalize_weights_ex(lw, normalize, 1e-12, stats=st)
        torch.cuda.synchronize()
        _check(st, w, x)
        # the separate pass on the same rows (a NaN sample keeps its NaN std, as clamp_min does)
        mean, std, ess = ops.posterior_stats(w, x, 1e-12)
        _check({"mean": mean, "std": std, "ess": ess}, w, x)


def test_infer_relative_takes_the_fused_forms():
    """infer_relative with MCM and IS: the same numbers as infer_posterior + the separate pass
    on an identically seeded engine."""
    for method, kw in (("monte_carlo_marginalization", {}), ("importance_sampling", {})):
        a, b = _vbn("mix12"), _vbn("mix12")
        a.set_inference_method(method, n_samples=512, seed=9, **kw)
        b.set_inference_method(method, n_samples=512, seed=9, **kw)
        topo = a.model.topo
        q = {"target": topo[0], "evidence": {topo[-1]: torch.tensor([[0.3], [-0.2]])}}
        out = a.infer_relative(q)
        qp, qs = b.infer_posterior(q)
        rp, rs = b.infer_posterior({"target": topo[0]})
        for stats, (p, s) in ((out["query_stats"], (qp, qs)), (out["reference_stats"], (rp, rs))):
            ref = b._posterior_stats(p, s)            # [1, ...] for the reference query: broadcast
            for got, want in ((stats["mean"], ref["mean"]), (stats["std"], ref["std"]),
                              (stats["effective_sample_size"], ref["ess"])):
                torch.testing.assert_close(got.cpu(), want.expand_as(got).cpu(), rtol=RTOL, atol=ATOL)
