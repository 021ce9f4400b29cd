"""HIP path vs the oracle on the golden fixtures (same recorded draws injected).

Tolerances (fp32, the MLPs' sums are reassociated by MFMA/FMA vs the CPU sgemm):
  samples / target values : |d| <= 1e-5 + 1e-5 |x|
  pdf (MCM), CPD log-probs: log-density |d| <= 1e-4  (pdf: |d| <= 1e-4 |pdf|)
  IS/LW weights           : |d| <= 1e-4 |w|  (+1e-30: weights that underflow to 0)
  ESS                     : rel 1e-4
  softmax_nn bin indices  : bit-exact (checked through the bin-boundary log_prob cases)
  IS fallback decision    : identical
Categorical near-ties (large-M KDE fixtures: a recorded point whose CDF interval is narrower
than WIDTH_TIE) are compared like every other particle; a particle outside tolerance must be
one of them, and at most TIE_CAP of them may differ (counted and printed per case).
All run through the C-ABI library (vbn_hip_walk / vbn_hip_normalize_weights).
"""
import math

import pytest
import torch

from conftest import golden_names, load_golden
from golden_noise import noise_dict, resample_uniforms, tie_mask
from oracle import vbn_oracle as O

pytestmark = pytest.mark.gpu

S_ATOL, S_RTOL = 1e-5, 1e-5
P_ATOL, P_RTOL = 1e-30, 1e-4
LP_ATOL, LP_RTOL = 1e-4, 0.0
# large-M KDE fixtures (make_golden_large.py): a point whose CDF interval is narrower than this
# (fp32 chunk sums over up to 640 points vs the reference's float64 interval) may flip
WIDTH_TIE = 2e-5
TIE_CAP = 0.5          # at most this fraction of the near-tie particles may differ


def _vbn(fx):
    from vectorizedbayesiannetwork_amd import VBN
    from vectorizedbayesiannetwork_amd.model import model_from_checkpoint
    model = model_from_checkpoint(fx["model"])
    return model, VBN.from_model(model, device="cuda")


def _close(name, got, ref, atol, rtol, ties=None):
    """Elementwise |got - ref| <= atol + rtol |ref| with identical NaN / +-inf patterns.
    ``ties`` [B|1, S]: particles with a categorical near-tie; a particle may be out of tolerance
    only if it is one of them, and at most TIE_CAP of them (at least one) may be."""
    got = got.detach().float().cpu()
    ref = ref.detach().float().cpu()
    assert got.shape == ref.shape, f"{name}: shape {tuple(got.shape)} vs {tuple(ref.shape)}"
    nan_g, nan_r = torch.isnan(got), torch.isnan(ref)
    pos_g, pos_r = torch.isinf(got) & (got > 0), torch.isinf(ref) & (ref > 0)
    neg_g, neg_r = torch.isinf(got) & (got < 0), torch.isinf(ref) & (ref < 0)
    fin = torch.isfinite(got) & torch.isfinite(ref)
    err = torch.where(fin, (got - ref).abs(), torch.zeros_like(got))
    bad = (nan_g != nan_r) | (pos_g != pos_r) | (neg_g != neg_r) | (fin & (err > atol + rtol * ref.abs()))
    n_tie = n_bad = 0
    if ties is not None and ties.any() and got.dim() >= 2 and got.shape[1] == ties.shape[1]:
        t = ties if ties.shape[0] == got.shape[0] else ties.any(0, keepdim=True).expand(got.shape[0], -1)
        pb = bad.reshape(got.shape[0], got.shape[1], -1).any(-1)          # per particle
        n_tie, n_bad = int(t.sum()), int(pb.sum())
        unexplained = pb & ~t
        assert not unexplained.any(), (f"{name}: {int(unexplained.sum())} particles out of tolerance without a "
                                       f"categorical near-tie, max err {float(err[bad].max()):.3g}")
        assert n_bad <= max(1, int(TIE_CAP * n_tie)), f"{name}: {n_bad} of {n_tie} near-tie particles differ"
        keep = ~pb.view(pb.shape + (1,) * (got.dim() - 2)).expand_as(got)
        emax = float(err[keep].max()) if keep.any() else 0.0
        print(f"{name}: {n_bad} of {n_tie} near-tie particles differ; max err elsewhere {emax:.3g}")
        return emax
    assert not bad.any(), (f"{name}: {int(bad.sum())} of {bad.numel()} out of tolerance, "
                           f"max err {float(err[bad].max()):.3g} (atol {atol}, rtol {rtol})")
    return float(err.max()) if err.numel() else 0.0


def _cases():
    out = []
    for name in golden_names():
        fx = load_golden(name)
        has_kde = any(str(v["cpd_key"]) == "kde" for v in fx["model"]["nodes"].values())
        for i, case in enumerate(fx["cases"]):
            out.append(pytest.param(name, i, False, id=f"{name}-{i}-{case['engine']}"))
            if has_kde and case["engine"] not in ("cpd", "posterior_stats", "conditional", "forward"):
                # the alternative KDE distance path (packed VALU)
                out.append(pytest.param(name, i, True, id=f"{name}-{i}-{case['engine']}-kde_valu"))
    return out


@pytest.mark.parametrize("name,idx,kde_valu", _cases())
def test_golden_case_on_gpu(name, idx, kde_valu):
    from vectorizedbayesiannetwork_amd import cpd as C
    from vectorizedbayesiannetwork_amd.engines import (AncestralSampler, ImportanceSampling,
                                                       LikelihoodWeighting, MonteCarloMarginalization)
    fx = load_golden(name)
    case = fx["cases"][idx]
    model, vbn = _vbn(fx)
    eng = case["engine"]
    n = case["n_samples"]
    nd0 = noise_dict(case, model, 0) if eng != "gibbs" else None
    if eng == "cpd":
        node = case["node"]
        rec = model.cpds[node]
        par = case["parents"]
        xs = C.cpd_sample(vbn, node, None if par is None else par.cuda(), n, _noise=nd0)
        ref = O.cpd_sample(rec, par, n, O.ReplayDraws(case["draws"]))
        tm = tie_mask(case, model, 1 if par is None else par.shape[0], n, WIDTH_TIE)
        _close("cpd.sample", xs, ref, S_ATOL, S_RTOL, tm)
        lp = C.cpd_log_prob(vbn, node, ref.cuda(), None if par is None else par.cuda())
        _close("cpd.log_prob(sampled)", lp, O.cpd_log_prob(rec, ref, par), LP_ATOL, LP_RTOL)
        if "x" in case:
            lpx = C.cpd_log_prob(vbn, node, case["x"].cuda(), None if par is None else par.cuda())
            _close("cpd.log_prob(x)", lpx, O.cpd_log_prob(rec, case["x"], par), LP_ATOL, LP_RTOL)
        return
    if eng == "conditional":                  # CPDHandle.conditional (cpd_handle.py:348-404)
        node = case["node"]
        par = case["parents"]
        got = vbn.cpd(node).conditional_tensors(None if par is None else par.cuda(), n_samples=n, _noise=nd0)
        ref = O.conditional(model.cpds[node], par, n, O.ReplayDraws(case["draws"]))
        assert got["format"] == ref["format"] == case["outputs"]["format"]
        for k, v in ref.items():
            if isinstance(v, torch.Tensor):
                _close(f"conditional.{k}", got[k], v, S_ATOL, S_RTOL)
            else:
                assert got[k] == v, k
        return
    if eng == "forward":                      # BaseCPD.forward (core/base.py:55-59), one walk
        node = case["node"]
        par = case["parents"]
        out = C.cpd_forward(vbn, node, None if par is None else par.cuda(), n, _noise=nd0)
        ref = O.cpd_forward(model.cpds[node], par, n, O.ReplayDraws(case["draws"]))
        _close("forward.samples", out.samples, ref["samples"], S_ATOL, S_RTOL)
        _close("forward.log_prob", out.log_prob, ref["log_prob"], LP_ATOL, LP_RTOL)
        _close("forward.pdf", out.pdf, ref["pdf"], P_ATOL, P_RTOL)
        return
    if eng == "posterior_stats":
        st = vbn._posterior_stats(case["pdf"].cuda(), case["samples_in"].cuda())
        ref = O.posterior_stats(case["pdf"], case["samples_in"])
        for k in ("mean", "std", "ess"):
            _close(k, st[k], ref[k], 1e-5, 1e-5)
        return
    q = case["query"]
    qq = vbn._normalize_query(q)
    p = case["params"]
    draws = O.ReplayDraws(case["draws"])
    nb = int(next(iter((q["evidence"] or q["do"]).values())).shape[0]) if (q["evidence"] or q["do"]) else 1
    tm = tie_mask(case, model, nb, n, WIDTH_TIE)
    if tm is not None and tm.any():
        print(f"{name}[{idx}]: {int(tm.sum())} particles with a categorical near-tie (< {WIDTH_TIE})")
    if eng == "monte_carlo_marginalization":
        pdf, xs = MonteCarloMarginalization(n_samples=n, kde_valu=kde_valu).infer_posterior(vbn, qq, _noise=nd0)
        rpdf, rxs = O.monte_carlo_marginalization(model, q["target"], q["evidence"], q["do"], n, draws)
        _close("samples", xs, rxs, S_ATOL, S_RTOL, tm)
        _close("pdf", pdf, rpdf, P_ATOL, P_RTOL, tm)
    elif eng == "likelihood_weighting":
        e = LikelihoodWeighting(n_samples=n, normalize=p.get("normalize", True), kde_valu=kde_valu)
        w, xs = e.infer_posterior(vbn, qq, _noise=nd0)
        rw, rxs = O.likelihood_weighting(model, q["target"], q["evidence"], q["do"], n, draws,
                                         normalize=p.get("normalize", True))
        _close("samples", xs, rxs, S_ATOL, S_RTOL, tm)
        _close("weights", w, rw, P_ATOL, P_RTOL, tm)
    elif eng == "importance_sampling":
        e = ImportanceSampling(n_samples=n, kde_valu=kde_valu)
        e.ess_threshold = p.get("ess_threshold", 0.1)
        w, xs = e.infer_posterior(vbn, qq, _noise=nd0, _noise_fallback=noise_dict(case, model, 1))
        rw, rxs, ress, rfb = O.importance_sampling(model, q["target"], q["evidence"], q["do"], n, draws,
                                                   ess_threshold=e.ess_threshold)
        assert e._last_fallback == rfb == case["outputs"]["fallback"]
        _close("ess", e._last_ess, ress, 1e-5, 1e-4)
        _close("samples", xs, rxs, S_ATOL, S_RTOL, tm)
        _close("weights", w, rw, P_ATOL, P_RTOL, tm)
    elif eng == "ancestral":
        xs = AncestralSampler(n_samples=n, kde_valu=kde_valu).sample(vbn, qq, n, _noise=nd0)
        rxs = O.ancestral(model, q["target"], q["evidence"], q["do"], n, draws)
        _close("samples", xs, rxs, S_ATOL, S_RTOL, tm)
    elif eng == "resampled_importance_sampling":
        from vectorizedbayesiannetwork_amd.engines import ResampledImportanceSampling
        e = ResampledImportanceSampling(n_samples=n, kde_valu=kde_valu, **p)
        w, xs = e.infer_posterior(vbn, qq, _noise=nd0, _resample_u=[u.cuda() for u in resample_uniforms(case)])
        rw, rxs, ress, rrs = O.resampled_importance_sampling(
            model, q["target"], q["evidence"], q["do"], n, draws, ess_threshold=p.get("ess_threshold", 0.5),
            resample=p.get("resample", True), clamp_obs=p.get("clamp_obs", True))
        assert e._last_resampled == rrs == case["outputs"]["resampled"]
        if ress is not None:
            _close("ess", e._last_ess, ress, 1e-5, 1e-4)
        _close("samples", xs, rxs, S_ATOL, S_RTOL)
        _close("weights", w, rw, P_ATOL, P_RTOL)
    elif eng == "rao_blackwellized_marginalization":
        from vectorizedbayesiannetwork_amd.engines import RaoBlackwellizedMarginalization
        e = RaoBlackwellizedMarginalization(n_samples=n, n_particles=p["n_particles"], kde_valu=kde_valu)
        pdf, xs = e.infer_posterior(vbn, qq, _noise=nd0, _noise_fallback=noise_dict(case, model, 1))
        rpdf, rxs, reason = O.rao_blackwellized(model, q["target"], q["evidence"], q["do"], n,
                                                p["n_particles"], draws)
        if reason:
            rpdf, rxs = O.likelihood_weighting(model, q["target"], q["evidence"], q["do"], n, draws)
        assert e._last_fallback == bool(reason) == case["outputs"]["fallback"]
        assert (e._last_reason or "") == (reason or "")
        _close("samples", xs, rxs, S_ATOL, S_RTOL)
        _close("pdf", pdf, rpdf, P_ATOL, P_RTOL)
    elif eng == "gibbs":
        from golden_noise import gibbs_noise
        from vectorizedbayesiannetwork_amd.engines import GibbsSampler
        e = GibbsSampler(n_samples=n, kde_valu=kde_valu, **p)
        pk_latent = [x for x in model.topo if x not in q["evidence"] and x not in q["do"]]
        noise = gibbs_noise(case, model, pk_latent, max(model.out_dim(x) for x in model.topo))
        xs = e.sample(vbn, qq, n, _noise=noise)
        rxs = O.gibbs(model, q["target"], q["evidence"], q["do"], n, draws, **p)
        _close("samples", xs, rxs, S_ATOL, S_RTOL)
        _close("samples(reference)", xs, case["outputs"]["samples"], S_ATOL, S_RTOL)
        # chain mode: every collected sweep (oracle keeping copies instead of views)
        ec = GibbsSampler(n_samples=n, kde_valu=kde_valu, collect="chain", **p)
        xc = ec.sample(vbn, qq, n, _noise=noise)
        rxc = O.gibbs(model, q["target"], q["evidence"], q["do"], n, O.ReplayDraws(case["draws"]),
                      copy_collected=True, **p)
        _close("samples(chain)", xc, rxc, S_ATOL, S_RTOL)
    else:
        raise AssertionError(eng)


def test_softmax_bins_bit_exact_on_gpu():
    """Values exactly on bin edges and outside the range land in the reference bins
    (tests/test_cpds.py:66-82): log_prob picks log_softmax[bin] + within-bin density, so an
    off-by-one bin shows as a different finite value or a different -inf pattern."""
    from vectorizedbayesiannetwork_amd import cpd as C
    seen = 0
    for name in golden_names():
        fx = load_golden(name)
        model, vbn = _vbn(fx)
        for node, rec in model.cpds.items():
            if rec.kind != "softmax_nn" or bool(rec.state["_is_discrete"].any()):
                continue
            edges = rec.state["_bin_edges"]
            xs = torch.cat([edges.t(), edges[:, :1].t() - 3.0, edges[:, -1:].t() + 3.0], 0)  # [C+3, D]
            nb = xs.shape[0]
            par = None
            if model.parents[node]:
                par = torch.zeros(nb, rec.input_dim)
            got = C.cpd_log_prob(vbn, node, xs.cuda(), None if par is None else par.cuda()).cpu()
            ref = O.cpd_log_prob(rec, xs, par)
            assert torch.equal(torch.isinf(got), torch.isinf(ref)), (name, node)
            fin = torch.isfinite(ref)
            assert torch.allclose(got[fin], ref[fin], atol=LP_ATOL, rtol=0.0), (name, node)
            bins = O.smx_x_to_bin(rec, xs.unsqueeze(1))
            assert int(bins.min()) >= 0 and int(bins.max()) <= int(rec.hp("n_classes")) - 1
            seen += 1
    assert seen >= 3
