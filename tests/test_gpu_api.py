"""Facade-level behaviour on the GPU that the golden cases do not cover directly
(reference tests/test_gaussian_exact_relative.py:40-57, tests/test_rao_blackwellized_marginalization.py)."""
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu


def _chain_vbn():
    from vectorizedbayesiannetwork_amd import VBN
    from vectorizedbayesiannetwork_amd.model import model_from_checkpoint
    return VBN.from_model(model_from_checkpoint(load_golden("ext_rb_chain")["model"]), device="cuda")


def test_infer_relative_shapes_and_direction():
    """x -> y linear chain (y ~ 1.2 x + 0.3): shifting the evidence up moves the posterior mean up."""
    vbn = _chain_vbn()
    vbn.set_inference_method("likelihood_weighting", n_samples=2048)
    torch.manual_seed(0)
    out = vbn.infer_relative(query={"target": "y", "evidence": {"x": torch.tensor([[1.0], [1.5]])}},
                             reference_query={"target": "y", "evidence": {"x": torch.tensor([[0.0]])}})
    assert out["target"] == "y"
    for k in ("delta_mean", "delta_std", "relative_mean_change", "relative_std_change"):
        assert out[k].shape == (2, 1) and torch.isfinite(out[k]).all()
    assert (out["delta_mean"] > 0).all()
    assert out["query_stats"]["effective_sample_size"].shape == (2,)
    with pytest.raises(ValueError, match="same target"):
        vbn.infer_relative({"target": "y", "evidence": {"x": torch.zeros(1, 1)}}, {"target": "z"})


def test_rb_mean_tracks_linear_conditional():
    """reference test_rb_marginalizes_missing_parents_for_linear_gaussian, on the GPU engine."""
    vbn = _chain_vbn()
    vbn.set_inference_method("rao_blackwellized_marginalization", n_samples=81, n_particles=256)
    pdf, samples = vbn.infer_posterior({"target": "y", "evidence": {"x": torch.tensor([[0.4]])}})
    assert pdf.shape == (1, 81) and samples.shape == (1, 81, 1)
    assert torch.isfinite(pdf).all() and torch.isfinite(samples).all()
    assert vbn._inference._last_fallback is False
    w = pdf / pdf.sum(dim=1, keepdim=True).clamp_min(1e-12)
    mean = (w.unsqueeze(-1) * samples).sum(dim=1).squeeze()
    rec = vbn.model.cpds["y"]
    expected = (torch.tensor([0.4]) @ rec.state["_weight"] + rec.state["_bias"]).squeeze()
    assert torch.allclose(mean.cpu(), expected, atol=0.25, rtol=0.15)
    vbn.set_inference_method("rao_blackwellized_marginalization", n_samples=9, n_particles=128)
    pdf, samples = vbn.infer_posterior({"target": "y", "evidence": {"z": torch.tensor([[0.2]])}})
    assert pdf.shape == (1, 9) and vbn._inference._last_fallback is True


def test_ris_production_rng_runs_and_normalizes():
    """RIS with Philox draws (no injected noise): weights normalised per query, resampling
    triggered by a threshold above S."""
    vbn = _chain_vbn()
    vbn.set_inference_method("resampled_importance_sampling", n_samples=512, ess_threshold=600.0)
    w, xs = vbn.infer_posterior({"target": "y", "evidence": {"z": torch.tensor([[0.2], [-0.4]])}})
    assert w.shape == (2, 512) and xs.shape == (2, 512, 1)
    assert torch.allclose(w.sum(dim=1).cpu(), torch.ones(2), atol=1e-5)
    assert vbn._inference._last_resampled is True


def test_gibbs_production_rng_chain_and_reference_modes():
    """GibbsSampler with Philox draws (gibbs.py:23-92): reference mode repeats the final sweep
    (gibbs.py:86 collects views), chain mode keeps every collected sweep; both target the same
    stationary distribution, and evidence on z moves y in the direction of y -> z (weight < 0)."""
    from vectorizedbayesiannetwork_amd.engines import GibbsSampler
    vbn = _chain_vbn()
    B = 1024
    ev = {"z": torch.cat([torch.full((B // 2, 1), 1.5), torch.full((B // 2, 1), -1.5)])}
    q = vbn._normalize_query({"target": "y", "evidence": ev})
    ref = GibbsSampler(n_samples=16, burn_in=20, n_steps=2, seed=3).sample(vbn, q)
    assert ref.shape == (B, 16, 1) and torch.isfinite(ref).all()
    assert torch.equal(ref, ref[:, :1].expand_as(ref))
    chain = GibbsSampler(n_samples=64, burn_in=20, n_steps=2, collect="chain", seed=4).sample(vbn, q)
    assert chain.shape == (B, 64, 1) and torch.isfinite(chain).all()
    assert float(chain.std(dim=1).mean()) > 1e-3                          # the chain moves
    w = float(vbn.model.cpds["z"].state["_weight"].squeeze())
    for half in (slice(0, B // 2), slice(B // 2, B)):
        m_ref, m_chain = float(ref[half, 0].mean()), float(chain[half].mean())
        assert abs(m_ref - m_chain) < 0.15, (m_ref, m_chain)
    up, down = float(chain[: B // 2].mean()), float(chain[B // 2:].mean())
    assert (up - down) * w > 0
    # n_samples = 0 and burn_in = 0: the initial ancestral state (gibbs.py:89-91)
    x0 = GibbsSampler(n_samples=0, burn_in=0, seed=5).sample(vbn, q, 0)
    assert x0.shape == (B, 1, 1)
    with pytest.raises(ValueError, match="collect"):
        GibbsSampler(collect="bogus")


@pytest.mark.parametrize("kinds", [("gaussian_nn",), ("gaussian_nn", "linear_gaussian", "mdn", "kde", "softmax_nn")])
def test_gibbs_half_wave_launch_matches_full_wave(kinds):
    """wave_particles 32 (lanes 32-63 mirror 0-31, one MFMA group, include/vbn_hip.h) gives the
    full-wave launch's chains: same Philox draws per (chain, candidate, sweep), same values; a
    chain count that is not a multiple of 4 leaves a partial last wave."""
    from vectorizedbayesiannetwork_amd import VBN, synthetic
    from vectorizedbayesiannetwork_amd.engines import GibbsSampler
    from vectorizedbayesiannetwork_amd.model import random_init_model
    g = synthetic.random_dag(12, seed=0)
    data = synthetic.sem_data(g, 512, seed=0)
    model = random_init_model(g, synthetic.round_robin_kinds(g, kinds), data, seed=0,
                              overrides={"kde": {"max_points": 256}})
    vbn = VBN.from_model(model, device="cuda")
    target, ev_nodes = synthetic.default_query_nodes(g, seed=1)
    B = 301
    torch.manual_seed(0)
    ev = {n: data[n][:B].reshape(B, 1).clone() for n in ev_nodes}
    q = vbn._normalize_query({"target": target, "evidence": ev})
    outs = [GibbsSampler(n_samples=6, burn_in=3, n_steps=2, collect="chain", seed=11, wave_particles=wp).sample(vbn, q)
            for wp in (64, 32)]
    assert outs[0].shape == (B, 6, 1) and torch.isfinite(outs[0]).all()
    torch.testing.assert_close(outs[1], outs[0], rtol=1e-5, atol=1e-5)
    with pytest.raises(ValueError, match="wave_particles"):
        GibbsSampler(wave_particles=16)
