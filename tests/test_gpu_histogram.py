"""Discrete weighted histogram on the GPU (vbn_hip_discrete_posterior) against
the reference adapter's recorded outputs (benchmarking/models/vbn.py:202-242): bit-identical
float64 probabilities (sample-order float64 bins, numpy's pairwise normalisation), the same
exception types, and, at a full bench size, the oracle on IS weights the engine produced."""
import os

import pytest
import torch

from oracle import vbn_oracle as O

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _cases():
    return torch.load(os.path.join(HERE, "golden", "discrete_hist.pt"), weights_only=True)["cases"]


@pytest.mark.parametrize("case", _cases(), ids=lambda c: c["name"])
def test_matches_reference_fixture(case):
    from vectorizedbayesiannetwork_amd import posterior
    s, w = case["samples"].cuda(), case["weights"].cuda()
    if case.get("error"):
        with pytest.raises((ValueError, OverflowError)) as ei:
            posterior.estimate_discrete_posterior_batch(s, w, case["k"])
        assert type(ei.value).__name__ == case["error"]
        assert str(ei.value) == case["message"]
        return
    got = posterior.discrete_posterior(s, w, case["k"])
    assert got.dtype == torch.float64 and torch.equal(got.cpu(), case["probs"])
    lists = posterior.estimate_discrete_posterior_batch(s, w, case["k"])
    assert lists == case["probs"].tolist()
    one = posterior.estimate_discrete_posterior(s, w, case["k"])
    assert one == case["probs"][0].tolist()


def test_full_size_is_weights_match_oracle():
    """cfg2-shaped IS output (4096 queries x 1024 samples, k = 8 over the rounded target): every
    query's bins on the device, a 64-query sample of them against the oracle bit for bit."""
    from vectorizedbayesiannetwork_amd import posterior
    g = torch.Generator(device="cuda").manual_seed(5)
    b, s, k = 4096, 1024, 8
    xs = torch.randn(b, s, 1, device="cuda", generator=g) * 2.0 + 3.5
    logw = torch.randn(b, s, device="cuda", generator=g) * 3.0
    w = torch.softmax(logw, dim=1)
    got = posterior.discrete_posterior(xs, w, k).cpu()
    assert torch.allclose(got.sum(dim=1), torch.ones(b, dtype=torch.float64), atol=1e-12)
    rows = torch.arange(0, b, b // 64)
    want = torch.tensor(O.estimate_discrete_posterior_batch(xs[rows].cpu(), w[rows].cpu(), k), dtype=torch.float64)
    assert torch.equal(got[rows], want)


def test_engine_output_histogram():
    """A histogram of the target from VBN.infer_posterior's own weights and samples equals the
    oracle's on the same tensors (the adapter's call sequence, vbn.py:546-550)."""
    from conftest import load_golden
    from vectorizedbayesiannetwork_amd import VBN, posterior
    from vectorizedbayesiannetwork_amd.model import model_from_checkpoint
    vbn = VBN.from_model(model_from_checkpoint(load_golden("ext_rb_chain")["model"]), device="cuda")
    vbn.set_inference_method("likelihood_weighting", n_samples=2048)
    pdf, samples = vbn.infer_posterior({"target": "y", "evidence": {"x": torch.tensor([[1.0], [2.0], [0.0]])}})
    got = posterior.estimate_discrete_posterior_batch(samples, pdf, 6)
    want = O.estimate_discrete_posterior_batch(samples.cpu(), pdf.cpu(), 6)
    assert got == want
