"""Per-query evidence read once per wave (S a multiple of 64: every lane of a wave belongs to
one query, so the walk reads the query's evidence with a scalar load).

The golden fixtures all use sample counts that are not multiples of 64 (per-lane evidence
reads), so these cases pin the wave-uniform read against the oracle: a 4-node chain with
per-query evidence on the root and on the leaf, MCM and LW at S = 128 and 192 with the same
injected normal draws on both sides.
"""
import networkx as nx
import pytest
import torch

from oracle import vbn_oracle as O

pytestmark = pytest.mark.gpu


class _Seq:
    """The oracle's RNG interface, handing out the given normal draws in call order."""

    def __init__(self, zs):
        self.zs = list(zs)

    def normal(self, shape):
        z = self.zs.pop(0)
        assert z.numel() == torch.Size(shape).numel()
        return z.reshape(shape)


def _model():
    from vectorizedbayesiannetwork_amd.model import random_init_model
    g = nx.DiGraph()
    g.add_edges_from([("a", "b"), ("b", "c"), ("c", "d")])
    gen = torch.Generator().manual_seed(0)
    a = torch.randn(512, 1, generator=gen)
    b = 0.5 * a + 0.3 * torch.randn(512, 1, generator=gen)
    c = 0.5 * b + 0.3 * torch.randn(512, 1, generator=gen)
    d = 0.5 * c + 0.3 * torch.randn(512, 1, generator=gen)
    kinds = {"a": "linear_gaussian", "b": "gaussian_nn", "c": "gaussian_nn", "d": "gaussian_nn"}
    return random_init_model(g, kinds, {"a": a, "b": b, "c": c, "d": d}, seed=7)


@pytest.mark.parametrize("S", [128, 192])
def test_wave_uniform_evidence_matches_oracle(S):
    from vectorizedbayesiannetwork_amd import VBN
    from vectorizedbayesiannetwork_amd.engines import LikelihoodWeighting, MonteCarloMarginalization, Query
    model = _model()
    vbn = VBN.from_model(model, device="cuda")
    B = 5
    gen = torch.Generator().manual_seed(S)
    ev = {"a": torch.randn(B, 1, generator=gen), "d": torch.randn(B, 1, generator=gen)}
    zb, zc = torch.randn(B, S, 1, generator=gen), torch.randn(B, S, 1, generator=gen)
    nd = {"b": (None, zb), "c": (None, zc)}
    q = Query(target="c", evidence={k: v.cuda() for k, v in ev.items()}, do={})

    pdf, xs = MonteCarloMarginalization(n_samples=S).infer_posterior(vbn, q, _noise=nd)
    rp, rx = O.monte_carlo_marginalization(model, "c", ev, {}, S, _Seq([zb, zc]))
    torch.cuda.synchronize()
    assert torch.allclose(xs.cpu(), rx, rtol=1e-5, atol=1e-5)
    assert torch.allclose(pdf.cpu(), rp, rtol=1e-4, atol=1e-30)

    w, xs = LikelihoodWeighting(n_samples=S).infer_posterior(vbn, q, _noise=nd)
    rw, rx = O.likelihood_weighting(model, "c", ev, {}, S, _Seq([zb, zc]))
    torch.cuda.synchronize()
    assert torch.allclose(xs.cpu(), rx, rtol=1e-5, atol=1e-5)
    assert torch.allclose(w.cpu(), rw, rtol=1e-4, atol=1e-30)
    # the queries' evidence differs, so each query's particles must differ too
    assert not torch.allclose(xs[0].cpu(), xs[1].cpu())
