"""Production draws (Philox on the GPU, no injected noise) are statistically right (SURVEY §8(c):
statistical parity for the production RNG), in particular the paired Box-Muller normals of
lean walks (plan.py _pair_normals, csrc draw_normal): the r cos / r sin halves of one pair feed
two nodes, which must stay independent N(0, 1) draws."""
import math

import networkx as nx
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _roots_model(n_roots=6, kinds=("linear_gaussian",)):
    """n independent roots (kinds round-robin) and one linear_gaussian child of the first two."""
    from vectorizedbayesiannetwork_amd import VBN, synthetic
    from vectorizedbayesiannetwork_amd.model import random_init_model
    g = nx.DiGraph()
    roots = [f"r{i}" for i in range(n_roots)]
    g.add_nodes_from(roots + ["c"])
    g.add_edge("r0", "c")
    g.add_edge("r1", "c")
    data = synthetic.sem_data(g, 2048, seed=0)
    kind_of = {n: kinds[i % len(kinds)] for i, n in enumerate(roots)}
    kind_of["c"] = "linear_gaussian"
    model = random_init_model(g, kind_of, data, seed=0, overrides={"kde": {"max_points": 512}})
    return model, VBN.from_model(model, device="cuda"), roots


def _ks_normal(z: np.ndarray) -> float:
    from scipy import stats
    return float(stats.kstest(z, "norm").statistic)


def test_paired_normals_are_independent_standard_normals():
    from vectorizedbayesiannetwork_amd import engines as E
    from vectorizedbayesiannetwork_amd.engines import AncestralSampler, Query
    model, vbn, roots = _roots_model()
    n = 1 << 18
    torch.manual_seed(0)
    xs = AncestralSampler(n_samples=n).sample(vbn, Query(target=None, evidence={}, do={}), n_samples=n)
    plan = E.LAST_LAUNCH["plan"]
    flags = plan.steps[:, 2].cpu().numpy()
    assert (flags & 512).sum() >= 2 and (flags & 1024).sum() >= 2          # pairs were formed
    z = {}
    for r in roots:
        rec = model.cpds[r]
        loc = float(rec.state["_bias"].reshape(-1)[0])
        x = xs[r].reshape(-1).double().cpu().numpy()
        sd = x.std()
        assert abs(x.mean() - loc) < 5 * sd / math.sqrt(n)
        z[r] = (x - x.mean()) / sd
        assert _ks_normal(z[r]) < 1.95 / math.sqrt(n) * 1.5                # KS at alpha ~ 1e-3, margin
    for i, a in enumerate(roots):
        for b in roots[i + 1:]:
            rho = float(np.corrcoef(z[a], z[b])[0, 1])
            assert abs(rho) < 5 / math.sqrt(n), (a, b, rho)
            # r cos and r sin share r: their squares would correlate if the pair were misused
            rho2 = float(np.corrcoef(z[a] ** 2, z[b] ** 2)[0, 1])
            assert abs(rho2) < 8 / math.sqrt(n), (a, b, rho2)


def test_paired_normals_leave_injected_noise_parity_alone():
    """With injected draws every step reads its own noise slot (the pairing is a production-
    path detail): each root is loc + its own injected normal x scale."""
    from vectorizedbayesiannetwork_amd import engines as E
    from vectorizedbayesiannetwork_amd.engines import AncestralSampler, Query
    model, vbn, roots = _roots_model(4)
    n = 256
    q = Query(target=None, evidence={}, do={})
    AncestralSampler(n_samples=n).sample(vbn, q, n_samples=n)
    pk, plan = E.LAST_LAUNCH["pk"], E.LAST_LAUNCH["plan"]
    g = torch.Generator(device="cpu").manual_seed(3)
    noise = torch.randn(len(plan.noise_nodes), 2, 1, n, pk.dmax, generator=g).cuda()
    xs = AncestralSampler(n_samples=n).sample(vbn, q, n_samples=n, _noise=noise)
    for r in roots:
        loc = float(model.cpds[r].state["_bias"].reshape(-1)[0])
        eps = noise[plan.noise_nodes.index(r), 1, 0, :, 0]
        ratio = (xs[r].reshape(-1) - loc) / eps
        assert torch.allclose(ratio, ratio[:1].expand_as(ratio), rtol=1e-4, atol=1e-5), r


def test_paired_normals_across_kinds_stay_independent():
    """Pairs also join mdn and kde draws (plan._pair_normals): roots of three kinds, sampled in
    the lean walk, stay pairwise uncorrelated (values and squares)."""
    from vectorizedbayesiannetwork_amd import engines as E
    from vectorizedbayesiannetwork_amd.engines import AncestralSampler, Query
    model, vbn, roots = _roots_model(6, kinds=("linear_gaussian", "mdn", "kde"))
    n = 1 << 17
    torch.manual_seed(2)
    xs = AncestralSampler(n_samples=n).sample(vbn, Query(target=None, evidence={}, do={}), n_samples=n)
    flags = E.LAST_LAUNCH["plan"].steps[:, 2].cpu().numpy()
    assert (flags & 1024).sum() >= 2
    z = {}
    for r in roots:
        x = xs[r].reshape(-1).double().cpu().numpy()
        assert np.isfinite(x).all()
        z[r] = (x - x.mean()) / x.std()
    for i, a in enumerate(roots):
        for b in roots[i + 1:]:
            assert abs(float(np.corrcoef(z[a], z[b])[0, 1])) < 5 / math.sqrt(n), (a, b)
            assert abs(float(np.corrcoef(z[a] ** 2, z[b] ** 2)[0, 1])) < 0.05, (a, b)   # heavy tails
