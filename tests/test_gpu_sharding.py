"""Query sharding on one GPU: a batch split into query slices walked with their global query
offset (``q_base``) reproduces the full-batch result bit for bit, with the production Philox
draws (no injected noise) -- the property ShardedEngine relies on across ranks (SURVEY §8(e):
per-query streams keyed by the global query index, shared root draws keyed without it).
Also: sharded injected noise, and the Gibbs do-value class check (gibbs.py:56-78)."""
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu


def _vbn(name):
    from vectorizedbayesiannetwork_amd import VBN
    from vectorizedbayesiannetwork_amd.model import model_from_checkpoint
    model = model_from_checkpoint(load_golden(name)["model"])
    return model, VBN.from_model(model, device="cuda")


def _mix12_query(b):
    g = torch.Generator().manual_seed(7)
    return {"target": "x10", "evidence": {"x0": torch.randn(b, 1, generator=g) * 0.3,
                                          "x6": torch.randn(b, 1, generator=g) * 0.3}}


def _same(a, b):
    """Bitwise equality with NaN == NaN."""
    return a.shape == b.shape and torch.equal(torch.isnan(a), torch.isnan(b)) and \
        torch.equal(torch.nan_to_num(a, nan=0.0), torch.nan_to_num(b, nan=0.0))


def _sliced(run, q, b, cut):
    from vectorizedbayesiannetwork_amd.distributed import shard_query
    from vectorizedbayesiannetwork_amd.engines import Query
    qq = Query(target=q["target"], evidence=q["evidence"], do=q.get("do", {}))
    return run(qq, 0), run(shard_query(qq, 0, cut), 0), run(shard_query(qq, cut, b), cut)


@pytest.mark.parametrize("engine", ["monte_carlo_marginalization", "importance_sampling",
                                    "likelihood_weighting", "resampled_importance_sampling"])
def test_query_slices_equal_full_batch(engine):
    from vectorizedbayesiannetwork_amd.registry import INFERENCE_REGISTRY
    _, vbn = _vbn("mix12")
    b, cut = 6, 4
    q = _mix12_query(b)
    # RIS: a threshold above S resamples at every check in every slice (the decision is
    # batch-global; ShardedEngine all-reduces it across ranks)
    extra = {"ess_threshold": 1e9} if engine == "resampled_importance_sampling" else {}
    # IS: its LW fallback is batch-global as well; ESS >= 1 always, so threshold 0 keeps it off

    def run(qq, q_base):
        eng = INFERENCE_REGISTRY[engine](n_samples=256, q_base=q_base, **extra)
        if hasattr(eng, "_lw"):
            eng._lw.q_base = q_base
            eng.ess_threshold = 0.0
        return eng.infer_posterior(vbn, qq, seed=1234)

    (pf, xf), (p0, x0), (p1, x1) = _sliced(run, q, b, cut)
    assert _same(torch.cat([p0, p1]), pf)
    assert _same(torch.cat([x0, x1]), xf)


@pytest.mark.parametrize("collect", ["reference", "chain"])
def test_gibbs_query_slices_equal_full_batch(collect):
    """Init walk (shared roots, per-query streams) and sweep walk (per-chain streams keyed by
    q_base + b) of a sliced batch reproduce the full batch exactly."""
    from vectorizedbayesiannetwork_amd.engines import GibbsSampler
    _, vbn = _vbn("ext_gibbs_mix10")
    b, cut = 5, 2
    g = torch.Generator().manual_seed(3)
    q = {"target": "x8", "evidence": {"x0": torch.randn(b, 1, generator=g) * 0.5}}

    def run(qq, q_base):
        return GibbsSampler(n_samples=6, burn_in=3, n_steps=2, collect=collect, q_base=q_base).sample(
            vbn, qq, seed=99)

    full, a, c = _sliced(run, q, b, cut)
    assert full.shape == (b, 6, 1)
    assert _same(torch.cat([a, c]), full)


def test_sharded_injected_noise_slices_with_the_queries():
    """slice_noise: the injected draws of a full batch, sliced per shard, give each shard the
    same outputs as the full-batch call (walk tensor form and node-dict form)."""
    from vectorizedbayesiannetwork_amd import engines as E
    from vectorizedbayesiannetwork_amd.distributed import shard_query, slice_noise
    model, vbn = _vbn("mix12")
    b, cut, n = 5, 3, 64
    q = E.Query(**_mix12_query(b))
    eng = E.LikelihoodWeighting(n_samples=n)
    g = torch.Generator().manual_seed(11)
    noise = {x: (torch.rand(b, n, generator=g), torch.randn(b, n, generator=g)) for x in model.topo}
    wf, xf = eng.infer_posterior(vbn, q, _noise=noise, seed=5)
    parts = []
    for b0, b1 in ((0, cut), (cut, b)):
        e = E.LikelihoodWeighting(n_samples=n, q_base=b0)
        parts.append(e.infer_posterior(vbn, shard_query(q, b0, b1), _noise=slice_noise(noise, b0, b1, b), seed=5))
    assert _same(torch.cat([p[0] for p in parts]), wf)
    assert _same(torch.cat([p[1] for p in parts]), xf)


def test_gibbs_rejects_out_of_class_do_value_on_scored_child():
    """A do-value on a discrete softmax_nn node with a latent parent is scored by every sweep
    (gibbs.py:56-78) and raises like softmax_nn._x_to_bin; with every parent observed the
    node is never scored and the value passes."""
    from vectorizedbayesiannetwork_amd import VBN
    from vectorizedbayesiannetwork_amd.engines import GibbsSampler
    from vectorizedbayesiannetwork_amd.model import model_from_checkpoint
    ck = load_golden("family_softmax_nn")["model"]
    ck = {**ck, "nodes": dict(ck["nodes"])}
    node = dict(ck["nodes"]["x5"])                  # x5 <- x3
    sd = dict(node["state_dict"])
    sd["_is_discrete"] = torch.tensor([True])
    sd["_class_values"] = torch.arange(8, dtype=torch.float32).view(1, 8)
    sd["_sample_values"] = torch.arange(8, dtype=torch.float32).view(1, 8)
    node["state_dict"] = sd
    ck["nodes"]["x5"] = node
    vbn = VBN.from_model(model_from_checkpoint(ck), device="cuda")
    gs = GibbsSampler(n_samples=2, burn_in=1, seed=0)
    ok = gs.sample(vbn, vbn._normalize_query({"target": "x7", "evidence": {}, "do": {"x5": torch.tensor([[3.0]])}}))
    assert ok.shape == (1, 2, 1)
    with pytest.raises(ValueError, match="outside discrete class set"):
        gs.sample(vbn, vbn._normalize_query({"target": "x7", "evidence": {}, "do": {"x5": torch.tensor([[3.5]])}}))
    # every parent of x5 observed: never scored, no error (as the reference)
    out = gs.sample(vbn, vbn._normalize_query({"target": "x7", "evidence": {"x3": torch.tensor([[0.1]])},
                                               "do": {"x5": torch.tensor([[3.5]])}}))
    assert out.shape == (1, 2, 1)
