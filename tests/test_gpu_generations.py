"""KDE walks launched in generations (engines.GEN_WAVES): the same particles, draws and outputs as
one launch, bit for bit (per-query draws are keyed by q_base + query, shared root draws by
sample only, per-query precompute rows sliced with the queries)."""
import pytest
import torch

from workloads import synthetic_workload

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg_name,engine", [("cfg4", "mcm"), ("cfg5", "mcm"), ("cfg5", "lw"), ("cfg4", "ancestral")])
def test_generations_equal_one_launch(cfg_name, engine, monkeypatch):
    from vectorizedbayesiannetwork_amd import engines as E
    from vectorizedbayesiannetwork_amd.engines import AncestralSampler, LikelihoodWeighting, MonteCarloMarginalization
    b, s = 8, 1024
    model, vbn, target, ev = synthetic_workload(cfg_name, b, "cuda")
    q = E.Query(target, {k: v.cuda() for k, v in ev.items()})

    def run():
        if engine == "mcm":
            return MonteCarloMarginalization(n_samples=s, plan_jit=False).infer_posterior(vbn, q, seed=99)
        if engine == "lw":
            return LikelihoodWeighting(n_samples=s, plan_jit=False).infer_posterior(vbn, q, seed=99)
        return (AncestralSampler(n_samples=s, plan_jit=False).sample(vbn, q, s, seed=99),)

    monkeypatch.setattr(E, "GEN_WAVES", 0)
    ref = run()
    torch.cuda.synchronize()
    monkeypatch.setattr(E, "GEN_WAVES", 40)             # 128 waves -> 3 launches (ragged: 3, 3, 2 queries)
    assert E._generations(E.LAST_LAUNCH["plan"], b, s) == 3
    got = run()
    torch.cuda.synchronize()
    for g, r in zip(got, ref):
        assert torch.equal(g, r)
