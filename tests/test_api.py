"""Facade / registry surface of the reference (vbn.py:257-335, 474-618; core/registry.py)."""
import pytest
import torch

from conftest import load_golden
from vectorizedbayesiannetwork_amd import INFERENCE_REGISTRY, SAMPLING_REGISTRY, VBN, ConfigItem, defaults
from vectorizedbayesiannetwork_amd.engines import (ImportanceSampling, LikelihoodWeighting,
                                                   MonteCarloMarginalization, Query)
from vectorizedbayesiannetwork_amd.model import model_from_checkpoint
from vectorizedbayesiannetwork_amd.registry import register_inference


@pytest.fixture()
def vbn_cpu():
    model = model_from_checkpoint(load_golden("readme")["model"])
    return VBN.from_model(model, device="cpu")


def test_registry_keys_match_reference_names():
    assert {"monte_carlo_marginalization", "importance_sampling", "likelihood_weighting"} <= set(INFERENCE_REGISTRY)
    assert "ancestral" in SAMPLING_REGISTRY
    with pytest.raises(ValueError):
        register_inference("importance_sampling")(type("X", (), {}))


def test_set_inference_method_forms(vbn_cpu):
    v = vbn_cpu
    v.set_inference_method("monte_carlo_marginalization", n_samples=7)
    assert isinstance(v._inference, MonteCarloMarginalization) and v._inference.n_samples == 7
    v.set_inference_method({"name": "likelihood_weighting", "normalize": False})
    assert isinstance(v._inference, LikelihoodWeighting) and v._inference.normalize is False
    v.set_inference_method(v.config.inference.importance_sampling, n_samples=33)
    assert isinstance(v._inference, ImportanceSampling) and v._inference.n_samples == 33
    assert v._inference.ess_threshold == 0.1
    v.set_inference_method(defaults.inference("monte_carlo_marginalization"))
    assert v._inference.n_samples == 1024                    # YAML default
    v.set_inference_method(ConfigItem(name="likelihood_weighting", params={"n_samples": 5}))
    assert v._inference.n_samples == 5
    fn = lambda *a, **k: None                                # noqa: E731
    v.set_inference_method(fn)
    assert v._inference is fn
    with pytest.raises(ValueError):
        v.set_inference_method("svgp")
    with pytest.raises(TypeError):
        v.set_inference_method({"n_samples": 3})
    with pytest.raises(TypeError):
        v.set_inference_method(3)
    v.set_sampling_method("ancestral", n_samples=4)
    assert v._sampling.n_samples == 4


def test_query_validation_errors(vbn_cpu):
    v = vbn_cpu
    with pytest.raises(RuntimeError):
        v.infer_posterior({"target": "feature_2"})
    with pytest.raises(RuntimeError):
        v.sample({"target": "feature_2"})
    v.set_inference_method("monte_carlo_marginalization", n_samples=4)
    with pytest.raises(ValueError, match="target"):
        v.infer_posterior({"evidence": {}})
    with pytest.raises(ValueError, match="Unknown target"):
        v.infer_posterior({"target": "nope"})
    with pytest.raises(ValueError, match="Unknown query nodes"):
        v.infer_posterior({"target": "feature_2", "evidence": {"zz": torch.zeros(2, 1)}})
    with pytest.raises(ValueError, match="both evidence and do"):
        v.infer_posterior({"target": "feature_2", "evidence": {"feature_0": torch.zeros(2, 1)},
                           "do": {"feature_0": torch.zeros(2, 1)}})
    with pytest.raises(ValueError, match="batch sizes must match"):
        v.infer_posterior({"target": "feature_2", "evidence": {"feature_0": torch.zeros(2, 1)},
                           "do": {"feature_1": torch.zeros(3, 1)}})
    with pytest.raises(TypeError):
        v.infer_posterior(["feature_2"])
    q = v._normalize_query({"target": "feature_2", "evidence": {"feature_0": [0.1, 0.2]}})
    assert q.evidence["feature_0"].shape == (2, 1) and q.evidence["feature_0"].dtype == torch.float32


def test_no_cpu_fallback(vbn_cpu):
    """The accelerated engines refuse to run off-GPU instead of silently using the CPU."""
    vbn_cpu.set_inference_method("importance_sampling", n_samples=4)
    with pytest.raises(RuntimeError, match="MI355X"):
        vbn_cpu.infer_posterior({"target": "feature_2", "evidence": {"feature_0": torch.zeros(2, 1)}})


def test_engine_accepts_reference_style_vbn_duck_type():
    """Engines read vbn.dag / vbn.nodes / vbn.device only (reference engine protocol)."""
    from vectorizedbayesiannetwork_amd.model import model_from_vbn

    class FakeCPD(torch.nn.Module):
        def __init__(self, d_in):
            super().__init__()
            self.input_dim, self.output_dim = d_in, 1
            self.register_buffer("_weight", torch.ones(d_in, 1))
            self.register_buffer("_bias", torch.zeros(1))
            self.register_buffer("_var", torch.ones(1))

        def get_init_kwargs(self):
            return {"ridge": 1e-6, "min_scale": 1e-3}

    FakeCPD.__name__ = "LinearGaussianCPD"

    class DAG:
        def topological_order(self):
            return ["a", "b"]

        def parents(self, n):
            return ["a"] if n == "b" else []

        def nodes(self):
            return ["a", "b"]

        def edges(self):
            return [("a", "b")]

    class RefVBN:
        dag = DAG()
        nodes = {"a": FakeCPD(0), "b": FakeCPD(1)}
        device = torch.device("cpu")

    ref = RefVBN()
    m1 = model_from_vbn(ref)
    assert m1.cpds["b"].kind == "linear_gaussian" and m1.parents["b"] == ["a"]
    assert model_from_vbn(ref) is m1                          # cached snapshot
    ref.nodes["b"]._bias.add_(1.0)                            # in-place update -> new snapshot
    m2 = model_from_vbn(ref)
    assert m2 is not m1 and float(m2.cpds["b"].state["_bias"]) == 1.0
    with pytest.raises(RuntimeError, match="MI355X"):
        MonteCarloMarginalization(n_samples=3).infer_posterior(
            ref, Query(target="b", evidence={"a": torch.zeros(2, 1)}))


def test_gibbs_registered_with_yaml_defaults(vbn_cpu):
    """sampling registry key "gibbs" (gibbs.py:12) with vbn/configs/sampling/gibbs.yaml defaults."""
    from vectorizedbayesiannetwork_amd.engines import GibbsSampler
    assert SAMPLING_REGISTRY["gibbs"] is GibbsSampler
    assert defaults.sampling("gibbs") == {"name": "gibbs", "n_samples": 512, "burn_in": 50, "n_steps": 5}
    vbn_cpu.set_sampling_method(defaults.sampling("gibbs"))
    s = vbn_cpu._sampling
    assert (s.n_samples, s.burn_in, s.n_steps, s.n_candidates) == (512, 50, 5, 8)
    g = GibbsSampler()                                   # constructor defaults (gibbs.py:14-16)
    assert (g.n_samples, g.burn_in, g.n_steps) == (200, 10, 1)
    with pytest.raises(RuntimeError, match="MI355X"):    # no CPU fallback
        vbn_cpu.sample({"target": "feature_2", "evidence": {"feature_0": torch.zeros(2, 1)}}, n_samples=4)
