"""Model I/O in the reference checkpoint format (reference vbn/vbn.py:644-824).

* ``VBN.save`` writes what the reference's ``save`` writes (same keys per node, ``_extra_state``
  inside every state_dict, ``meta.json`` for directory paths), loadable with
  ``torch.load(weights_only=True)``; loading it back gives the same model.
* When the reference is importable (this container, not the GPU box) its own ``VBN.load``
  reads our file and its CPDs produce the same log-probabilities as the reference model the
  fixture was recorded from, and a random-init model (bench.py's synthetic workloads)
  round-trips through the reference's strict ``load_state_dict``.
"""
import json
import os
import sys

import pytest
import torch

from conftest import golden_names, load_golden
from vectorizedbayesiannetwork_amd import VBN, synthetic
from vectorizedbayesiannetwork_amd.model import model_from_checkpoint, random_init_model

REF = os.environ.get("VBN_REFERENCE", "/root/reference")
HAVE_REF = os.path.isdir(os.path.join(REF, "vbn"))


def _same_state(a, b):
    assert set(a) == set(b)
    for k in a:
        if isinstance(a[k], torch.Tensor):
            assert torch.equal(a[k], b[k]), k
        else:
            assert a[k] == b[k], k


@pytest.mark.parametrize("name", golden_names())
def test_save_round_trip(tmp_path, name):
    fx = load_golden(name)
    model = model_from_checkpoint(fx["model"])
    vbn = VBN.from_model(model, device="cpu", seed=0)
    vbn.set_inference_method("importance_sampling", n_samples=64)
    path = tmp_path / "m.pt"
    vbn.save(str(path))
    ck = torch.load(path, weights_only=True)
    assert set(ck) == {"dag", "nodes", "meta", "extra", "config"}
    assert ck["config"]["inference"] == {"name": "importance_sampling", "params": {"n_samples": 64}}
    assert list(ck["nodes"]) == list(model.topo)
    ref_nodes = fx["model"]["nodes"]
    for node, info in ck["nodes"].items():
        r = ref_nodes[node]
        assert {k for k in info} == {"cpd_key", "class_name", "input_dim", "output_dim", "seed", "init_kwargs",
                                     "state_dict", "extra_state"}
        for k in ("cpd_key", "class_name", "input_dim", "output_dim"):
            assert info[k] == r[k], (node, k)
        assert set(info["state_dict"]) == set(r["state_dict"]), node     # incl. _extra_state
        assert info["init_kwargs"] == r["init_kwargs"], node
    back = model_from_checkpoint(ck)
    assert back.topo == model.topo and back.parents == model.parents
    for node in model.topo:
        _same_state(back.cpds[node].state, model.cpds[node].state)
        assert back.cpds[node].hparams == model.cpds[node].hparams
        if model.cpds[node].extra:
            _same_state(back.cpds[node].extra, model.cpds[node].extra)
    d = tmp_path / "dir"
    vbn.save(str(d))
    meta = json.loads((d / "meta.json").read_text())
    assert meta["nodes"] == {n: {"cpd_key": model.cpds[n].kind} for n in model.topo}
    assert torch.load(d / "checkpoint.pt", weights_only=True)["dag"] == ck["dag"]


@pytest.fixture(scope="module")
def ref_vbn():
    if not HAVE_REF:
        pytest.skip("reference not present (GPU box)")
    sys.path.insert(0, REF)
    os.environ.setdefault("CI", "1")
    import vbn
    return vbn


@pytest.mark.parametrize("name", ["readme", "mix12", "variants", "family_kde", "family_softmax_nn"])
def test_reference_loads_our_checkpoint(tmp_path, ref_vbn, name):
    fx = load_golden(name)
    model = model_from_checkpoint(fx["model"])
    ours = tmp_path / "ours.pt"
    VBN.from_model(model, device="cpu", seed=0).save(str(ours))
    theirs = tmp_path / "theirs.pt"
    torch.save(fx["model"], theirs)
    a = ref_vbn.VBN.load(str(ours), map_location="cpu")
    b = ref_vbn.VBN.load(str(theirs), map_location="cpu")
    g = torch.Generator().manual_seed(0)
    for node in model.topo:
        d_in = model.cpds[node].input_dim
        par = torch.randn(5, d_in, generator=g) if d_in else None
        x = torch.randn(5, model.out_dim(node), generator=g)
        rec = model.cpds[node]
        if rec.kind == "softmax_nn" and bool(rec.state["_is_discrete"].any()):
            cv = rec.state["_class_values"]                        # discrete dims take class values
            x = torch.stack([cv[d, torch.randint(0, cv.shape[1], (5,), generator=g)]
                             for d in range(cv.shape[0])], dim=1)
        with torch.no_grad():
            la, lb = a.nodes[node].log_prob(x, par), b.nodes[node].log_prob(x, par)
        assert torch.equal(la, lb), node


@pytest.mark.parametrize("cfg_name", ["cfg2", "cfg3", "cfg5"])
def test_random_init_models_load_in_the_reference(tmp_path, ref_vbn, cfg_name):
    cfg = dict(synthetic.CONFIGS[cfg_name])
    g = synthetic.random_dag(min(cfg["n_nodes"], 24), seed=0)
    data = synthetic.sem_data(g, 512, seed=0)
    model = random_init_model(g, synthetic.round_robin_kinds(g, cfg["kinds"]), data, seed=0,
                              overrides={"kde": {"max_points": 256}})
    p = tmp_path / "m.pt"
    VBN.from_model(model, device="cpu").save(str(p))
    r = ref_vbn.VBN.load(str(p), map_location="cpu")          # strict load_state_dict per CPD
    assert list(r.dag.topological_order()) == model.topo
