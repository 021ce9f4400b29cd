"""Model import: reference checkpoint format (vbn.py:644-824) and random-init builder."""
import pytest
import torch

from conftest import golden_names, load_golden
from vectorizedbayesiannetwork_amd import synthetic
from vectorizedbayesiannetwork_amd.model import CPD_KINDS, model_from_checkpoint, random_init_model


@pytest.mark.parametrize("name", golden_names())
def test_checkpoint_dicts_import(name):
    ck = load_golden(name)["model"]
    m = model_from_checkpoint(ck)
    assert m.topo == ck["dag"]["topological_order"]
    for node, rec in m.cpds.items():
        assert rec.kind in CPD_KINDS
        assert rec.input_dim == sum(m.out_dim(p) for p in m.parents[node])
        if rec.kind == "kde":
            assert rec.extra["targets"].shape[0] > 0


def test_checkpoint_file_roundtrip(tmp_path):
    ck = load_golden("mix12")["model"]
    path = tmp_path / "model.pt"
    torch.save(ck, path)
    from vectorizedbayesiannetwork_amd.model import load_checkpoint
    m = model_from_checkpoint(load_checkpoint(str(path)))
    assert set(m.cpds) == set(ck["nodes"])


def test_unsupported_cpd_is_rejected():
    ck = load_golden("readme")["model"]
    bad = dict(ck)
    bad["nodes"] = dict(ck["nodes"])
    node = next(iter(bad["nodes"]))
    bad["nodes"][node] = dict(bad["nodes"][node], cpd_key="categorical_table")
    with pytest.raises(ValueError, match="not on the accelerated path"):
        model_from_checkpoint(bad)


def test_synthetic_generator_matches_survey_spec():
    g = synthetic.random_dag(32, seed=0)
    assert len(g.nodes) == 32
    indeg = sum(d for _, d in g.in_degree()) / 32
    assert abs(indeg - 1.44) < 0.05                          # 1.44 for N=32
    target, ev = synthetic.default_query_nodes(g, seed=1)
    assert len(ev) == 8 and target not in ev
    data = synthetic.sem_data(g, 100)
    m = random_init_model(g, synthetic.round_robin_kinds(g, ["gaussian_nn"]), data)
    assert all(r.kind == "gaussian_nn" for r in m.cpds.values())
