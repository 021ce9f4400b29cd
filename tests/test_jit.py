"""Plan-specialised walks (vectorizedbayesiannetwork_amd/jit.py) on the CPU host: the
generated translation unit compiles for gfx950 with hiprtc (no GPU needed), the cache key
names the exact step table, and the launch layer only specialises lean full-wave walks."""
import os

import numpy as np
import pytest

from vectorizedbayesiannetwork_amd import jit, synthetic
from vectorizedbayesiannetwork_amd.model import random_init_model
from vectorizedbayesiannetwork_amd.plan import MODE_MCM, PackedModel, build_plan


def _plan():
    g = synthetic.random_dag(6, seed=3)
    data = synthetic.sem_data(g, 256, seed=0)
    model = random_init_model(g, synthetic.round_robin_kinds(g, ["gaussian_nn", "linear_gaussian"]), data, seed=0)
    pk = PackedModel(model, "cpu")
    topo = model.topo
    return build_plan(pk, latent=list(topo), fixed=[], logp=[topo[-1]], out_nodes=[topo[-1]], shared_roots=True,
                      mode=MODE_MCM)


def test_plan_carries_host_copy_and_key():
    plan = _plan()
    steps, ic, key = plan.steps._vbn_host
    assert np.array_equal(steps, plan.steps.numpy()) and np.array_equal(ic, plan.in_cols.numpy())
    assert key == _plan().steps._vbn_host[2]                      # deterministic
    src = jit.plan_source(steps, ic, 131)
    assert f"#define VBN_PLAN_N_STEPS {len(steps)}" in src and "vbn_walk_plan_body<131u>" in src


@pytest.mark.skipif(not os.path.exists("/opt/rocm/lib/libhiprtc.so"), reason="hiprtc not installed")
def test_plan_source_compiles_with_hiprtc(tmp_path, monkeypatch):
    monkeypatch.setenv("VBN_HIP_CACHE", str(tmp_path))
    plan = _plan()
    steps, ic, _ = plan.steps._vbn_host
    key, code = jit.code_object(steps, ic, 131)                      # gaussian_nn + linear_gaussian, lean
    assert code[:4] == b"\x7fELF" and len(code) > 1000              # an AMDGPU code object
    assert (tmp_path / f"{key}.hsaco").exists()
    key2, code2 = jit.code_object(steps, ic, 131)                    # from the disk cache
    assert key2 == key and code2 == code
