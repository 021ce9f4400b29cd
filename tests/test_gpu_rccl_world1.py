"""The multi-GPU path's RCCL collectives on one GPU.

A one-GPU box cannot hold a world of several RCCL ranks (RCCL refuses two ranks on one GPU;
tests/test_gpu_0_sharded_ranks.py covers two ranks over gloo).  Here a world of ONE rank on the
nccl backend runs ``ShardedEngine(..., force_collectives=True)``: the seed broadcast, the
importance-sampling fallback flag's MAX all-reduce (a device tensor, no host sync) and the
asynchronous gathers into the ``[world, shard, ...]`` buffer all execute as RCCL collectives.
The results must equal the unsharded engines bit for bit with the broadcast seed.
"""
from __future__ import annotations

import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def rccl_results(tmp_path_factory):
    tmp = tmp_path_factory.mktemp("rccl")
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    p = subprocess.run([sys.executable, "-u", os.path.join(HERE, "_rccl_worker.py"), "--init",
                        "file://" + str(tmp / "store"), "--out", str(tmp / "out.pt")], env=env, timeout=300)
    assert p.returncode == 0, f"RCCL worker exited with {p.returncode}"
    return torch.load(tmp / "out.pt", weights_only=True)


@pytest.mark.parametrize("name", ["mcm", "mcm_overlap", "is", "is_hot", "ancestral"])
def test_rccl_world1_matches_unsharded(rccl_results, name):
    sys.path.insert(0, HERE)
    from test_gpu_0_sharded_ranks import _reference
    r = rccl_results[name]
    assert rccl_results["backend"] == "nccl"
    pdf, xs, fb = _reference(name, r["seeds"][-1])
    assert r["fallback"] == fb == (name == "is_hot"), "the fallback flag went through the RCCL all-reduce"
    assert torch.equal(r["xs"], xs)
    if pdf is not None:
        assert torch.equal(r["pdf"], pdf)
