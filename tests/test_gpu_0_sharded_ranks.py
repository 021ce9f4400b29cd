"""Query sharding across processes with the real engines.

Two rank processes (tests/_sharded_worker.py) are started before this process makes any
GPU call (the module sorts first among the GPU tests).  Each runs the HIP engines behind
``ShardedEngine(..., gather=True)`` on its half of a 64-query cfg2 batch: MCM (plain and
with the overlapped gather), IS without fallback, IS whose *last* query -- on rank 1 only --
carries off-manifold evidence, so the batch-global fallback (importance_sampling.py:85-88)
must fire on both ranks through the flag all-reduce, and the ancestral sampler.  Rank 0's
gathered results must equal a single-process run of the whole batch with the same seed bit
for bit (per-query Philox keys use the global query index; shared root draws carry no
query key).  The collectives run over gloo because RCCL does not admit two ranks on one
GPU; the RCCL path is the same code with ``backend="nccl"`` (bench.py --gpus N).
"""
from __future__ import annotations

import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
WORKER = os.path.join(HERE, "_sharded_worker.py")


@pytest.fixture(scope="module")
def rank_results(tmp_path_factory):
    tmp = tmp_path_factory.mktemp("ranks")
    init = "file://" + str(tmp / "store")
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    procs = [subprocess.Popen([sys.executable, "-u", WORKER, "--rank", str(r), "--world", "2", "--init", init,
                               "--out", str(tmp / f"rank{r}.pt")], env=env) for r in range(2)]
    rcs = []
    for p in procs:
        try:
            rcs.append(p.wait(timeout=300))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert rcs == [0, 0], f"rank processes exited with {rcs}"
    return [torch.load(tmp / f"rank{r}.pt", weights_only=True) for r in range(2)]


def _reference(name, seed):
    sys.path.insert(0, HERE)
    import _sharded_worker as W
    from workloads import synthetic_workload
    from vectorizedbayesiannetwork_amd.engines import AncestralSampler, Query
    model, vbn, target, ev = synthetic_workload("cfg2", W.B, "cuda")
    if name == "ancestral":
        xs = AncestralSampler(n_samples=W.S).sample(vbn, Query(target, {k: v.cuda() for k, v in ev.items()}),
                                                     W.S, seed=seed)
        return None, xs.cpu(), False
    for n, make, query, _ in W.cases(vbn, target, ev):
        if n == name:
            eng = make()
            pdf, xs = eng.infer_posterior(vbn, query, seed=seed)
            torch.cuda.synchronize()
            return pdf.cpu(), xs.cpu(), bool(getattr(eng, "_last_fallback", False))
    raise KeyError(name)


def _reference_big(seed):
    """cfg3 IS over the whole 1536-query batch in one process, auto mode: >= 2^20 particles, so
    the plan-specialised walk (compiled before the timed call if it was not cached)."""
    sys.path.insert(0, HERE)
    import _sharded_worker as W
    from workloads import synthetic_workload
    from vectorizedbayesiannetwork_amd import jit, ops
    from vectorizedbayesiannetwork_amd.engines import ImportanceSampling, Query
    model, vbn, target, ev = synthetic_workload("cfg3", W.B_BIG, "cuda")
    q = Query(target, {k: v.cuda() for k, v in ev.items()})
    ImportanceSampling(n_samples=W.S).infer_posterior(vbn, q, seed=seed)
    jit.wait_pending()
    eng = ImportanceSampling(n_samples=W.S)
    pdf, xs = eng.infer_posterior(vbn, q, seed=seed)
    torch.cuda.synchronize()
    return pdf.cpu(), xs.cpu(), bool(eng._last_fallback), bool(ops.LAST_WALK.get("specialised"))


def test_sharded_interpreter_equals_single_process_specialised(rank_results):
    """The plan-specialised / interpreter choice never changes results: rank halves
    on the interpreter gather to exactly the single-process specialised walk (split-f16 MFMA
    heads included: cfg3 is mdn + softmax_nn)."""
    from vectorizedbayesiannetwork_amd import jit
    r0, r1 = rank_results[0]["is_big_cfg3"], rank_results[1]["is_big_cfg3"]
    assert r0["seeds"] == r1["seeds"] and r1["xs"] is None
    pdf, xs, fb, spec = _reference_big(r0["seeds"][-1])
    assert spec or not jit.enabled(), "the single-process reference did not run the specialised walk"
    assert r0["fallback"] == fb
    assert torch.equal(r0["xs"], xs) and torch.equal(r0["pdf"], pdf)


@pytest.mark.parametrize("name", ["mcm", "mcm_overlap", "is", "is_hot", "ancestral"])
def test_two_ranks_match_single_process(rank_results, name):
    r0, r1 = rank_results[0][name], rank_results[1][name]
    assert r0["seeds"] == r1["seeds"], "ranks must agree on every call's seed"
    assert r1["xs"] is None and r1["pdf"] is None, "results are gathered on rank 0 only"
    assert r0["fallback"] == r1["fallback"]
    pdf, xs, fb = _reference(name, r0["seeds"][-1])
    assert r0["fallback"] == fb == (name == "is_hot"), "the IS fallback is batch-global"
    assert torch.equal(r0["xs"], xs), f"{name}: gathered samples differ from the single-process batch"
    if pdf is not None:
        assert torch.equal(r0["pdf"], pdf), f"{name}: gathered pdf/weights differ from the single-process batch"


def test_precompile_behind_sharded_engine(rank_results):
    """VBN.precompile with a ShardedEngine as the inference method (world 2, one-query dummy
    batch): plans built on each rank with no collective, and the sharded calls after it get the
    same seeds and outputs as without the precompile (the "mcm" case)."""
    r0, r1 = rank_results[0]["mcm_precompiled"], rank_results[1]["mcm_precompiled"]
    assert r0["plans"] >= 1 and r1["plans"] >= 1
    assert r0["seeds"] == r1["seeds"] == rank_results[0]["mcm"]["seeds"]
    assert r1["xs"] is None
    assert torch.equal(r0["xs"], rank_results[0]["mcm"]["xs"])
    assert torch.equal(r0["pdf"], rank_results[0]["mcm"]["pdf"])
