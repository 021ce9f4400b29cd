"""Walk orders other than the model's (plan.liveness_order, engines._plan): host checks.

The liveness order is a topological order that keeps fewer node values live, so a wave needs
fewer LDS slots; engines use it only where the plan's LDS bounds the waves per CU (cfg5's
128-node DAG: 32 -> 25 slots with the greedy, 24 after seeded restarts: 13 -> 16 waves per CU).  Draws are keyed by node, so the order
changes only the slot assignment and which normals share a Box-Muller pair; the host replica of
the draws (tests/philox_draws.py) pairs by the step table, so the oracle comparisons of the GPU
tests hold for any order.
"""
import numpy as np
import pytest
import torch

from philox_draws import F_BM_FIRST, F_BM_SECOND, F_SHARED, PhiloxDraws
from workloads import synthetic_workload
from vectorizedbayesiannetwork_amd import engines as E
from vectorizedbayesiannetwork_amd.plan import (MODE_MCM, MODE_SAMPLE, MODE_WEIGHTED, S_FLAGS, S_NODEID,
                                                build_plan, liveness_order)


def _mcm_plan(cfg, order=None):
    model, vbn, target, ev = synthetic_workload(cfg, 2, "cpu")
    pk = E.packed_model(vbn, torch.device("cpu"))
    vals = set(ev)
    kw = dict(latent=[x for x in model.topo if x not in vals], fixed=[x for x in model.topo if x in vals],
              logp=[target], out_nodes=[target], shared_roots=True, mode=MODE_MCM)
    if order == "liveness":
        order = liveness_order(model, fixed=kw["fixed"], logp=kw["logp"], out_nodes=kw["out_nodes"])
    return model, pk, build_plan(pk, order=order, **kw), kw


@pytest.mark.parametrize("cfg", ["cfg2", "cfg3", "cfg4", "cfg5"])
def test_liveness_order_is_topological_and_never_worse(cfg):
    model, pk, base, _ = _mcm_plan(cfg)
    _, _, lv, _ = _mcm_plan(cfg, "liveness")
    seen = set()
    for n in lv.order:
        assert all(p in seen for p in model.parents[n]), n
        seen.add(n)
    assert sorted(lv.order) == sorted(model.topo)
    assert lv.n_slots <= base.n_slots
    if cfg == "cfg5":
        assert (base.n_slots, lv.n_slots) == (32, 25)


def test_engine_uses_liveness_order_only_when_lds_bound():
    for cfg, reordered in (("cfg2", False), ("cfg5", True)):
        model, pk, base, kw = _mcm_plan(cfg)
        p = E._plan(pk, ("test-order", cfg), **kw)                # not an ordered key: model order
        assert p.order == list(model.topo)
        p = E._plan(pk, ("mcm", cfg, "test"), **kw)
        assert (p.order != list(model.topo)) == reordered
        assert E._lds_bound(base) == reordered
        if reordered:                    # the restarted greedy ends the bound: 16 waves per CU
            assert p.n_slots == 24 and not E._lds_bound(p)


def test_box_muller_pairs_follow_the_table():
    """every SECOND step's partner is the nearest FIRST step before it in the table, with the same
    shared flag, and the replica pairs them so whatever order the oracle calls the nodes in"""
    model, pk, lv, _ = _mcm_plan("cfg5", "liveness")
    rows = lv.steps._vbn_host[0]
    first = None
    pairs = 0
    for r in rows:
        fl = int(r[S_FLAGS])
        if fl & F_BM_FIRST:
            assert first is None
            first = r
        elif fl & F_BM_SECOND:
            assert first is not None and (int(first[S_FLAGS]) & F_SHARED) == (fl & F_SHARED)
            first = None
            pairs += 1
    assert pairs > 10
    d = PhiloxDraws(lv.steps, pk.node_id, seed=123, n_queries=1, n_samples=64)
    name_of = {v: k for k, v in pk.node_id.items()}
    for r in rows:
        if int(r[S_FLAGS]) & F_BM_SECOND:
            part = d.partner[int(r[S_NODEID])]
            # the partner's r sin(2 pi u2) is this node's dim-0 normal
            d.begin_node(name_of[int(part[S_NODEID])])
            a = d.normal((1, 64, 1))
            d.begin_node(name_of[int(r[S_NODEID])])
            b = d.normal((1, 64, 1))
            assert torch.isfinite(a).all() and torch.isfinite(b).all()
            assert not torch.equal(a, b)
            q = np.zeros(64, np.int64)
            s = np.arange(64)
            w0, w1 = d._words(q, s, np.zeros(64, np.int64), 0, row=part)
            from philox_draws import box_muller_pair
            assert torch.equal(b.reshape(-1), torch.from_numpy(box_muller_pair(w0, w1)[1]))
            break


def test_lds_bound_counts_staged_weight_buffers():
    """a gaussian_nn plan whose value slots alone fit 16 waves per CU but whose two
    staged weight buffers (walk_shape in csrc/vbn_walk.hip) do not is LDS-bound; the same plan
    in an unstaged kind set (a KDE node) is not."""
    from types import SimpleNamespace
    from vectorizedbayesiannetwork_amd import engines as E
    p = SimpleNamespace(n_slots=20, max_out=2, kind_mask=1, wbuf=8192)
    assert (p.n_slots + p.max_out) * 64 * 4 * 16 <= 160 * 1024          # slots alone: 16 waves
    assert E._resident_waves(p) == 4 and E._lds_bound(p)                # 2 x 32 KiB per workgroup
    p.wbuf = 256
    assert E._resident_waves(p) == 16 and not E._lds_bound(p)
    p.kind_mask, p.wbuf = 1 | 8, 8192                                   # kde: weights read from the blob
    assert E._resident_waves(p) == 16 and not E._lds_bound(p)
