"""Per-sample and per-query precompute (plan.precompute_plans) on CPU: which nodes qualify,
that the per-sample pre-pass draws exactly the main walk's root values (same root rows, same
Box-Muller pairs), and that the per-query pre-pass reads the main walk's fixed-buffer layout."""
import numpy as np
import pytest
import torch

from vectorizedbayesiannetwork_amd import plan as P

NN_KDE = ("gaussian_nn", "mdn", "softmax_nn", "kde")


def _plan(cfg_name, engine="mcm"):
    import bench
    cfg, model, target, ev = bench.build_model(cfg_name)
    pk = P.PackedModel(model, torch.device("cpu"))
    vals = set(ev)
    latent = [x for x in model.topo if x not in vals]
    fixed = [x for x in model.topo if x in vals]
    if engine == "mcm":
        plan = P.build_plan(pk, latent=latent, fixed=fixed, logp=[target], out_nodes=[target],
                            shared_roots=True, mode=P.MODE_MCM)
    else:                                                    # IS (per-query roots) / LW (shared)
        plan = P.build_plan(pk, latent=latent, fixed=fixed, logp=fixed, out_nodes=[target],
                            shared_roots=engine == "lw", mode=P.MODE_WEIGHTED)
    return model, pk, plan, vals


def _want(model, vals, plan, shared):
    """nodes the precompute must mark: per sample (parents all shared latent roots) and per
    query (parents all evidence); NN kinds latent or evidence with a log-prob, KDE latent
    without a moment table (a table makes the chunk sums cheap in the walk itself)"""
    rows = plan.steps._vbn_host[0]
    roots = {n for n in model.topo if not model.parents[n] and n not in vals} if shared else set()
    ws, wq = set(), set()
    for i, n in enumerate(model.topo):
        kind = model.cpds[n].kind
        if not model.parents[n] or kind not in NN_KDE or (kind == "kde" and rows[i][P.S_RES7] >= 0):
            continue
        latent = n not in vals
        if not latent and not (kind != "kde" and rows[i][P.S_FLAGS] & P.F_LOGP):
            continue
        if all(p in roots for p in model.parents[n]):
            ws.add(n)
        if all(p in vals for p in model.parents[n]):
            wq.add(n)
    # an evidence node some other candidate reads keeps its value slot (stays per particle)
    wq = {n for n in wq if not (n in vals and any(n in model.parents[m] for m in wq))}
    return ws, wq


def _check_cols(model, pk, rows, nodes, stride, width=None):
    cols = []
    for i, n in enumerate(model.topo):
        if n not in nodes:
            continue
        r = rows[i]
        assert r[P.S_AUX2] >> 16 == stride
        w = P.KDE_CHUNKS + 1 if model.cpds[n].kind == "kde" else int(r[P.S_NOUT])
        assert w == P.precompute_width(pk, n) > 0
        cols.append((r[P.S_AUX2] & 0xFFFF, w))
        assert r[P.S_WBLK_LEN] == 0                          # no MLP runs: nothing to stage
    cols.sort()
    assert cols[0][0] == 0 and all(a + w == c for (a, w), (c, _) in zip(cols, cols[1:]))
    assert cols[-1][0] + cols[-1][1] == (stride if width is None else width)


@pytest.mark.parametrize("cfg_name,engine", [("cfg2", "mcm"), ("cfg4", "mcm"), ("cfg5", "mcm"), ("anchor64", "mcm"),
                                             ("cfg2", "is"), ("cfg3", "is"), ("cfg3", "lw"), ("cfg5", "lw")])
def test_precompute_marks_nodes(cfg_name, engine):
    model, pk, plan, vals = _plan(cfg_name, engine)
    shared = engine != "is"
    want_s, want_q = _want(model, vals, plan, shared)
    assert want_q, "every §8(d) query has nodes whose parents are all evidence"
    pc, pre, pre_q = P.precompute_plans(pk, plan)
    base, rows = plan.steps._vbn_host[0], pc.steps._vbn_host[0]
    got_s = {n for i, n in enumerate(model.topo) if rows[i][P.S_FLAGS] & P.F_PRECOMP
             and not rows[i][P.S_FLAGS] & P.F_PRECOMP_Q}
    got_q = {n for i, n in enumerate(model.topo) if rows[i][P.S_FLAGS] & P.F_PRECOMP_Q}
    assert got_s == want_s and got_q == want_q
    assert all(rows[i][P.S_FLAGS] & P.F_PRECOMP for i, n in enumerate(model.topo) if n in got_q)
    for i, n in enumerate(model.topo):
        diff = np.nonzero(rows[i] != base[i])[0].tolist()
        if n in got_s | got_q:
            assert set(diff) <= {P.S_FLAGS, P.S_AUX2, P.S_WBLK_OFF, P.S_WBLK_LEN}
        else:
            assert diff == []                                # every other step unchanged
    if got_s:
        assert pc.steps._vbn_precomp_stride == pre.out_cols.numel()
        _check_cols(model, pk, rows, got_s, pc.steps._vbn_precomp_stride)
        # the per-sample pre-pass: every latent root with the main walk's row flags
        roots = {n for n in model.topo if not model.parents[n] and n not in vals}
        prow = pre.steps._vbn_host[0]
        porder = [n for n in model.topo if n in roots | got_s]
        assert len(porder) == len(prow)
        for i, n in enumerate(porder):
            r = prow[i]
            if n in roots:
                b = base[model.topo.index(n)]
                assert r[P.S_ROLE] == P.ROLE_LATENT and r[P.S_FLAGS] == b[P.S_FLAGS]
                assert r[P.S_NODEID] == b[P.S_NODEID]
            else:
                assert not r[P.S_FLAGS] & (P.F_BM_FIRST | P.F_BM_SECOND)
                assert r[P.S_ROLE] == P.ROLE_LATENT and r[P.S_FLAGS] & P.F_PRE_OUT
    else:
        assert pre is None and not hasattr(pc.steps, "_vbn_precomp_stride")
    # the per-query pre-pass: the main walk's fixed steps (same fixed-buffer columns), then the
    # candidates writing their quantities
    # the walk reads row 64 b of the pre-pass's [B * 64, w] out_x in place: stride 64 w
    stride_q = pc.steps._vbn_precomp_q_stride
    assert stride_q == 64 * pre_q.out_cols.numel()
    _check_cols(model, pk, rows, got_q, stride_q, width=pre_q.out_cols.numel())
    assert pre_q.fixed_nodes == plan.fixed_nodes and pre_q.fixed_ld == plan.fixed_ld
    qrow = pre_q.steps._vbn_host[0]
    qorder = [n for n in model.topo if n in vals or n in got_q]
    assert len(qorder) == len(qrow)
    for i, n in enumerate(qorder):
        r = qrow[i]
        if n in vals and n not in got_q:
            assert r[P.S_ROLE] == P.ROLE_FIXED and not r[P.S_FLAGS] & P.F_LOGP
            assert r[P.S_FIXEDCOL] == base[model.topo.index(n)][P.S_FIXEDCOL]
        else:
            assert r[P.S_ROLE] == P.ROLE_LATENT and r[P.S_FLAGS] & P.F_PRE_OUT
            assert not r[P.S_FLAGS] & (P.F_BM_FIRST | P.F_BM_SECOND)


def test_is_has_no_per_sample_precompute():
    model, pk, plan, vals = _plan("cfg2", "is")                 # IS: per-query root draws
    pc, pre, pre_q = P.precompute_plans(pk, plan)
    assert pre is None and pre_q is not None


def test_side_stream_only_for_kde_per_sample_prepasses(monkeypatch):
    """engines._pre_side: the per-sample pre-pass goes on a side stream when it has KDE nodes
    (cfg4 / cfg5: long, latency-bound) and stays on the main stream for NN-only ones (cfg2 /
    anchor64); VBN_PRE_STREAM forces either way."""
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
    import precompile_plans as PP
    from vectorizedbayesiannetwork_amd import engines as E
    want = {"cfg2": False, "anchor64": False, "cfg4": True, "cfg5": True}
    for cfg, side in want.items():
        plan = PP.plans_for(cfg)[1][0][1]
        assert plan.pre is not None and plan.pre_q is not None
        monkeypatch.setattr(E, "PRE_SIDE_STREAM", None)
        plan.__dict__.pop("_pre_has_kde", None)
        assert E._pre_side(plan) == side, cfg
        for forced in (True, False):
            monkeypatch.setattr(E, "PRE_SIDE_STREAM", forced)
            assert E._pre_side(plan) == forced
