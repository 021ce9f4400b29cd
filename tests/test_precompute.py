"""Shared-sample precompute (plan.precompute_plans) on CPU: which nodes qualify, and that the
pre-pass draws exactly the main walk's root values (same root rows, same Box-Muller pairs)."""
import numpy as np
import pytest
import torch

from vectorizedbayesiannetwork_amd import plan as P


def _mcm(cfg_name):
    import bench
    cfg, model, target, ev = bench.build_model(cfg_name)
    pk = P.PackedModel(model, torch.device("cpu"))
    vals = set(ev)
    plan = P.build_plan(pk, latent=[x for x in model.topo if x not in vals],
                        fixed=[x for x in model.topo if x in vals], logp=[target], out_nodes=[target],
                        shared_roots=True, mode=P.MODE_MCM)
    return model, pk, plan, vals


@pytest.mark.parametrize("cfg_name", ["cfg2", "cfg4", "cfg5", "anchor64"])
def test_precompute_marks_nodes_with_shared_root_parents(cfg_name):
    model, pk, plan, vals = _mcm(cfg_name)
    pc, pre = P.precompute_plans(pk, plan)
    base, rows = plan.steps._vbn_host[0], pc.steps._vbn_host[0]
    roots = {n for n in model.topo if not model.parents[n] and n not in vals}
    want = {n for n in model.topo if n not in vals and model.parents[n]
            and all(p in roots for p in model.parents[n])
            and model.cpds[n].kind in ("gaussian_nn", "mdn", "softmax_nn", "kde")}
    got = {n for i, n in enumerate(model.topo) if rows[i][P.S_FLAGS] & P.F_PRECOMP}
    assert got == want and got
    stride = pc.steps._vbn_precomp_stride
    assert stride == pre.out_cols.numel()
    cols = []
    for i, n in enumerate(model.topo):
        r, b = rows[i], base[i]
        diff = np.nonzero(r != b)[0].tolist()
        if n not in got:
            assert diff == []                                # every other step unchanged
            continue
        assert P.precompute_width(pk, n) > 0
        assert set(diff) <= {P.S_FLAGS, P.S_AUX2, P.S_WBLK_OFF, P.S_WBLK_LEN}
        assert r[P.S_AUX2] >> 16 == stride
        w = P.KDE_CHUNKS + 1 if model.cpds[n].kind == "kde" else int(r[P.S_NOUT])
        assert w == P.precompute_width(pk, n)
        cols.append((r[P.S_AUX2] & 0xFFFF, w))
        assert r[P.S_WBLK_LEN] == 0                          # no MLP runs: nothing to stage
    cols.sort()
    assert cols[0][0] == 0 and all(a + w == c for (a, w), (c, _) in zip(cols, cols[1:]))
    assert cols[-1][0] + cols[-1][1] == stride
    # the pre-pass: every latent root with the main walk's row flags (same draws, same pairs)
    prow = pre.steps._vbn_host[0]
    porder = [n for n in model.topo if n in roots | got]
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


def test_no_precompute_without_shared_roots():
    import bench
    cfg, model, target, ev = bench.build_model("cfg2")
    pk = P.PackedModel(model, torch.device("cpu"))
    vals = set(ev)
    plan = P.build_plan(pk, latent=[x for x in model.topo if x not in vals],
                        fixed=[x for x in model.topo if x in vals], logp=list(vals), out_nodes=[target],
                        shared_roots=False, mode=P.MODE_WEIGHTED)
    assert P.precompute_plans(pk, plan) is None             # IS: per-query root draws
