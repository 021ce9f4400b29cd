"""vbn_hip::pack_plan (ops.py) on CPU: the packed blob of a plan with its
precompute variant and pre-passes unpacks to the same step tables, slot lists and launch
metadata, and malformed blobs are refused."""
import numpy as np
import pytest
import torch

from vectorizedbayesiannetwork_amd import ops
from vectorizedbayesiannetwork_amd import plan as P


def _sections(cfg_name="cfg2"):
    import bench
    cfg, model, target, ev = bench.build_model(cfg_name)
    pk = P.PackedModel(model, torch.device("cpu"))
    vals = set(ev)
    plan = P.build_plan(pk, latent=[x for x in model.topo if x not in vals],
                        fixed=[x for x in model.topo if x in vals], logp=[target], out_nodes=[target],
                        shared_roots=True, mode=P.MODE_MCM)
    pc, pre, pre_q = P.precompute_plans(pk, plan)
    return pk, [plan, pc, pre, pre_q]


def _pack(pk, secs):
    steps, ics, ocs, meta = [], [], [], []
    for p in secs:
        if p is None:
            e = torch.zeros(0, dtype=torch.int32)
            steps.append(e), ics.append(e), ocs.append(e)
            meta += [0] * 8
            continue
        steps.append(torch.from_numpy(p.steps._vbn_host[0]))
        ics.append(torch.from_numpy(p.steps._vbn_host[1]))
        ocs.append(p.out_cols.cpu())
        meta += [p.n_slots, p.max_out, p.fixed_ld, p.mode, p.kind_mask, p.wbuf, pk.dmax, len(p.noise_nodes)]
    return ops.pack_plan(steps, ics, ocs, meta)


@pytest.mark.parametrize("cfg_name", ["cfg2", "cfg5"])
def test_pack_unpack_round_trip(cfg_name):
    pk, secs = _sections(cfg_name)
    blob = _pack(pk, secs)
    assert blob.dtype == torch.int32 and blob.dim() == 1 and int(blob[0]) == ops.PLAN_MAGIC
    got = ops._unpack(blob, torch.device("cpu"))
    for p, g in zip(secs, got):
        if p is None:
            assert g is None
            continue
        st, ic, oc, h = g
        assert np.array_equal(st.numpy(), p.steps._vbn_host[0])
        assert np.array_equal(ic.numpy()[:p.steps._vbn_host[1].size], p.steps._vbn_host[1])
        assert np.array_equal(oc.numpy(), p.out_cols.numpy())
        assert h[4:12] == [p.n_slots, p.max_out, p.fixed_ld, p.mode, p.kind_mask, p.wbuf, pk.dmax,
                           len(p.noise_nodes)]
        assert st._vbn_wblk_max == p.steps._vbn_wblk_max
        assert st._vbn_host[2] == p.steps._vbn_host[2]          # same plan-cache key as the engines'
        for attr in ("_vbn_precomp_stride", "_vbn_precomp_q_stride"):
            assert getattr(st, attr, None) == getattr(p.steps, attr, None)


def test_pack_refuses_malformed_blobs():
    pk, secs = _sections()
    blob = _pack(pk, secs)
    with pytest.raises(ValueError):
        ops._unpack(blob[:3].clone(), torch.device("cpu"))
    bad = blob.clone()
    bad[0] = 7
    with pytest.raises(ValueError):
        ops._unpack(bad, torch.device("cpu"))
    with pytest.raises(ValueError):
        ops._unpack(blob.to(torch.int64), torch.device("cpu"))
    with pytest.raises(ValueError):
        ops.pack_plan([torch.zeros(0, dtype=torch.int32)], [], [], [])
