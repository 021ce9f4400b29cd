"""Moment tables of one-feature KDE nodes (plan.kde_moment_table, csrc kde_pass1_moments).

The kernel's pass 1 of a one-feature node evaluates, per chunk, sum_k d^k T[g][c][k] around the
grid centre u_g nearest u = 2 x'.  These CPU checks replay the kernel's float32 arithmetic
(centre choice, centre value, Horner order) on the host and compare the chunk sums with
float64 sums of the exact weights exp2(u y' - |y'|^2) of kde.py:172-177 (softmax of log K_p
up to the per-particle factor the factored form drops): relative error <= 4e-7, the f32
rounding of the table entries and of three FMAs.
"""
import math

import numpy as np
import pytest
import torch

from vectorizedbayesiannetwork_amd import plan as P


def _kernel_sums(tab, u):
    """The kernel's chunk sums for particle u (float32 replay), or None outside the grid."""
    lo, inv, dl = np.float32(tab[0]), np.float32(tab[1]), np.float32(tab[2])
    n = int(tab[3:4].view(np.int32)[0])
    T = tab[4:].reshape(n, P.KDE_CHUNKS, P.KDE_MT_TERMS).astype(np.float32)
    u = np.float32(u)
    gr = np.float32(np.rint(np.float32(np.float32(u - lo) * inv)))
    if not (0 <= gr < n):
        return None
    ug = np.float32(np.float64(gr) * np.float64(dl) + np.float64(lo))     # fmaf(gr, dl, lo)
    d = np.float64(np.float32(u - ug))
    out = []
    for c in range(P.KDE_CHUNKS):
        t = T[int(gr), c].astype(np.float64)
        s = np.float32(t[3] * d + t[2])                                    # fmaf: one rounding
        s = np.float32(np.float64(s) * d + t[1])
        s = np.float32(np.float64(s) * d + t[0])
        out.append(float(s))
    return np.array(out)


def _exact_sums(y, u, m_chunk):
    y64 = np.asarray(y, np.float32).astype(np.float64)
    sq = (y64 * y64).astype(np.float32).astype(np.float64)
    m = y64.size
    out = []
    for c in range(P.KDE_CHUNKS):
        j0, j1 = min(m, c * m_chunk), min(m, (c + 1) * m_chunk)
        out.append(np.exp2(np.float64(np.float32(u)) * y64[j0:j1] - sq[j0:j1]).sum())
    return np.array(out)


@pytest.mark.parametrize("m,sd", [(10000, 0.36), (4096, 0.6), (100, 0.3), (17, 1.0), (1, 0.5)])
def test_moment_chunk_sums_match_exact(m, sd):
    rng = np.random.default_rng(m)
    y = (rng.standard_normal(m) * sd).astype(np.float32)
    mc = P._kde_cb(m) * 16
    tab = P.kde_moment_table(y, mc)
    assert tab is not None
    lo, dl = float(tab[0]), float(tab[2])
    n = int(tab[3:4].view(np.int32)[0])
    hi = lo + (n - 1) * dl
    # the covered range holds the data range with margin on both sides
    assert lo <= 2 * (float(y.min()) - 1.9) and hi >= 2 * (float(y.max()) + 1.9)
    us = np.concatenate([rng.uniform(lo, hi, 300), [lo, hi, 0.0, 2 * float(y.max()), 2 * float(y.min())]])
    worst = 0.0
    for u in us:
        got = _kernel_sums(tab, u)
        if got is None:
            continue
        ref = _exact_sums(y, u, mc)
        mask = ref > 0
        assert np.all(got[~mask] == 0)
        worst = max(worst, float(np.max(np.abs(got[mask] - ref[mask]) / ref[mask])))
    assert worst <= 4e-7, worst
    # outside the grid the kernel takes the MFMA pass
    assert _kernel_sums(tab, lo - 10 * dl) is None and _kernel_sums(tab, hi + 10 * dl) is None
    assert _kernel_sums(tab, float("nan")) is None


def test_moment_series_bound():
    """KDE_MT_Z bounds |d| ln2 |y'| at a cell edge: the truncated series' relative error."""
    z = P.KDE_MT_Z
    assert z ** P.KDE_MT_TERMS / math.factorial(P.KDE_MT_TERMS) * math.exp(z) < 3e-8


def test_moment_table_declines_wide_data():
    """Weights beyond [2^-80, 2^100] on the covered range: no table (the MFMA pass runs)."""
    y = (np.random.default_rng(0).standard_normal(2000) * 3.0 * 1.2).astype(np.float32)
    assert P.kde_moment_table(y, P._kde_cb(2000) * 16) is None


def test_cfg4_one_feature_steps_carry_tables():
    """The packed cfg4 model (reference-fitted, M = 10,000): every one-parent KDE node has a
    moment table (step reserved[7] = its blob offset), every other node -1; the table's sums
    match the exact ones at the node's own data points."""
    import bench
    cfg, model, target, ev = bench.build_model("cfg4")
    pk = P.PackedModel(model, torch.device("cpu"))
    n1 = 0
    for n in model.topo:
        npk = pk.nodes[n]
        if npk.kind != P.KIND_ID["kde"]:
            continue
        if npk.aux0 == 1:
            assert "kmt" in npk.offs, n
            n1 += 1
        else:
            assert "kmt" not in npk.offs, n
    assert n1 == sum(1 for n in model.topo if len(model.parents[n]) == 1)
    node = next(n for n in model.topo if len(model.parents[n]) == 1)
    npk = pk.nodes[node]
    blob = pk.params.cpu().numpy()
    m = npk.k
    n_cells = int(blob[npk.offs["kmt"] + 3:npk.offs["kmt"] + 4].view(np.int32)[0])
    tab = blob[npk.offs["kmt"]:npk.offs["kmt"] + 4 + n_cells * P.KDE_CHUNKS * P.KDE_MT_TERMS]
    c_p = np.float32(P._KDE_C / (max(float(model.cpds[node].hparams["parent_bandwidth"]), 1e-3)
                                 + float(model.cpds[node].hparams["min_scale"])))
    y = (model.cpds[node].extra["parents"].float().numpy() * c_p).reshape(-1)
    for x in model.cpds[node].extra["parents"].float().numpy()[:20, 0]:
        u = np.float32(2.0) * (c_p * np.float32(x))
        got, ref = _kernel_sums(tab, u), _exact_sums(y, u, P._kde_cb(m) * 16)
        assert np.max(np.abs(got - ref) / ref) <= 4e-7
    # plan rows: reserved[7] holds the offset for that node, -1 elsewhere
    plan = P.build_plan(pk, latent=[n for n in model.topo if n not in ev], fixed=[n for n in model.topo if n in ev],
                        out_nodes=[target], logp=[target], skip=[], shared_roots=True, mode=P.MODE_MCM)
    rows = plan.steps._vbn_host[0]
    for r in rows:
        if r[P.S_KIND] == P.KIND_ID["kde"] and r[P.S_AUX0] == 1:
            assert r[P.S_RES7] > 0
        else:
            assert r[P.S_RES7] == -1
