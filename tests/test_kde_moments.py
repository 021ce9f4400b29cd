"""Moment tables of one-feature KDE nodes (plan.kde_moment_table, csrc kde_index_moments).

The kernel's sampling step of a one-feature node evaluates, per table row (chunk of ~M/64
points, group of 8 chunks, whole set), sum_k d^k T[g][row][k] around the grid centre u_g nearest
u = 2 x', locates the group and then the chunk holding u_cat * total, and scans that chunk.
These CPU checks replay the kernel's float32 arithmetic (centre choice, centre value, Horner
order) and compare the row sums with float64 sums of the exact weights exp2(u y' - |y'|^2) of
kde.py:172-177 (softmax of log K_p up to the per-particle factor the factored form drops):
relative error <= 4e-7, the f32 rounding of the table entries and of three FMAs; and the
located index with the exact inverse-CDF index (differing only at near-ties).
"""
import math

import numpy as np
import pytest
import torch

from vectorizedbayesiannetwork_amd import plan as P


def _table(tab):
    lo, inv, dl = np.float32(tab[0]), np.float32(tab[1]), np.float32(tab[2])
    n, nch, per = (int(v) for v in tab[3:6].view(np.int32))
    rows = P.kde_moment_rows(nch)
    T = tab[P.KDE_MT_HEADER:].reshape(n, rows, P.KDE_MT_TERMS).astype(np.float32)
    return lo, inv, dl, n, nch, per, T


def _kernel_rows(tab, u):
    """The kernel's float32 sums of every row of u's cell (chunks, groups, total), or None
    outside the grid."""
    lo, inv, dl, n, nch, per, T = _table(tab)
    u = np.float32(u)
    gr = np.float32(np.rint(np.float32(np.float32(u - lo) * inv)))
    if not (0 <= gr < n):
        return None
    ug = np.float32(np.float64(gr) * np.float64(dl) + np.float64(lo))     # fmaf(gr, dl, lo)
    d = np.float64(np.float32(u - ug))
    t = T[int(gr)].astype(np.float64)
    s = (t[:, 3] * d + t[:, 2]).astype(np.float32).astype(np.float64)      # fmaf: one rounding each
    s = (s * d + t[:, 1]).astype(np.float32).astype(np.float64)
    s = (s * d + t[:, 0]).astype(np.float32)
    return s.astype(np.float64)


def _exact_rows(y, u, nch, per):
    y64 = np.asarray(y, np.float32).astype(np.float64)
    sq = (y64 * y64).astype(np.float32).astype(np.float64)
    w = np.exp2(np.float64(np.float32(u)) * y64 - sq)
    ch = [w[c * per:(c + 1) * per].sum() for c in range(nch)]
    grp = [sum(ch[g * P.KDE_MT_GROUP:(g + 1) * P.KDE_MT_GROUP]) for g in range(-(-nch // P.KDE_MT_GROUP))]
    return np.array(ch + grp + [w.sum()]), w


def _kernel_index(tab, y, u, ucat):
    """kde_index_moments replayed: the group, then the chunk whose running sum passes
    ucat * total (float64 running sums of the float32 row sums), then the point inside the chunk
    (exact float64 weights here: the kernel's float32 scan only moves near-ties)."""
    lo, inv, dl, n, nch, per, T = _table(tab)
    rows = _kernel_rows(tab, u)
    ng = -(-nch // P.KDE_MT_GROUP)
    thr = float(np.float32(ucat)) * rows[nch + ng]
    cum, g = 0.0, ng - 1
    for k in range(ng):
        if cum + rows[nch + k] > thr:
            g = k
            break
        cum += rows[nch + k]
    else:
        cum -= rows[nch + g]
    c1 = min(nch, (g + 1) * P.KDE_MT_GROUP)
    ch = c1 - 1
    for c in range(g * P.KDE_MT_GROUP, c1):
        if cum + rows[c] > thr:
            ch = c
            break
        cum += rows[c]
    else:
        cum -= rows[ch]
    rem = thr - cum
    _, w = _exact_rows(y, u, nch, per)
    part = np.cumsum(w[ch * per:min(len(w), (ch + 1) * per)])
    k = int(np.searchsorted(part, rem, side="right"))
    return min(ch * per + k, min(len(w), (ch + 1) * per) - 1)


@pytest.mark.parametrize("m,sd", [(10000, 0.36), (4096, 0.6), (100, 0.3), (17, 1.0), (1, 0.5)])
def test_moment_rows_match_exact(m, sd):
    """Every row (chunk, group of chunks, whole set) of the kernel's replay against float64
    sums of the exact weights, across the grid; the index the kernel locates equals the exact
    inverse-CDF index except where the draw lies within 1e-6 of a point boundary."""
    rng = np.random.default_rng(m)
    y = (rng.standard_normal(m) * sd).astype(np.float32)
    tab = P.kde_moment_table(y)
    assert tab is not None
    lo, inv, dl, n, nch, per, _ = _table(tab)
    assert nch == -(-m // per) and per == -(-m // P.KDE_MT_CHUNKS) and nch <= P.KDE_MT_CHUNKS
    hi = float(lo) + (n - 1) * float(dl)
    # the covered range holds the data range with margin on both sides
    assert lo <= 2 * (float(y.min()) - 1.9) and hi >= 2 * (float(y.max()) + 1.9)
    us = np.concatenate([rng.uniform(float(lo), hi, 200), [float(lo), hi, 0.0, 2 * float(y.max()), 2 * float(y.min())]])
    worst, flips = 0.0, 0
    for u in us:
        got = _kernel_rows(tab, u)
        if got is None:
            continue
        ref, w = _exact_rows(y, u, nch, per)
        mask = ref > 0
        assert np.all(got[~mask] == 0)
        worst = max(worst, float(np.max(np.abs(got[mask] - ref[mask]) / ref[mask])))
        for ucat in rng.uniform(0, 1, 5):
            idx = _kernel_index(tab, y, u, ucat)
            cdf = np.cumsum(w)
            thr = float(np.float32(ucat)) * cdf[-1]
            exact = min(int(np.searchsorted(cdf, thr, side="right")), m - 1)
            if idx != exact:
                margin = np.min(np.abs(cdf - thr)) / cdf[-1]
                assert margin < 1e-6, (u, ucat, idx, exact, margin)
                flips += 1
    assert worst <= 4e-7, worst
    assert flips <= 2
    # outside the grid the kernel takes the MFMA pass
    assert _kernel_rows(tab, float(lo) - 10 * float(dl)) is None and _kernel_rows(tab, hi + 10 * float(dl)) is None
    assert _kernel_rows(tab, float("nan")) is None


def test_moment_series_bound():
    """KDE_MT_Z bounds |d| ln2 |y'| at a cell edge: the truncated series' relative error."""
    z = P.KDE_MT_Z
    assert z ** P.KDE_MT_TERMS / math.factorial(P.KDE_MT_TERMS) * math.exp(z) < 3e-8


def test_moment_table_declines_wide_data():
    """Weights beyond [2^-80, 2^100] on the covered range: no table (the MFMA pass runs)."""
    y = (np.random.default_rng(0).standard_normal(2000) * 3.0 * 1.2).astype(np.float32)
    assert P.kde_moment_table(y) is None


def test_cfg4_one_feature_steps_carry_tables():
    """The packed cfg4 model (reference-fitted, M = 10,000): every one-parent KDE node has a
    moment table (step reserved[7] = its blob offset), every other node -1; the table's rows
    match the exact sums at the node's own data points; such nodes are not precomputed (the
    table makes their chunk sums cheap in the walk)."""
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
    o = npk.offs["kmt"]
    n_cells, nch, per = (int(v) for v in blob[o + 3:o + 6].view(np.int32))
    tab = blob[o:o + P.KDE_MT_HEADER + n_cells * P.kde_moment_rows(nch) * P.KDE_MT_TERMS]
    c_p = np.float32(P._KDE_C / (max(float(model.cpds[node].hparams["parent_bandwidth"]), 1e-3)
                                 + float(model.cpds[node].hparams["min_scale"])))
    y = (model.cpds[node].extra["parents"].float().numpy() * c_p).reshape(-1)
    for x in model.cpds[node].extra["parents"].float().numpy()[:20, 0]:
        u = np.float32(2.0) * (c_p * np.float32(x))
        got, (ref, _) = _kernel_rows(tab, u), _exact_rows(y, u, nch, per)
        assert np.max(np.abs(got - ref) / ref) <= 4e-7
    # plan rows: reserved[7] holds the offset for those nodes, -1 elsewhere; none precomputed
    latent = [n for n in model.topo if n not in ev]
    plan = P.build_plan(pk, latent=latent, fixed=[n for n in model.topo if n in ev],
                        out_nodes=[target], logp=[target], skip=[], shared_roots=True, mode=P.MODE_MCM)
    rows = plan.steps._vbn_host[0]
    for r in rows:
        if r[P.S_KIND] == P.KIND_ID["kde"] and r[P.S_AUX0] == 1:
            assert r[P.S_RES7] > 0
        else:
            assert r[P.S_RES7] == -1
    pc = P.precompute_plans(pk, plan)
    assert pc is not None
    for r in pc[0].steps._vbn_host[0]:
        if r[P.S_RES7] >= 0:
            assert not r[P.S_FLAGS] & P.F_PRECOMP
