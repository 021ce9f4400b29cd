"""Gibbs step table (plan.build_gibbs_plan) and the fixture -> injected-noise mapping, on CPU."""
import pytest
import torch

from conftest import load_golden
from golden_noise import gibbs_noise
from vectorizedbayesiannetwork_amd import plan as P
from vectorizedbayesiannetwork_amd.model import model_from_checkpoint

NAMES = ["ext_gibbs_mix10", "ext_gibbs_kde6"]


@pytest.mark.parametrize("name", NAMES)
def test_gibbs_step_table(name):
    fx = load_golden(name)
    model = model_from_checkpoint(fx["model"])
    pk = P.PackedModel(model, torch.device("cpu"))
    children = model.children()
    for case in fx["cases"]:
        q = case["query"]
        fixed = set(q["evidence"]) | set(q["do"])
        latent = [n for n in model.topo if n not in fixed]
        gp = P.build_gibbs_plan(pk, latent=latent, fixed=[n for n in model.topo if n in fixed], target=q["target"])
        rows = gp.steps.numpy()
        slot = gp.init.slot_of
        # every node keeps its own slots for the whole walk
        spans = sorted((slot[n], slot[n] + model.out_dim(n)) for n in model.topo)
        assert all(a[1] <= b[0] for a, b in zip(spans, spans[1:]))
        i = 0
        for j, n in enumerate(latent):
            r = rows[i]
            assert (r[P.S_ROLE], r[P.S_OUTCOL], r[P.S_NOISE]) == (P.ROLE_LATENT, slot[n], 2 * j)
            assert r[P.S_FLAGS] & P.F_LOGP and r[P.S_FLAGS] & P.F_LPRESET
            i += 1
            for c in children[n]:
                r = rows[i]
                assert (r[P.S_ROLE], r[P.S_OUTCOL]) == (P.ROLE_FIXED, slot[c])
                assert r[P.S_FLAGS] & P.F_KEEP and r[P.S_FLAGS] & P.F_LOGP
                ins = gp.in_cols.numpy()[r[P.S_INOFF]:r[P.S_INOFF] + r[P.S_NIN]].tolist()
                want = [k for p in model.parents[c] for k in range(slot[p], slot[p] + model.out_dim(p))]
                assert ins == want                                   # candidate + current parents
                i += 1
            r = rows[i]
            assert (r[P.S_ROLE], r[P.S_OUTCOL], r[P.S_NOISE]) == (P.ROLE_SELECT, slot[n], 2 * j + 1)
            i += 1
        assert rows[i][P.S_ROLE] == P.ROLE_COLLECT and rows[i][P.S_OUTCOL] == slot[q["target"]]
        assert i + 1 == gp.n_steps and gp.n_noise == max(2 * len(latent), 1)


@pytest.mark.parametrize("name", NAMES)
def test_gibbs_noise_consumes_every_draw(name):
    fx = load_golden(name)
    model = model_from_checkpoint(fx["model"])
    dmax = max(model.out_dim(n) for n in model.topo)
    for case in fx["cases"]:
        q = case["query"]
        latent = [n for n in model.topo if n not in q["evidence"] and n not in q["do"]]
        init, sweeps = gibbs_noise(case, model, latent, dmax)       # asserts every record is placed
        thin = max(case["params"]["n_steps"], 1)
        assert sweeps.shape[0] == case["params"]["burn_in"] + case["n_samples"] * thin
        u = sweeps[:, 1::2, 0, :, 0, 0]
        assert bool(((u > 0) & (u < 1)).all())                       # every choice uniform is set


def test_reference_gibbs_collects_final_state():
    """gibbs.py:86 appends views of the chain state: every collected entry is the last sweep."""
    for name in NAMES:
        for case in load_golden(name)["cases"]:
            s = case["outputs"]["samples"]
            assert torch.equal(s, s[:, :1].expand_as(s))


def _group_rw(rows, ic, b, e):
    cols = lambda r: set(range(int(r[P.S_OUTCOL]), int(r[P.S_OUTCOL]) + int(r[P.S_OUTDIM])))
    rd, wr = set(), cols(rows[b])
    for k in range(b, e):
        r = rows[k]
        rd |= set(int(c) for c in ic[int(r[P.S_INOFF]):int(r[P.S_INOFF]) + int(r[P.S_NIN])])
        if int(r[P.S_ROLE]) == P.ROLE_FIXED:
            rd |= cols(r)
    return rd, wr


@pytest.mark.parametrize("name", NAMES + ["cfg2"])
@pytest.mark.parametrize("n_waves", [1, 2, 4])
def test_gibbs_levels_schedule(name, n_waves):
    """plan.gibbs_levels: every node update (LATENT .. SELECT) runs exactly once per sweep, the
    updates of one level touch no slot another one writes, and every conflicting pair keeps its
    sweep order -- so the wave-parallel sweep is the sequential one, bit for bit."""
    if name == "cfg2":
        import bench
        cfg, model, target, ev = bench.build_model("cfg2")
        cases = [{"query": {"target": target, "evidence": dict.fromkeys(ev), "do": {}}}]
    else:
        fx = load_golden(name)
        model = model_from_checkpoint(fx["model"])
        cases = fx["cases"]
    pk = P.PackedModel(model, torch.device("cpu"))
    for case in cases:
        q = case["query"]
        fixed = set(q["evidence"]) | set(q["do"])
        gp = P.build_gibbs_plan(pk, latent=[n for n in model.topo if n not in fixed],
                                fixed=[n for n in model.topo if n in fixed], target=q["target"])
        rows, ic, _ = gp.steps._vbn_host
        levels = P.gibbs_levels(rows, ic, n_waves)
        assert all(len(lv) == n_waves for lv in levels)
        ranges = [(lv, w, b, e) for lv, waves in enumerate(levels) for w, rs in enumerate(waves) for b, e in rs]
        covered = sorted(i for _, _, b, e in ranges for i in range(b, e))
        assert covered == list(range(len(rows)))                        # each step exactly once
        coll = [r for r in ranges if rows[r[2]][P.S_ROLE] == P.ROLE_COLLECT]
        assert coll and all(lv == len(levels) - 1 and w == 0 for lv, w, _, _ in coll)
        groups = [r for r in ranges if rows[r[2]][P.S_ROLE] == P.ROLE_LATENT]
        assert len(groups) == len(gp.latent)
        for i, (lv1, _, b1, e1) in enumerate(groups):
            r1, w1 = _group_rw(rows, ic, b1, e1)
            for lv2, _, b2, e2 in groups[i + 1:]:
                r2, w2 = _group_rw(rows, ic, b2, e2)
                conflict = bool(w1 & (r2 | w2) or r1 & w2)
                if lv1 == lv2:
                    assert not conflict
                if conflict:
                    assert (lv1 < lv2) == (b1 < b2)
        if len(groups) > 2 and n_waves > 1:
            assert len(levels) < len(groups) + 1                         # some updates run together


def _cases(name):
    if name == "cfg2":
        import bench
        cfg, model, target, ev = bench.build_model("cfg2")
        return model, [{"query": {"target": target, "evidence": dict.fromkeys(ev), "do": {}}}]
    fx = load_golden(name)
    return model_from_checkpoint(fx["model"]), fx["cases"]


def _schedule_violations(rows, ic, phases):
    """Ordering constraints a phased schedule breaks, restated independently of
    plan.gibbs_step_deps: inside an update the LATENT step comes first and the SELECT last; for
    updates h < g (sweep order) a step of g reading a slot h writes runs after h's SELECT, and a
    step of h reading a slot g writes runs before g's LATENT.  "a before b" = an earlier phase,
    or the same wave earlier in the same phase."""
    pos = {op[1]: (k, w, j) for k, ph in enumerate(phases) for w, wops in enumerate(ph) for j, op in enumerate(wops)}

    def before(a, b):
        (ka, wa, ja), (kb, wb, jb) = pos[a], pos[b]
        return ka < kb or (ka == kb and wa == wb and ja < jb)

    def reads(i):
        return set() if rows[i][P.S_ROLE] == P.ROLE_SELECT else set(_group_rw(rows, ic, i, i + 1)[0])

    bad = []
    groups, _, _ = P._gibbs_update_levels(rows, ic)
    for g, (b, e) in enumerate(groups):
        bad += [(b, i) for i in range(b + 1, e) if not before(b, i)]
        bad += [(i, e - 1) for i in range(b, e - 1) if not before(i, e - 1)]
        wg = _group_rw(rows, ic, b, e)[1]
        for bh, eh in groups[:g]:
            wh = _group_rw(rows, ic, bh, eh)[1]
            bad += [(eh - 1, i) for i in range(b, e) if reads(i) & wh and not before(eh - 1, i)]
            bad += [(i, b) for i in range(bh, eh) if reads(i) & wg and not before(i, b)]
    return bad


def test_schedule_checker_catches_reordering():
    """_schedule_violations flags a step moved ahead of what it depends on (so the phase tests
    above cannot pass vacuously)."""
    model, cases = _cases("cfg2")
    pk = P.PackedModel(model, torch.device("cpu"))
    q = cases[0]["query"]
    gp = P.build_gibbs_plan(pk, latent=[n for n in model.topo if n not in q["evidence"]],
                            fixed=[n for n in model.topo if n in q["evidence"]], target=q["target"])
    rows, ic, _ = gp.steps._vbn_host
    phases, _ = P.gibbs_schedule(rows, ic, 4, split="dag")
    assert _schedule_violations(rows, ic, phases) == []
    # move the last phase's first op into phase 0: it depends on something later
    k = max(k for k, ph in enumerate(phases) if any(ph) and any(op[0] != "run" for ops in ph for op in ops))
    w = next(w for w, ops in enumerate(phases[k]) if ops)
    moved = [[list(ops) for ops in ph] for ph in phases]
    op = moved[k][w].pop(0)
    moved[0][0].insert(0, op)
    assert _schedule_violations(rows, ic, moved)


@pytest.mark.parametrize("name", NAMES + ["cfg2"])
@pytest.mark.parametrize("n_waves", [1, 2, 4])
@pytest.mark.parametrize("split", [None, True, "dag"])
def test_gibbs_schedule_phases(name, n_waves, split):
    """plan.gibbs_schedule: the phases run every step once and every ordering constraint of
    plan.gibbs_step_deps holds (checked against an independent restatement: a step before
    another = an earlier phase, or the same wave earlier in the same phase); the level forms
    keep gibbs_levels' levels; a split step scores into its own row and the SELECT adds its
    rows in sweep order -- so the score each SELECT sees is the sequential sweep's float32 sum,
    bit for bit (emulated here)."""
    import numpy as np
    model, cases = _cases(name)
    pk = P.PackedModel(model, torch.device("cpu"))
    for case in cases:
        q = case["query"]
        fixed = set(q["evidence"]) | set(q["do"])
        gp = P.build_gibbs_plan(pk, latent=[n for n in model.topo if n not in fixed],
                                fixed=[n for n in model.topo if n in fixed], target=q["target"])
        rows, ic, _ = gp.steps._vbn_host
        phases, n_rows = P.gibbs_schedule(rows, ic, n_waves, split=split)
        assert all(len(ph) == n_waves for ph in phases)
        ops = [(k, w, op) for k, ph in enumerate(phases) for w, wops in enumerate(ph) for op in wops]
        assert sorted(op[1] for _, _, op in ops) == list(range(len(rows)))   # each step once
        phase_of = {op[1]: k for k, _, op in ops}
        assert _schedule_violations(rows, ic, phases) == []
        groups, level, _ = P._gibbs_update_levels(rows, ic)
        for b, e in groups:
            assert P.gibbs_step_deps(rows, ic)[e - 1] >= set(range(b, e - 1))
        if split is True:                                   # the level form keeps the levels
            for (b, e), lv in zip(groups, level):
                for (b2, e2), lv2 in zip(groups, level):
                    if lv < lv2:
                        assert max(phase_of[i] for i in range(b, e)) < min(phase_of[i] for i in range(b2, e2))
        for b, e in groups:
            whole = phase_of[b] == phase_of[e - 1]                        # one wave, register score
            if whole:
                assert len({w for _, w, op in ops if b <= op[1] < e}) == 1
                assert all(op[0] == "run" for _, _, op in ops if b <= op[1] < e)
        # float32 score emulation: random per-step terms, sequential vs scheduled
        rng = np.random.default_rng(0)
        term = rng.standard_normal(len(rows)).astype(np.float32) * np.float32(100)
        seq, lp = {}, np.float32(0)
        for i, r in enumerate(rows):
            role = int(r[P.S_ROLE])
            if role == P.ROLE_LATENT:
                lp = np.float32(0) + term[i]
            elif role == P.ROLE_FIXED:
                lp = np.float32(lp + term[i])
            elif role == P.ROLE_SELECT:
                seq[i] = lp
        lds = np.full(max(n_rows, 1), np.nan, np.float32)
        reg = [np.float32(0)] * n_waves
        got = {}
        for ph in phases:
            for w, wops in enumerate(ph):
                for op in wops:
                    i, role = op[1], int(rows[op[1]][P.S_ROLE])
                    if op[0] == "lpout":
                        assert role in (P.ROLE_LATENT, P.ROLE_FIXED)
                        lds[op[2]] = np.float32(0) + term[i]
                    elif op[0] == "select":
                        t = lds[op[2][0]]
                        for rr in op[2][1:]:
                            t = np.float32(t + lds[rr])
                        got[i] = t
                    elif role == P.ROLE_LATENT:
                        reg[w] = np.float32(0) + term[i]
                    elif role == P.ROLE_FIXED:
                        reg[w] = np.float32(reg[w] + term[i])
                    elif role == P.ROLE_SELECT:
                        got[i] = reg[w]
        assert got.keys() == seq.keys()
        assert all(got[i].tobytes() == seq[i].tobytes() for i in seq)
        if split in (True, "dag"):
            assert n_rows > 0 and not any(op[0] == "run" and int(rows[op[1]][P.S_ROLE]) != P.ROLE_COLLECT
                                          for _, _, op in ops)


def test_gibbs_schedule_splits_uneven_levels():
    """The cost model splits cfg2's uneven levels on 4 waves and the modelled sweep shortens
    (whole updates 24.15 step units, split where it pays 19.7; one wave stays whole)."""
    model, cases = _cases("cfg2")
    pk = P.PackedModel(model, torch.device("cpu"))
    q = cases[0]["query"]
    gp = P.build_gibbs_plan(pk, latent=[n for n in model.topo if n not in q["evidence"]],
                            fixed=[n for n in model.topo if n in q["evidence"]], target=q["target"])
    rows, ic, _ = gp.steps._vbn_host
    whole = P.gibbs_schedule_cost(P.gibbs_schedule(rows, ic, 4, split=False)[0], rows)
    auto, n_rows = P.gibbs_schedule(rows, ic, 4)
    assert n_rows > 0 and P.gibbs_schedule_cost(auto, rows) < 0.85 * whole
    one, n1 = P.gibbs_schedule(rows, ic, 1)
    assert n1 == 0 and len(one) == len(P.gibbs_levels(rows, ic, 1))


def test_chain_sweep_source():
    """jit.plan_source with a phased schedule: the chain-workgroup sweep, every step once."""
    import re
    import bench
    from vectorizedbayesiannetwork_amd import jit
    cfg, model, target, ev = bench.build_model("cfg2")
    pk = P.PackedModel(model, torch.device("cpu"))
    gp = P.build_gibbs_plan(pk, latent=[n for n in model.topo if n not in ev],
                            fixed=[n for n in model.topo if n in ev], target=target)
    rows, ic, _ = gp.steps._vbn_host
    phases, n_rows = P.gibbs_schedule(rows, ic, 4)
    src = jit.plan_source(rows, ic, gp.kind_mask | 64 | 256, (phases, n_rows))
    assert "#define VBN_PLAN_CHAIN_WAVES 4" in src
    assert f"__shared__ float vbn_lp_rows[{n_rows} * WAVE];" in src
    assert src.count("__syncthreads();") == len(phases)
    idx = [int(x) for x in re.findall(r"vbn_plan_step_(?:direct|lpout|select)<KM, ([0-9]+)", src)]
    assert sorted(idx) == list(range(len(rows)))
    assert "VBN_PLAN_CHAIN_WAVES" not in jit.plan_source(rows, ic, gp.kind_mask | 64 | 256)
    assert "__launch_bounds__(4 * WAVE)" in src
    src8 = jit.plan_source(rows, ic, gp.kind_mask | 256, P.gibbs_schedule(rows, ic, 8))
    assert "#define VBN_PLAN_CHAIN_WAVES 8" in src8 and "__launch_bounds__(8 * WAVE)" in src8


def _gibbs_plan_of(n_nodes, kinds=("linear_gaussian",)):
    from vectorizedbayesiannetwork_amd import synthetic
    from vectorizedbayesiannetwork_amd.model import random_init_model
    g = synthetic.random_dag(n_nodes, seed=0)
    data = synthetic.sem_data(g, 256, seed=0)
    model = random_init_model(g, synthetic.round_robin_kinds(g, kinds), data, seed=0)
    pk = P.PackedModel(model, torch.device("cpu"))
    ev = set(model.topo[: n_nodes // 4])
    gp = P.build_gibbs_plan(pk, latent=[n for n in model.topo if n not in ev],
                            fixed=[n for n in model.topo if n in ev], target=model.topo[-1])
    return gp


def test_chain_waves_fit_lds():
    """the auto chain-wave choice counts the sweep unit's static score rows
    (vbn_lp_rows) as well as the dynamic slots + scratch rows, and falls back to fewer waves, then
    the one-wave form, when a chain workgroup would not fit the CU's 160 KiB of LDS."""
    from vectorizedbayesiannetwork_amd import jit, ops
    small = _gibbs_plan_of(32)
    init = small.init
    rows, ic, key = small.steps._vbn_host
    for cw in (1, 2, 4, 8):
        _, n_rows = P.gibbs_schedule(rows, ic, cw)
        want = (init.n_slots + cw * max(init.max_out, 1)) * 256 + max(n_rows, 1) * 256
        assert jit.chain_lds_bytes(rows, ic, key, cw, init.n_slots, init.max_out) == want
    assert ops.fit_chain_waves(small.steps, 8, init.n_slots, init.max_out) == 8
    # a wide DAG: its score rows alone (one per LATENT / child step) exceed 160 KiB at 8 waves
    wide = _gibbs_plan_of(700)
    wi = wide.init
    wrows, wic, wkey = wide.steps._vbn_host
    assert jit.chain_lds_bytes(wrows, wic, wkey, 8, wi.n_slots, wi.max_out) > jit.LDS_BYTES
    cw = ops.fit_chain_waves(wide.steps, 8, wi.n_slots, wi.max_out)
    assert cw < 8
    if cw > 0:
        assert jit.chain_lds_bytes(wrows, wic, wkey, cw, wi.n_slots, wi.max_out) <= jit.LDS_BYTES
    # steps without a host copy (no specialised unit) keep the requested count
    assert ops.fit_chain_waves(torch.zeros(1, 32, dtype=torch.int32), 4, 10, 1) == 4
