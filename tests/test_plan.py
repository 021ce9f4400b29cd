"""Host-side plan logic: liveness slot allocation and MFMA fragment packing.

``emulate_mlp`` replays csrc/vbn_walk_impl.h's mlp_forward data flow in numpy with the
documented gfx950 lane layouts of v_mfma_f32_32x32x2_f32 (A[i=l&31][k=l>>5],
B[k=l>>5][j=l&31], D row (r&3)+8(r>>2)+4(l>>5), col l&31) and v_permlane32_swap, so the
packed parameter blocks are checked against torch's MLP without a GPU.
"""
import numpy as np
import pytest
import torch

from conftest import golden_names, load_golden
from vectorizedbayesiannetwork_amd import synthetic
from vectorizedbayesiannetwork_amd.model import model_from_checkpoint, random_init_model
from vectorizedbayesiannetwork_amd.plan import (F_LOGP, MODE_MCM, MODE_WEIGHTED, ROLE_FIXED, ROLE_LATENT,
                                                S_INOFF, S_NIN, S_OFF_B2, S_OFF_B3, S_OFF_W2H, S_OFF_STD, S_OFF_W1,
                                                S_OFF_W2, S_OFF_W3, S_OUTCOL, S_OUTDIM, S_ROLE, S_FLAGS,
                                                PackedModel, build_plan)


def _row(r, h):
    return (r & 3) + 8 * (r >> 2) + 4 * h


def mfma_32x32x2(a_lane, b_lane, c):
    """a_lane, b_lane: [64]; c: [64,16] (lane, reg) -> d [64,16]."""
    A = np.zeros((32, 2)); B = np.zeros((2, 32))
    for l in range(64):
        A[l & 31, l >> 5] = a_lane[l]
        B[l >> 5, l & 31] = b_lane[l]
    D = A.astype(np.float64) @ B
    d = c.astype(np.float64).copy()
    for l in range(64):
        for r in range(16):
            d[l, r] += D[_row(r, l >> 5), l & 31]
    return d


def permlane32_swap(vdst, vsrc):
    a, b = vdst.copy(), vsrc.copy()
    a[32:], b[:32] = vsrc[:32].copy(), vdst[32:].copy()
    return a, b


def mfma_32x32x16_split(P, row, hb, lanes):
    """Layer 2 as the kernel's split-f16 product: A/B lane l, element j <-> k = 8(l>>5) + j of
    the K=16 step; B from the layer-1 accumulator registers 8s + j (hi by masking the low 13
    mantissa bits, lo = x - hi rounded to f16); accumulator starts from the packed b2."""
    halfs = P.astype(np.float32)[row[S_OFF_W2H]: row[S_OFF_W2H] + 4 * 64 * 4].view(np.float16)
    frag = halfs.reshape(4, 64, 8).astype(np.float64)          # hi s0, hi s1, lo s0, lo s1
    d = acc_init(P, row, 1)
    for s in range(2):
        A = np.zeros((32, 16)); Bh = np.zeros((16, 32)); Bl = np.zeros((16, 32)); Al = np.zeros((32, 16))
        for l in range(64):
            h = l >> 5
            x = hb[l, 8 * s: 8 * s + 8].astype(np.float32)
            hi = (x.view(np.int32) & np.int32(-8192)).view(np.float32)
            Bh[8 * h: 8 * h + 8, l & 31] = hi.astype(np.float16)
            Bl[8 * h: 8 * h + 8, l & 31] = (x - hi).astype(np.float16)
            A[l & 31, 8 * h: 8 * h + 8] = frag[s, l]
            Al[l & 31, 8 * h: 8 * h + 8] = frag[2 + s, l]
        D = Al @ Bh + A @ Bl + A @ Bh
        for l in range(64):
            for r in range(16):
                d[l, r] += D[_row(r, l >> 5), l & 31]
    return d


def acc_init(P, row, layer):
    """[64, 16] accumulator initial values: lane l, register r <- b[row(r, l >> 5)]."""
    b = P[row[S_OFF_B2] + 64 * layer: row[S_OFF_B2] + 64 * layer + 32].reshape(2, 16)
    return b[np.arange(64) >> 5].astype(np.float64)


def emulate_mlp(P, row, parents64, std, split=False):
    """parents64: [nin, 64] values of the 64 particles of a wave -> head [n_out, 64]."""
    nin = row[S_NIN]
    t1 = (nin + 1) // 2
    lanes = np.arange(64)
    half, c = lanes >> 5, lanes & 31
    h2 = []
    for g in range(2):
        acc = acc_init(P, row, 0)
        for t in range(t1):
            kk = 2 * t + half
            z = np.zeros(64)
            for l in range(64):
                if kk[l] < nin:
                    v = parents64[kk[l], c[l] + 32 * g]
                    if std:
                        v = (v - P[row[S_OFF_STD] + kk[l]]) * P[row[S_OFF_STD] + nin + kk[l]]
                    z[l] = v
            acc = mfma_32x32x2(P[row[S_OFF_W1] + t * 64: row[S_OFF_W1] + t * 64 + 64], z, acc)
        hb = np.maximum(acc, 0)
        if split:
            b = mfma_32x32x16_split(P, row, hb, lanes)
        else:
            w2 = P[row[S_OFF_W2]: row[S_OFF_W2] + 1024].reshape(4, 64, 4)
            b = acc_init(P, row, 1)
            for s in range(16):
                b = mfma_32x32x2(w2[s // 4, :, s % 4], hb[:, s], b)
        h2.append(b)
    # head in the accumulator layout (csrc mlp_head): lane half h sums its 16 rows with the
    # weights w3[j][16 h + r], one permlane32 swap per output adds the halves
    n_out = row[10]
    w3 = P[row[S_OFF_W3]: row[S_OFF_W3] + 32 * n_out].reshape(n_out, 32)
    b3 = P[row[S_OFF_B3]: row[S_OFF_B3] + n_out]
    out = np.zeros((n_out, 64))
    for j in range(n_out):
        wl = w3[j].reshape(2, 16)[half]                              # [64, 16]
        p0 = (wl * np.maximum(h2[0], 0)).sum(1)
        p1 = (wl * np.maximum(h2[1], 0)).sum(1)
        a, b = permlane32_swap(p0, p1)
        out[j] = a + b + b3[j]
    return out


@pytest.mark.parametrize("name", ["readme", "family_gaussian_nn", "family_mdn", "mix12"])
def test_mfma_fragment_packing_reproduces_torch_mlp(name):
    model = model_from_checkpoint(load_golden(name)["model"])
    pk = PackedModel(model, torch.device("cpu"))
    P = pk.params.numpy().astype(np.float64)
    rng = np.random.default_rng(0)
    checked = 0
    for node in model.topo:
        rec = model.cpds[node]
        if rec.kind not in ("gaussian_nn", "mdn", "softmax_nn") or rec.is_root:
            continue
        plan = build_plan(pk, latent=[node], fixed=model.parents[node], logp=[], out_nodes=[node],
                          shared_roots=False, mode=MODE_WEIGHTED,
                          skip=[n for n in model.topo if n != node and n not in model.parents[node]])
        row = plan.steps[-1].numpy()
        parents64 = rng.normal(size=(rec.input_dim, 64))
        std = rec.kind == "gaussian_nn"
        got = emulate_mlp(P, row, parents64, std)
        got_split = emulate_mlp(P, row, parents64, std, split=True)
        x = torch.tensor(parents64.T, dtype=torch.float64)
        if std:
            x = (x - rec.state["mean_x"].double()) / rec.state["std_x"].double()
        h = x
        layers = rec.mlp_layers()
        for i, (w, b) in enumerate(layers):
            h = h @ w.double().t() + b.double()
            if i + 1 < len(layers):
                h = torch.relu(h)
        np.testing.assert_allclose(got, h.numpy().T, rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(got_split, h.numpy().T, rtol=2e-5, atol=2e-5)
        checked += 1
    assert checked > 0


@pytest.mark.parametrize("cfg", ["cfg2", "cfg3", "cfg5"])
def test_weight_blocks_cover_the_mlp_fragments(cfg):
    """Each NN step's LDS-staged weight block (wblk_off, wblk_len) starts at W1 and holds the
    accumulator-init biases, the split-f16 W2 fragments and the head; lengths are whole 1-KiB
    DMA chunks; plan.wbuf is the largest block; steps without an MLP stage nothing."""
    from vectorizedbayesiannetwork_amd.plan import (S_KIND, S_NOUT, S_WBLK_LEN, S_WBLK_OFF, WBLK_CHUNK, F_ROOT,
                                                    build_gibbs_plan, ROLE_SELECT, ROLE_COLLECT)
    c = synthetic.CONFIGS[cfg]
    g = synthetic.random_dag(c["n_nodes"], seed=0)
    model = random_init_model(g, synthetic.round_robin_kinds(g, c["kinds"]), synthetic.sem_data(g, 300, seed=0),
                              overrides={"kde": {"max_points": 64}})
    pk = PackedModel(model, torch.device("cpu"))
    target, ev = synthetic.default_query_nodes(g, seed=1)
    latent = [n for n in model.topo if n not in ev]
    plan = build_plan(pk, latent=latent, fixed=ev, logp=[target] + ev, out_nodes=[target],
                      shared_roots=True, mode=MODE_MCM)
    steps = plan.steps.numpy()
    nn = 0
    for row in steps:
        mlp = row[S_KIND] in (0, 2, 4) and not (row[S_FLAGS] & F_ROOT) and (
            row[S_ROLE] == ROLE_LATENT or (row[S_FLAGS] & F_LOGP))
        if not mlp:
            assert row[S_WBLK_LEN] == 0
            continue
        nn += 1
        off, ln = row[S_WBLK_OFF], row[S_WBLK_LEN]
        assert off == row[S_OFF_W1] and ln > 0 and ln % WBLK_CHUNK == 0
        assert off % 4 == 0 and row[S_OFF_B2] % 4 == 0 and row[S_OFF_W2H] % 4 == 0 and row[S_OFF_W3] % 4 == 0
        assert off < row[S_OFF_B2] < row[S_OFF_W2H] < row[S_OFF_W3] <= row[S_OFF_B3]
        assert row[S_OFF_B2] + 128 <= row[S_OFF_W2H] and row[S_OFF_W2H] + 1024 <= row[S_OFF_W3]
        assert row[S_OFF_B3] + row[S_NOUT] <= off + ln <= pk.params.numel()
    assert nn > 0 and plan.wbuf == steps[:, S_WBLK_LEN].max()
    gp = build_gibbs_plan(pk, latent=latent, fixed=ev, target=target)
    gs = gp.steps.numpy()
    sel = (gs[:, S_ROLE] == ROLE_SELECT) | (gs[:, S_ROLE] == ROLE_COLLECT)
    assert (gs[sel, S_WBLK_LEN] == 0).all() and gp.wbuf == gs[:, S_WBLK_LEN].max() > 0


def _check_liveness(model, plan):
    """Replay the slot writes; every read must find the right parent's value."""
    steps = plan.steps.numpy()
    in_cols = plan.in_cols.numpy()
    holder = {}
    order = [n for n in model.topo if n in plan.slot_of]
    for i, node in enumerate(order):
        row = steps[i]
        reads = row[S_ROLE] == ROLE_LATENT or (row[S_FLAGS] & F_LOGP)
        if reads:
            cols = in_cols[row[S_INOFF]: row[S_INOFF] + row[S_NIN]]
            expect = []
            for p in model.parents[node]:
                expect += [(p, d) for d in range(model.out_dim(p))]
            assert [holder.get(int(c)) for c in cols] == expect, (node, cols)
        for d in range(row[S_OUTDIM]):
            holder[int(row[S_OUTCOL] + d)] = (node, d)
        assert row[S_OUTCOL] + row[S_OUTDIM] <= plan.n_slots
    outs = plan.out_cols.numpy()
    want = []
    for n in plan.out_nodes:
        want += [(n, d) for d in range(model.out_dim(n))]
    assert [holder.get(int(c)) for c in outs] == want


@pytest.mark.parametrize("name", golden_names())
def test_liveness_slots_never_clobber_live_values(name):
    model = model_from_checkpoint(load_golden(name)["model"])
    pk = PackedModel(model, torch.device("cpu"))
    topo = model.topo
    for k in range(0, len(topo), 2):
        ev = topo[:k:3]
        target = topo[-1 - (k % 3)]
        latent = [n for n in topo if n not in ev]
        plan = build_plan(pk, latent=latent, fixed=ev, logp=[target] + ev, out_nodes=[target],
                          shared_roots=True, mode=MODE_MCM)
        _check_liveness(model, plan)
        joint = build_plan(pk, latent=latent, fixed=ev, logp=[], out_nodes=list(topo),
                           shared_roots=True, mode=MODE_MCM)
        _check_liveness(model, joint)
        assert joint.n_slots == sum(model.out_dim(n) for n in topo)


@pytest.mark.parametrize("cfg", ["cfg2", "cfg3", "cfg4", "anchor64", "cfg5"])
def test_bench_configs_pack(cfg):
    c = synthetic.CONFIGS[cfg]
    g = synthetic.random_dag(c["n_nodes"], seed=0)
    data = synthetic.sem_data(g, 300, seed=0)
    model = random_init_model(g, synthetic.round_robin_kinds(g, c["kinds"]), data,
                              overrides={"kde": {"max_points": 64}})
    pk = PackedModel(model, torch.device("cpu"))
    target, ev = synthetic.default_query_nodes(g, seed=1)
    plan = build_plan(pk, latent=[n for n in model.topo if n not in ev], fixed=ev, logp=[target],
                      out_nodes=[target], shared_roots=True, mode=MODE_MCM)
    _check_liveness(model, plan)
    assert plan.n_slots < len(model.topo)               # liveness reuses slots
    assert (plan.steps[:, S_ROLE] == ROLE_FIXED).sum() == len(ev)


def test_rb_params_plan_roles_and_widths():
    """RB target walks as role PARAMS with loc++scale (gaussian) or C probabilities (softmax_nn)."""
    from vectorizedbayesiannetwork_amd.plan import ROLE_PARAMS, S_KIND
    model = model_from_checkpoint(load_golden("ext_rb_mix10")["model"])
    pk = PackedModel(model, torch.device("cpu"))
    seen = set()
    for target in model.topo:
        rec = model.cpds[target]
        if rec.kind not in ("gaussian_nn", "linear_gaussian", "softmax_nn"):
            continue
        desc, stack = set(), [target]
        ch = model.children()
        while stack:
            for c in ch[stack.pop()]:
                if c not in desc:
                    desc.add(c)
                    stack.append(c)
        keep = [x for x in model.topo if x not in desc]
        ev = [x for x in keep if x != target][:2]
        plan = build_plan(pk, latent=[x for x in keep if x not in ev and x != target], fixed=ev, logp=ev,
                          out_nodes=[target], params=[target], shared_roots=True, mode=MODE_WEIGHTED,
                          skip=sorted(desc))
        row = [r for r in plan.steps.tolist() if r[S_OUTCOL] == plan.slot_of[target] and r[S_ROLE] == ROLE_PARAMS]
        assert len(row) == 1
        width = 2 if rec.kind != "softmax_nn" else int(rec.hp("n_classes"))
        assert plan.out_cols.numel() == width
        assert plan.out_cols.tolist() == list(range(plan.slot_of[target], plan.slot_of[target] + width))
        seen.add(rec.kind)
    assert seen == {"gaussian_nn", "linear_gaussian", "softmax_nn"}


def _mfma_16x16x4(a_lane, b_lane, c_lane):
    """v_mfma_f32_16x16x4_f32: A[l&15][l>>4], B[l>>4][l&15]; D lane l rows 4(l>>4)+r, col l&15."""
    A = np.zeros((16, 4)); B = np.zeros((4, 16))
    for l in range(64):
        A[l & 15, l >> 4] = a_lane[l]
        B[l >> 4, l & 15] = b_lane[l]
    D = A @ B
    return np.array([[D[4 * (l >> 4) + r, l & 15] + c_lane[l][r] for r in range(4)] for l in range(64)])


@pytest.mark.parametrize("nf", [1, 2, 3])
def test_kde_mfma_pack_gives_kernel_weights(nf):
    """The KDE point packs (plan._kde_pack) in the 16x16x4 operand layout, with the particle
    operands of csrc kde_operands (zero-C form for nf <= 2, C = -|x'|^2 for nf = 3), give
    exp2(D) = exp(-|x - y|^2 / (2 s^2)) for every (particle, point); padding points weigh 0."""
    from vectorizedbayesiannetwork_amd.plan import _KDE_C, _kde_cb, _kde_pack, KDE_CHUNKS
    rng = np.random.default_rng(nf)
    m, s = 37, 0.7
    c = np.float32(_KDE_C / s)
    pts = rng.normal(size=(m, nf)).astype(np.float32)
    parts = rng.normal(size=(64, nf)).astype(np.float32)
    pack = _kde_pack([pts * c])                                 # [blocks][4][16]
    assert pack.shape == (KDE_CHUNKS * _kde_cb(m), 4, 16)
    xv = parts * c
    w = np.zeros((64, pack.shape[0] * 16))
    for t in range(4):
        b_lane, c_lane = np.zeros(64), np.zeros((64, 4))
        for l in range(64):
            g, n = l >> 4, l & 15
            x = xv[16 * t + n].astype(np.float64)
            sq = float((x ** 2).sum())
            b_lane[l] = 2 * x[g] if g < nf else (-1.0 if g == nf else (-sq if (g == nf + 1 and nf <= 2) else 0.0))
            c_lane[l] = 0.0 if nf <= 2 else -sq
        for blk in range(pack.shape[0]):
            a_lane = pack[blk].reshape(-1)                      # lane l reads element blk*64 + l
            d = _mfma_16x16x4(a_lane, b_lane, c_lane)
            for l in range(64):
                for r in range(4):
                    w[16 * t + (l & 15), blk * 16 + 4 * (l >> 4) + r] = np.exp2(d[l, r])
    ref = np.exp(-0.5 * ((parts[:, None, :].astype(np.float64) - pts[None].astype(np.float64)) ** 2).sum(-1) / s ** 2)
    np.testing.assert_allclose(w[:, :m], ref, rtol=1e-5, atol=1e-30)
    assert (w[:, m:] == 0).all()


@pytest.mark.parametrize("nf", [1, 2, 3, 4])
def test_kde_bf16_pack_gives_kernel_weights(nf):
    """The bf16x3 point pack (plan._kde_pack_b32) in the v_mfma_f32_32x32x16_bf16 operand layout
    (lane l of K group g: A = point l & 31's slots 16 g + 8 (l >> 5) .. +7; B = the particle's
    slots, csrc kde_b32_ops: 2x' split into bf16 hi / mid / lo in the _BF16_B pattern, -1 against
    |y'|^2's split, the split of -|x'|^2 against 1.0; C = 0; K = 16 for one feature, 32 for 2-4)
    gives, with exact bf16 products summed in float64, -|x' - y'|^2 to float32 accuracy (the
    float32 contraction's rounding): exp2 of it = exp(-|x - y|^2 / (2 s^2)) within 1e-5 (the f32
    inputs' rounding); padding points weigh 0; the three-way splits are exact."""
    from vectorizedbayesiannetwork_amd.plan import (_BF16_B, _KDE_C, _bf16_split3, _kde_cb, _kde_pack,
                                                    _kde_pack_b32, KDE_CHUNKS)
    rng = np.random.default_rng(10 + nf)
    m, s = 77, 0.6
    c = np.float32(_KDE_C / s)
    pts = rng.normal(size=(m, nf)).astype(np.float32) * 2
    parts = rng.normal(size=(64, nf)).astype(np.float32) * 2
    v = (rng.normal(size=1000) * 10.0 ** rng.integers(-6, 6, 1000)).astype(np.float32)
    bits = [(h.astype(np.uint32) << 16).view(np.float32).astype(np.float64) for h in _bf16_split3(v)]
    assert np.array_equal(bits[0] + bits[1] + bits[2], v.astype(np.float64))

    def f64(h):
        return (np.asarray(h).astype(np.uint32) << 16).view(np.float32).astype(np.float64)
    kg = 1 if nf == 1 else 2
    K = 16 * kg
    pk = _kde_pack_b32(pts * c).view(np.uint16)
    rows = KDE_CHUNKS * _kde_cb(m) * 16
    assert _kde_cb(m) % 4 == 0
    assert pk.size == rows * K
    lanes = pk.reshape(rows // 32, kg, 64, 8)                 # lane l of block b, K group g
    a = np.zeros((rows, K))
    for g in range(kg):
        for l in range(64):
            k0 = 16 * g + 8 * (l >> 5)
            a[np.arange(rows // 32) * 32 + (l & 31), k0:k0 + 8] = f64(lanes[:, g, l])
    x = (parts * c).astype(np.float32)
    w = np.zeros((64, rows))
    for p in range(64):
        u = (2 * x[p]).astype(np.float32)
        sq = np.float32(0)
        for f in range(nf):
            sq = np.float32(sq + np.float32(x[p, f] * x[p, f]))
        b = np.zeros(K)
        for f in range(nf):
            sp = [f64(h)[0] for h in _bf16_split3(np.array([u[f]], np.float32))]
            for j in range(6):
                b[6 * f + j] = sp[_BF16_B[j]]
        b[6 * nf:6 * nf + 3] = -1.0
        b[6 * nf + 3:6 * nf + 6] = [f64(h)[0] for h in _bf16_split3(np.array([-sq], np.float32))]
        d = a @ b
        w[p] = np.exp2(d)
        # the float32 form of the same contraction (csrc kde_arg_rec, the pass-2 replica)
        yq = (pts * c).astype(np.float32)
        ysq = (yq.astype(np.float64) ** 2).sum(1).astype(np.float32)
        d32 = np.full(m, -sq, np.float32)
        for f in range(nf):
            d32 = (d32 + u[f] * yq[:, f]).astype(np.float32)
        d32 = (d32 - ysq).astype(np.float32)
        scale = np.abs(2 * x[p] @ yq.T) + ysq + sq
        assert (np.abs(d[:m] - d32) <= 4e-7 * scale + 1e-30).all()
    ref = np.exp(-0.5 * ((parts[:, None, :].astype(np.float64) - pts[None].astype(np.float64)) ** 2).sum(-1) / s ** 2)
    # the contraction's f32 rounding is absolute in the exponent: pairs 1e12 below the peak
    # weight (|x' - y'|^2 > 40) carry up to ~3e-5 relative with 4 features
    near = ref > 1e-12
    np.testing.assert_allclose(w[:, :m][near], ref[near], rtol=1e-5, atol=1e-30)
    np.testing.assert_allclose(w[:, :m], ref, rtol=3e-5, atol=1e-30)
    assert (w[:, m:] == 0).all()


def test_kde_records_carry_a_reversed_copy():
    """Records pack (csrc kde_scan): [4 + nb16 + KDE_REC_TAIL] forward rows (weight-0 padding
    around the points), then the points reversed in [nb16 + KDE_REC_TAIL] rows, so backward
    scans walk forward and a trip of 4 plus its prefetch never leaves the array."""
    from vectorizedbayesiannetwork_amd.plan import KDE_REC_TAIL, _kde_pack
    rng = np.random.default_rng(3)
    for m, nf in ((1, 1), (37, 2), (64, 3)):
        y = rng.normal(size=(m, nf)).astype(np.float32)
        r = _kde_pack([y], records=True)
        nb16 = (m + 15) // 16 * 16
        assert r.shape == (4 + nb16 + KDE_REC_TAIL + nb16 + KDE_REC_TAIL, 4)
        fwd, rev = r[4:4 + m], r[4 + nb16 + KDE_REC_TAIL:]
        np.testing.assert_array_equal(fwd[:, :nf], y)
        np.testing.assert_array_equal(rev[:m], fwd[::-1])
        pad = np.ones(len(r), bool)
        pad[4:4 + m] = False
        pad[4 + nb16 + KDE_REC_TAIL:4 + nb16 + KDE_REC_TAIL + m] = False
        assert (r[pad, nf] == np.float32(1e30)).all()


def test_normal_pairs_are_consecutive_and_class_pure():
    """plan._pair_normals: every VBN_F_BM_FIRST step is followed (not necessarily adjacently) by
    its VBN_F_BM_SECOND step before any other FIRST, both are one-dimensional gaussian LATENT
    steps of the same F_SHARED class, and FIXED / other-kind steps are never flagged."""
    import networkx as nx
    from vectorizedbayesiannetwork_amd import synthetic
    from vectorizedbayesiannetwork_amd.model import random_init_model
    from vectorizedbayesiannetwork_amd.plan import (F_BM_FIRST, F_BM_SECOND, F_SHARED, KIND_ID, MODE_MCM,
                                                    ROLE_LATENT, S_FLAGS, S_KIND, S_OUTDIM, S_ROLE,
                                                    PackedModel, build_plan)
    g = synthetic.random_dag(20, seed=0)
    data = synthetic.sem_data(g, 512, seed=0)
    kinds = synthetic.round_robin_kinds(g, ["gaussian_nn", "linear_gaussian", "mdn", "softmax_nn"])
    pk = PackedModel(random_init_model(g, kinds, data, seed=0), "cpu")
    topo = pk.model.topo
    ev = set(topo[3::5])
    plan = build_plan(pk, latent=[n for n in topo if n not in ev], fixed=list(ev), logp=[topo[-1]],
                      out_nodes=[topo[-1]], shared_roots=True, mode=MODE_MCM)
    rows = plan.steps.cpu().numpy()
    open_first = None
    n_pairs = 0
    for r in rows:
        f = int(r[S_FLAGS])
        if f & (F_BM_FIRST | F_BM_SECOND):
            assert r[S_ROLE] == ROLE_LATENT and r[S_OUTDIM] == 1
            assert r[S_KIND] in (KIND_ID["gaussian_nn"], KIND_ID["linear_gaussian"], KIND_ID["mdn"], KIND_ID["kde"])
        if f & F_BM_FIRST:
            assert open_first is None
            open_first = f & F_SHARED
        if f & F_BM_SECOND:
            assert open_first is not None and open_first == (f & F_SHARED)
            open_first = None
            n_pairs += 1
    assert open_first is None and n_pairs >= 3
