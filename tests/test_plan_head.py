"""Host-side packing of the NN fast paths (no GPU): the layer-1 operand bound and the split-f16
MFMA head fragments of wide heads (plan._pack_mlp; csrc mlp_l1_act / head_mfma)."""
import numpy as np
import pytest

from vectorizedbayesiannetwork_amd import synthetic
from vectorizedbayesiannetwork_amd.model import random_init_model
from vectorizedbayesiannetwork_amd.plan import (F_HEAD_MFMA, MODE_WEIGHTED, S_FLAGS, S_KIND,
                                                S_NOUT, S_OFF_KQ, S_OFF_KQY, PackedModel, _ROWS, build_plan)


def _model():
    g = synthetic.random_dag(10, seed=4)
    data = synthetic.sem_data(g, 256, seed=0)
    kinds = synthetic.round_robin_kinds(g, ["mdn", "softmax_nn", "gaussian_nn"])
    return random_init_model(g, kinds, data, seed=0)


def _plan(model, pk):
    topo = model.topo
    return build_plan(pk, latent=list(topo[:-2]), fixed=list(topo[-2:]), logp=list(topo[-2:]),
                      out_nodes=[topo[0]], shared_roots=False, mode=MODE_WEIGHTED)


def test_wide_heads_carry_mfma_fragments(monkeypatch):
    import vectorizedbayesiannetwork_amd.plan as P
    monkeypatch.setattr(P, "HEAD_MFMA_MIN", 8)     # the packing of the (optional) MFMA head
    HEAD_MFMA_MIN = 8
    model = _model()
    pk = PackedModel(model, "cpu")
    plan = _plan(model, pk)
    steps = plan.steps.numpy()
    blob = pk.params.numpy()
    seen = 0
    for i, n in enumerate(model.topo):
        r = steps[i]
        rec = model.cpds[n]
        if not model.parents[n] or rec.kind not in ("mdn", "softmax_nn", "gaussian_nn"):
            assert not (r[S_FLAGS] & F_HEAD_MFMA)
            continue
        wide = HEAD_MFMA_MIN <= r[S_NOUT] <= 32
        assert bool(r[S_FLAGS] & F_HEAD_MFMA) == wide, (n, rec.kind, r[S_NOUT])
        if not wide:
            continue
        seen += 1
        off = int(r[S_OFF_KQY])
        assert off == pk.nodes[n].offs["w3h"] and off >= 0
        frag = blob[off:off + 1024].view(np.float16).reshape(4, 64, 8).astype(np.float32)
        (w3, b3) = [(np.asarray(w, np.float32), np.asarray(b, np.float32)) for w, b in rec.mlp_layers()[-1:]][0]
        n_out = w3.shape[0]
        w3p = np.zeros((32, 32), np.float32)
        w3p[:n_out] = w3
        j = np.arange(8)
        for s in range(2):
            for ln in range(64):
                want = w3p[ln & 31, 16 * s + 8 * (j >> 2) + 4 * (ln >> 5) + (j & 3)]
                got = frag[s, ln] + frag[2 + s, ln]                  # hi + lo
                assert np.allclose(got, want, rtol=1e-6, atol=1e-7)   # f16 lo parts may be subnormal
        b3p = np.zeros(32, np.float32)
        b3p[:n_out] = b3
        assert np.array_equal(blob[off + 1024:off + 1056].reshape(2, 16), b3p[_ROWS])
    assert seen > 0


def test_layer1_operand_bound_is_conservative():
    model = _model()
    pk = PackedModel(model, "cpu")
    plan = _plan(model, pk)
    steps = plan.steps.numpy()
    rng = np.random.default_rng(0)
    for i, n in enumerate(model.topo):
        if not model.parents[n] or "zlim" not in pk.nodes[n].offs:
            continue
        zlim = steps[i, S_OFF_KQ:S_OFF_KQ + 1].view(np.float32)[0]
        assert zlim == np.float32(pk.nodes[n].offs["zlim"])
        w1, b1 = [np.asarray(t, np.float64) for t in model.cpds[n].mlp_layers()[0]]
        if zlim <= 0:
            continue
        x = rng.uniform(-1, 1, size=(4096, w1.shape[1])) * min(float(zlim), 1e30)
        z = x @ w1.T + b1
        assert np.abs(z).max() <= 32768.0
