"""Query-sharded multi-process path on CPU (gloo, world_size 2).

The local engine is a deterministic CPU stand-in with the accelerated engines' interface
(``q_base`` + ``seed`` + optional ``_reduce_flag``), so the test checks the sharding,
seed broadcast, batch-global fallback decision and the gather exactly.
"""
import os
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from vectorizedbayesiannetwork_amd.distributed import ShardedEngine, shard_bounds
from vectorizedbayesiannetwork_amd.engines import Query

S = 6


class StubEngine:
    """pdf[b, s] depends on (global query, sample, seed); a 'fallback' flips the sign when any
    query of the WHOLE batch has evidence > 10 (batch-global decision, like IS -> LW)."""

    def __init__(self):
        self.q_base = 0
        self.last_fallback = None

    def infer_posterior(self, vbn, query, seed=None, _reduce_flag=None, **kw):
        ev = query.evidence["x"]
        b = ev.shape[0]
        q = torch.arange(self.q_base, self.q_base + b, dtype=torch.float64).unsqueeze(1)
        s = torch.arange(S, dtype=torch.float64).unsqueeze(0)
        pdf = torch.sin(q * 1.7 + s * 0.3 + (seed % 1000) * 1e-3).float()
        flag = (ev > 10).any()
        if _reduce_flag is not None:
            flag = _reduce_flag(flag)
        self.last_fallback = bool(flag)
        if bool(flag):
            pdf = -pdf
        return pdf, (pdf.unsqueeze(-1) + ev.unsqueeze(1))


def _expected_seed(calls: int = 1) -> int:
    """The seed of call ``calls`` of a ShardedEngine: rank 0's first torch draw (seeded 123),
    broadcast once, seeds the rank-replicated stream the per-call seeds come from."""
    from vectorizedbayesiannetwork_amd.distributed import seed_stream
    torch.manual_seed(123)
    gen = seed_stream(int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item()))
    for _ in range(calls):
        seed = int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64, generator=gen).item())
    return seed


def _val(t):
    """A tensor sent through an mp.Queue by value: torch pickles tensors as shared-memory fds
    served by the sending process, which may have exited before the parent unpickles (a
    ConnectionResetError); numpy arrays pickle their bytes."""
    return None if t is None else t.detach().cpu().numpy().copy()


def _ten(a):
    return None if a is None else torch.from_numpy(a)


def _rendezvous():
    """A fresh file:// rendezvous for one world (no TCP port to race for between tests)."""
    return "file://" + os.path.join(tempfile.mkdtemp(prefix="vbn_gloo_"), "store")


def _worker(rank, world, init, ev, out_q, calls=1, overlap=False):
    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    try:
        torch.manual_seed(123 + rank)                 # ranks disagree; the seed is broadcast
        eng = ShardedEngine(StubEngine(), gather=True, overlap=overlap)
        for _ in range(calls):                        # later calls: no collective for the seed
            pdf, xs = eng.infer_posterior(None, Query(target="y", evidence={"x": ev}, do={}))
        eng.wait()
        out_q.put((rank, _val(pdf), _val(xs), eng.engine.last_fallback))
    finally:
        dist.destroy_process_group()


def _run(ev, world=2, calls=1, overlap=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    init = _rendezvous()
    procs = [ctx.Process(target=_worker, args=(r, world, init, ev, q, calls, overlap)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    return sorted([(r, _ten(a), _ten(b), fb) for r, a, b, fb in res], key=lambda r: r[0])


@pytest.mark.parametrize("ragged", [False, True])
def test_gloo_world2_overlapped_gather_third_call(ragged):
    """overlap=True (async gather, results valid after wait()) on the third call: seeds come
    from the replicated stream, equal shards gather straight into the batch buffer."""
    ev = torch.linspace(-1, 1, 7 if ragged else 8).unsqueeze(1)
    (r0, pdf, xs, fb0), (r1, pdf1, xs1, fb1) = _run(ev, calls=3, overlap=True)
    assert pdf1 is None and xs1 is None
    rpdf, rxs = StubEngine().infer_posterior(None, Query(target="y", evidence={"x": ev}, do={}),
                                             seed=_expected_seed(3))
    assert torch.equal(pdf, rpdf) and torch.equal(xs, rxs)


def test_shard_bounds_cover_batch():
    for n in (2, 5, 8, 4096, 4097):
        for w in (1, 2, 3, 8):
            if n < w:
                continue
            spans = [shard_bounds(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


@pytest.mark.parametrize("hot", [False, True])
def test_gloo_world2_matches_single_process(hot):
    ev = torch.linspace(-1, 1, 7).unsqueeze(1)
    if hot:
        ev[6, 0] = 50.0                               # only rank 1 sees it; fallback is global
    res = _run(ev)
    (r0, pdf, xs, fb0), (r1, pdf1, xs1, fb1) = res
    assert pdf1 is None and xs1 is None                # gathered on rank 0 only
    assert fb0 == fb1 == hot
    seed = _expected_seed()
    ref = StubEngine()
    rpdf, rxs = ref.infer_posterior(None, Query(target="y", evidence={"x": ev}, do={}), seed=seed)
    assert torch.equal(pdf, rpdf)
    assert torch.equal(xs, rxs)


class StubChainSampler:
    """Sampler interface of GibbsSampler (``sample(vbn, query, n_samples, seed=...)`` with
    chains keyed by the global query index ``q_base + b``): a deterministic [b, n, 1] chain."""

    def __init__(self):
        self.q_base = 0

    def sample(self, vbn, query, n_samples=None, seed=None, **kw):
        ev = query.evidence["x"]
        b = ev.shape[0]
        q = torch.arange(self.q_base, self.q_base + b, dtype=torch.float64).view(b, 1, 1)
        t = torch.arange(n_samples, dtype=torch.float64).view(1, -1, 1)
        return (torch.cos(q * 0.9 + t * 0.2 + (seed % 1000) * 1e-3) + ev.view(b, 1, 1)).float()


def _chain_worker(rank, world, init, ev, out_q):
    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    try:
        torch.manual_seed(123 + rank)
        eng = ShardedEngine(StubChainSampler(), gather=True)
        xs = eng.sample(None, Query(target="y", evidence={"x": ev}, do={}), 5)
        out_q.put((rank, _val(xs)))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_sharded_chains_match_single_process():
    """Gibbs chains shard by query with no data-path collective; the gather rebuilds the batch."""
    ev = torch.linspace(-1, 1, 5).unsqueeze(1)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    init = _rendezvous()
    procs = [ctx.Process(target=_chain_worker, args=(r, 2, init, ev, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    (_, xs), (_, xs1) = res
    xs = _ten(xs)
    assert xs1 is None
    seed = _expected_seed()
    ref = StubChainSampler().sample(None, Query(target="y", evidence={"x": ev}, do={}), 5, seed=seed)
    assert torch.equal(xs, ref)


def test_slice_noise_forms():
    """Injected draws shard with the queries (ShardedEngine._shard_kwargs): node dicts on axis
    0, walk tensors [n_latent, 2, B, S, Dmax] on axis 2, Gibbs (init, sweep) pairs with the
    sweep [iters, n_noise, 2, B, 8, Dmax] on axis 3; broadcast (size-1) batch axes are kept."""
    from vectorizedbayesiannetwork_amd.distributed import slice_noise
    B = 5
    d = {"a": (torch.arange(B * 3.0).view(B, 3), torch.zeros(1, 3)), "b": (None, torch.ones(B, 3, 2))}
    s = slice_noise(d, 1, 4, B)
    assert torch.equal(s["a"][0], d["a"][0][1:4]) and s["a"][1].shape == (1, 3)
    assert s["b"][0] is None and torch.equal(s["b"][1], d["b"][1][1:4])
    w = torch.randn(2, 2, B, 3, 1)
    assert torch.equal(slice_noise(w, 2, 5, B), w[:, :, 2:5])
    sweep = torch.randn(4, 3, 2, B, 8, 1)
    init, sw = slice_noise((w, sweep), 0, 2, B)
    assert torch.equal(init, w[:, :, :2]) and torch.equal(sw, sweep[:, :, :, :2])
    assert slice_noise((None, None), 0, 2, B) == (None, None)
    with pytest.raises(ValueError):
        slice_noise(torch.randn(2, 2, B + 1, 3, 1), 0, 2, B)
    with pytest.raises(ValueError):
        slice_noise((w, torch.randn(3, B)), 0, 2, B)


class SeededStub(StubEngine):
    """A stub with the engines' own deterministic seed sequence (``seed`` set: seed + call)."""

    def __init__(self, seed):
        super().__init__()
        self.seed = seed
        self._calls = 0

    def _seed(self, kwargs):
        s = self.seed + self._calls
        self._calls += 1
        return s


def _seeded_worker(rank, world, init, ev, out_q, calls):
    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    try:
        torch.manual_seed(999 + rank)                 # irrelevant: the engine's own sequence rules
        eng = ShardedEngine(SeededStub(4242), gather=True, overlap=True)
        outs, pending = [], []
        for _ in range(calls):
            pdf, xs = eng.infer_posterior(None, Query(target="y", evidence={"x": ev}, do={}))
            pending.append(len(eng._pending))
            if pdf is not None:
                eng.wait()
                outs.append(_val(pdf))
        out_q.put((rank, outs, pending, eng.gather_bytes))
    finally:
        dist.destroy_process_group()


def test_gloo_sharded_engine_keeps_a_seeded_engines_sequence():
    """A wrapped engine with ``seed`` set keeps its own sequence (seed + call index) on every
    rank, so sharded calls equal the unsharded engine's; non-destination ranks that never
    wait() hold no unbounded list of finished gathers; rank 0 counts the bytes it receives."""
    ev = torch.linspace(-1, 1, 8).unsqueeze(1)
    calls = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    init = _rendezvous()
    procs = [ctx.Process(target=_seeded_worker, args=(r, 2, init, ev, q, calls)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    (_, outs, _, nbytes), (_, outs1, pending1, _) = res
    ref = SeededStub(4242)
    for k in range(calls):
        rpdf, _ = ref.infer_posterior(None, Query(target="y", evidence={"x": ev}, do={}), seed=ref._seed({}))
        assert torch.equal(_ten(outs[k]), rpdf)
    assert outs1 == [] and max(pending1) <= 2, pending1           # one call (pdf + samples) in flight
    shard = 4 * S * 4 + 4 * S * 1 * 4                 # pdf [4, S] + samples [4, S, 1] fp32 from rank 1
    assert nbytes == calls * shard


def _verify_worker(rank, world, init, out_q):
    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    try:
        eng = ShardedEngine(StubEngine(), gather=True, verify=True)
        ev = torch.linspace(-1, 1, 8).unsqueeze(1)
        pdf, _ = eng.infer_posterior(None, Query(target="y", evidence={"x": ev}, do={}))
        ok = pdf is not None or rank != 0
        # the second call diverges: rank 1 queries another target (a different plan, and in a
        # real engine possibly another collective sequence) -- every rank must refuse it
        try:
            eng.infer_posterior(None, Query(target="y" if rank == 0 else "z", evidence={"x": ev}, do={}))
            err = None
        except RuntimeError as e:
            err = str(e)
        out_q.put((rank, ok, err))
    finally:
        dist.destroy_process_group()


def test_gloo_verify_refuses_diverging_calls():
    """ShardedEngine(verify=True): a call some rank issues differently raises on every rank
    (instead of a collective one rank never joins)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    init = _rendezvous()
    procs = [ctx.Process(target=_verify_worker, args=(r, 2, init, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    for rank, ok, err in res:
        assert ok
        assert err is not None and "disagree" in err, (rank, err)
