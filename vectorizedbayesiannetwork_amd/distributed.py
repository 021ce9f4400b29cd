"""Query-sharded data parallelism: one process per GPU over ``torch.distributed``.

Queries are independent, so the batch is split into contiguous shards and each rank walks
its own shard with no data-path collective.  Two things keep the result
identical to a single-GPU run of the whole batch:

* every rank uses the same RNG seed and its shard's global query offset (``q_base``) keys the
  per-query Philox streams; root-node draws that the reference shares across the batch (Q5)
  are keyed without the query and so agree.  The seed of each call comes from a
  rank-replicated generator seeded once from rank 0's torch generator (one 8-byte broadcast
  on the first call), so later calls need no collective and no host sync;
* the importance-sampling fallback stays batch-global (Q6): the per-rank "any ESS below
  threshold" flag is all-reduced with MAX (a 4-byte RCCL all-reduce) before deciding.

``gather=True`` additionally collects pdf/samples on ``dst`` (RCCL gather over xGMI: every
peer sends its shard over its own link to ``dst``, straight into one preallocated
``[world, shard, ...]`` buffer whose view is the batch).  ``overlap=True`` issues the gather
asynchronously so that it runs on RCCL's stream while the next call's walk computes; the
returned tensors are then valid after :meth:`ShardedEngine.wait` (as with any
``async_op`` collective).  At most one call's gathers are in flight: the next call's gather
joins the previous one first (a stream wait on RCCL).  The same code runs on ``gloo`` (CPU collectives) for the
multi-process tests.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.distributed as dist

from .engines import Query, infer_batch_size

__all__ = ["shard_bounds", "shard_query", "ShardedEngine", "seed_stream"]


def seed_stream(base: int) -> torch.Generator:
    """The rank-replicated generator the per-call seeds of a :class:`ShardedEngine` come from."""
    return torch.Generator().manual_seed(int(base))


def shard_bounds(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous, balanced [b0, b1) of ``n`` queries for ``rank`` (first n % world ranks +1)."""
    q, r = divmod(n, world)
    b0 = rank * q + min(rank, r)
    return b0, b0 + q + (1 if rank < r else 0)


def shard_query(query, b0: int, b1: int) -> Query:
    ev = {k: v[b0:b1] for k, v in (query.evidence or {}).items()}
    do = {k: v[b0:b1] for k, v in (getattr(query, "do", None) or {}).items()}
    return Query(target=query.target, evidence=ev, do=do)


def _slice_rows(t, axis: int, b0: int, b1: int, n_total: int):
    """Rows [b0, b1) of a per-query tensor along ``axis``; a broadcast (size-1) axis is kept."""
    if t is None or not isinstance(t, torch.Tensor):
        return t
    if t.dim() <= axis or t.shape[axis] == 1:
        return t
    if t.shape[axis] != n_total:
        raise ValueError(f"injected noise has {t.shape[axis]} rows on axis {axis}, expected {n_total} or 1")
    return t.narrow(axis, b0, b1 - b0)


def slice_noise(noise, b0: int, b1: int, n_total: int):
    """Shard injected draws (``_noise`` / ``_noise_fallback``) with the queries.

    Forms (engines.noise_tensor, GibbsSampler.sample): a dict node -> (slot0, slot1) of
    [B|1, S(, D)] tensors (batch axis 0); a walk tensor [n_latent, 2, B|1, S, Dmax] (axis 2);
    a Gibbs pair (init, sweep) with init in either walk form and sweep
    [iters, n_noise, 2, B, 8, Dmax] (axis 3).
    """
    if noise is None:
        return None
    if isinstance(noise, dict):
        return {k: tuple(_slice_rows(v, 0, b0, b1, n_total) for v in vs) for k, vs in noise.items()}
    if isinstance(noise, (tuple, list)) and len(noise) == 2:          # Gibbs (init, sweep)
        init, sweep = noise
        if sweep is not None and (not isinstance(sweep, torch.Tensor) or sweep.dim() != 6):
            raise ValueError("Gibbs sweep noise must be [iters, n_noise, 2, B, 8, Dmax]")
        return (slice_noise(init, b0, b1, n_total), _slice_rows(sweep, 3, b0, b1, n_total))
    if isinstance(noise, torch.Tensor) and noise.dim() == 5:
        return _slice_rows(noise, 2, b0, b1, n_total)
    raise ValueError("unrecognised injected-noise form for a sharded call")


def _world(group) -> Tuple[int, int]:
    if not dist.is_available() or not dist.is_initialized():
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


class ShardedEngine:
    """Wrap an engine (``infer_posterior`` or ``sample``) for query-sharded multi-GPU runs."""

    def __init__(self, engine, group=None, gather: bool = False, dst: int = 0, overlap: bool = False,
                 force_collectives: bool = False, verify: bool = False):
        self.engine = engine
        # verify=True: before each call, all-gather (call index, method, batch size, target) and
        # raise on any rank that disagrees -- ranks issuing different collective sequences would
        # otherwise hang in a collective another rank never issues (one 32-byte all-gather per
        # call; bench.py turns it on outside its timed region)
        self.verify = bool(verify)
        # issue the seed broadcast, flag all-reduce and gathers even in a world of one rank (an
        # initialised process group of size 1: the RCCL code path on a one-GPU box, tests)
        self.force_collectives = bool(force_collectives)
        self.group = group
        self.gather = bool(gather)
        self.dst = int(dst)
        self.overlap = bool(overlap)
        self._gen: Optional[torch.Generator] = None
        self._pending = []
        self.last_seed: Optional[int] = None
        self.gather_bytes = 0           # bytes dst received from its peers over all calls (bench.py)
        self._calls = 0                 # calls made (tags the pending gathers)

    def _device(self):
        backend = dist.get_backend(self.group) if dist.is_initialized() else "gloo"
        if backend == "nccl":
            return torch.device("cuda", torch.cuda.current_device())
        return torch.device("cpu")

    def _shared_seed(self, kwargs) -> int:
        """The call's seed, identical on every rank without a per-call collective: an explicit
        ``seed=``; else a wrapped engine's own deterministic sequence (``engine.seed`` set: seed +
        call index, as the unsharded engine would use); else the rank-replicated stream, seeded
        once from rank 0's torch generator (so ``torch.manual_seed`` before the FIRST call fixes
        every later call's seed; later reseeding does not change the stream)."""
        if kwargs.get("seed") is not None:
            return int(kwargs["seed"])
        if getattr(self.engine, "seed", None) is not None and hasattr(self.engine, "_seed"):
            return int(self.engine._seed({}))
        if self._gen is None:                        # once: rank 0's draw, broadcast
            rank, world = _world(self.group)
            s = torch.randint(0, 2 ** 62, (1,), dtype=torch.int64)
            if world > 1 or (self.force_collectives and dist.is_initialized()):
                s = s.to(self._device())
                dist.broadcast(s, src=dist.get_global_rank(self.group, 0) if self.group is not None else 0,
                               group=self.group)
            self._gen = seed_stream(int(s.item()))
        return int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64, generator=self._gen).item())

    def wait(self) -> None:
        """Order the current stream after every pending (``overlap=True``) gather."""
        for _, w in self._pending:
            w.wait()
        self._pending.clear()

    def _flag_reducer(self):
        rank, world = _world(self.group)
        if world == 1 and not (self.force_collectives and dist.is_initialized()):
            return None
        dev = self._device()

        def reduce(flag: torch.Tensor) -> torch.Tensor:
            f = flag.to(device=dev, dtype=torch.int32).reshape(1)
            dist.all_reduce(f, op=dist.ReduceOp.MAX, group=self.group)
            return f[0] > 0
        return reduce

    def _set_base(self, b0: int) -> None:
        self.engine.q_base = b0
        lw = getattr(self.engine, "_lw", None)
        if lw is not None:
            lw.q_base = b0

    def _gather(self, t: torch.Tensor, n_total: int) -> Optional[torch.Tensor]:
        rank, world = _world(self.group)
        b0, b1 = shard_bounds(n_total, rank, world)
        forced = self.force_collectives and dist.is_initialized()
        if (world == 1 and not forced) or t.shape[0] != b1 - b0:   # e.g. MCM root target: (1, S)
            return t
        dev = self._device()
        q_max = -(-n_total // world)
        src = t.to(dev).contiguous()
        if src.shape[0] != q_max:                     # ragged last shards: pad to q_max rows
            pad = torch.zeros((q_max,) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
            pad[: src.shape[0]] = src
            src = pad
        out = parts = None
        if rank == self.dst:
            out = torch.empty((world, q_max) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
            parts = list(out.unbind(0))
        if self.overlap and self._pending and self._pending[-1][0] != self._calls:
            # at most one earlier call's gathers in flight: join them before issuing this call's
            # (RCCL: the current stream waits, the host does not; gloo: the host waits).  Ranks
            # that never wait() -- every non-destination rank -- pile up no Works, and gloo's
            # queue of matched async collectives stays one call deep
            self.wait()
        work = dist.gather(src, parts, dst=self.dst, group=self.group, async_op=self.overlap)
        if rank == self.dst:
            self.gather_bytes += (world - 1) * src.numel() * src.element_size()   # received from peers
        if self.overlap:
            self._pending.append((self._calls, work))
        if rank != self.dst:
            return None
        if n_total == world * q_max:                  # equal shards: the buffer is the batch
            return out.view((n_total,) + tuple(t.shape[1:]))
        self.wait()
        sizes = [shard_bounds(n_total, r, world) for r in range(world)]
        return torch.cat([out[r, : b1 - b0] for r, (b0, b1) in enumerate(sizes)], dim=0)

    def _shard_kwargs(self, kwargs, b0: int, b1: int, n_total: int) -> dict:
        kw = dict(kwargs)
        kw["seed"] = self.last_seed = self._shared_seed(kwargs)
        for k in ("_noise", "_noise_fallback"):
            if k in kw:
                kw[k] = slice_noise(kw[k], b0, b1, n_total)
        if kw.get("_resample_u"):                    # RIS resampling uniforms, [B, S] each
            kw["_resample_u"] = [_slice_rows(u, 0, b0, b1, n_total) for u in kw["_resample_u"]]
        return kw

    def _check(self, n_total: int, world: int, method: int = 0, target=None) -> None:
        if n_total < world:
            raise ValueError(f"{n_total} queries cannot be sharded over {world} ranks")
        if not self.verify or not dist.is_initialized() or (world == 1 and not self.force_collectives):
            return
        import zlib
        tag = zlib.crc32(repr(target).encode()) & 0x7FFFFFFF
        mine = torch.tensor([self._calls + 1, method, n_total, tag], dtype=torch.int64, device=self._device())
        outs = [torch.empty_like(mine) for _ in range(dist.get_world_size(self.group))]
        dist.all_gather(outs, mine, group=self.group)
        rows = [tuple(int(v) for v in o.tolist()) for o in outs]
        if any(r != rows[0] for r in rows):
            raise RuntimeError("ShardedEngine: ranks disagree on the collective sequence "
                               f"(call, method, n_queries, target tag) per rank: {rows}")

    def infer_posterior(self, vbn, query, **kwargs):
        rank, world = _world(self.group)
        n_total = infer_batch_size(query.evidence, getattr(query, "do", None))
        self._check(n_total, world, 1, query.target)
        self._calls += 1
        b0, b1 = shard_bounds(n_total, rank, world)
        self._set_base(b0)
        kw = self._shard_kwargs(kwargs, b0, b1, n_total)
        red = self._flag_reducer()
        if red is not None:
            kw["_reduce_flag"] = red
        pdf, xs = self.engine.infer_posterior(vbn, shard_query(query, b0, b1), **kw)
        if not self.gather:
            return pdf, xs
        return self._gather(pdf, n_total), self._gather(xs, n_total)

    def sample(self, vbn, query, n_samples=None, **kwargs):
        rank, world = _world(self.group)
        n_total = infer_batch_size(query.evidence, getattr(query, "do", None))
        self._check(n_total, world, 2, query.target)
        self._calls += 1
        b0, b1 = shard_bounds(n_total, rank, world)
        self._set_base(b0)
        kw = self._shard_kwargs(kwargs, b0, b1, n_total)
        xs = self.engine.sample(vbn, shard_query(query, b0, b1), n_samples, **kw)
        if not self.gather or isinstance(xs, dict):
            return xs
        return self._gather(xs, n_total)
