"""Host replica of the HIP walk's production RNG, as a draw provider for the oracle.

The production ("lean") walk never reads injected draws: each latent step makes its own
draws from counter-based Philox-2x32-10 (csrc/vbn_walk_impl.h ``rng_words``,
``draw_normal``, ``draw_uniforms``).  :class:`PhiloxDraws` recomputes exactly those words on
the host and hands them to the oracle (oracle/vbn_oracle.py) through the same
``normal / uniform / categorical / randint`` calls the reference makes, so the oracle runs
the reference op sequence on the kernel's own random numbers:

* key ``(uint32)seed + sid``, ``sid = (offset & 0xff) << 24 | node_id << 10 | dim << 2 |
  stream``; counter ``(sample, qkey ^ (seed >> 32))`` with ``qkey = 0`` for draws shared by
  every query (root nodes of MCM / LW / ancestral), else ``q_base + query + 1``;
* stream 0: a standard normal by Box-Muller on both words, ``r cos(2 pi u2)``; in lean walks
  a ``VBN_F_BM_FIRST`` step also yields ``r sin(2 pi u2)`` for the next ``VBN_F_BM_SECOND``
  step's dim-0 normal in the walk's order (plan.py ``_pair_normals``; the walk order may
  differ from the oracle's topological call order, plan.liveness_order);
* stream 1: two uniforms ``(w >> 8) * 2^-24``: word 0 picks the categorical / KDE index
  (inverse CDF: the smallest k with cumsum(p)[k] > u * sum(p)), word 1 is softmax_nn's
  within-bin uniform.

Categorical choices are made here from the *oracle's* probabilities (float64 inverse CDF);
the kernel makes them from its own fp32 probabilities, so a draw whose uniform lies within
rounding of a CDF boundary may pick the neighbouring class.  Every categorical draw's
distance to the nearest CDF boundary (in CDF units) is recorded per particle
(:meth:`PhiloxDraws.min_margin`), so a test can check that every particle where the GPU and
the oracle disagree is one with such a near-tie, and count them.
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np
import torch

MASK32 = np.uint64(0xFFFFFFFF)
F_ROOT, F_SHARED, F_BM_FIRST, F_BM_SECOND = 2, 4, 512, 1024
S_KIND, S_FLAGS, S_OUTDIM, S_NODEID = 0, 2, 7, 11
KIND_MDN, KIND_KDE, KIND_SOFTMAX = 2, 3, 4


def philox2x32(c0, c1, key):
    """Philox-2x32-10 (Random123), vectorised; csrc ``philox2x32``."""
    c0 = np.asarray(c0).astype(np.uint64) & MASK32
    c1 = np.asarray(c1).astype(np.uint64) & MASK32
    k = np.asarray(key).astype(np.uint64) & MASK32
    for _ in range(10):
        p = c0 * np.uint64(0xD256D193)
        c0, c1 = ((p >> np.uint64(32)) ^ k ^ c1) & MASK32, p & MASK32
        k = (k + np.uint64(0x9E3779B9)) & MASK32
    return c0, c1


def u01(w) -> np.ndarray:
    """csrc ``u01``: (w >> 8) * 2^-24, exact in fp32."""
    return ((np.asarray(w, np.uint64) >> np.uint64(8)).astype(np.float64) * 2.0 ** -24).astype(np.float32)


def box_muller_pair(a, b):
    """(r cos(2 pi u2), r sin(2 pi u2)) of csrc ``box_muller`` / ``draw_normal`` (float64
    here; the device's v_log / v_sqrt / v_cos approximations differ by ~1e-7 relative)."""
    u1 = ((np.asarray(a, np.uint64) >> np.uint64(8)) + np.uint64(1)).astype(np.float64) * 2.0 ** -24
    u2 = (np.asarray(b, np.uint64) >> np.uint64(8)).astype(np.float64) * 2.0 ** -24
    r = np.sqrt(-2.0 * np.log(u1))
    return (r * np.cos(2 * np.pi * u2)).astype(np.float32), (r * np.sin(2 * np.pi * u2)).astype(np.float32)


class PhiloxDraws:
    """Draw provider for the oracle that replays a lean walk's Philox draws.

    ``steps``: the walk's step table (``QueryPlan.steps``, [n_steps, 32] int32) -- it gives
    each node's ``node_id`` and flags (shared draws, Box-Muller pairing); ``node_ids``: node
    name -> ``PackedModel.node_id``; ``n_queries`` x ``n_samples``: the walk's batch.
    """

    def __init__(self, steps, node_ids: Dict[str, int], *, seed: int, offset: int = 0, q_base: int = 0,
                 n_queries: int, n_samples: int, lean: bool = True):
        rows = steps.detach().cpu().numpy() if isinstance(steps, torch.Tensor) else np.asarray(steps)
        self.row_of = {int(r[S_NODEID]): r for r in rows}
        # a VBN_F_BM_SECOND step takes r sin of the nearest VBN_F_BM_FIRST step before it in the
        # walk's order (plan._pair_normals), whatever order the oracle calls the nodes in
        self.partner = {}
        first = None
        for r in rows:
            if int(r[S_FLAGS]) & F_BM_FIRST:
                first = r
            elif int(r[S_FLAGS]) & F_BM_SECOND:
                self.partner[int(r[S_NODEID])] = first
        self.node_ids = dict(node_ids)
        self.seed = int(seed) & ((1 << 64) - 1)
        self.offset = int(offset)
        self.q_base = int(q_base)
        self.B = int(n_queries)
        self.S = int(n_samples)
        self.lean = bool(lean)
        self.margin = np.full((self.B, self.S), np.inf)
        self.n_categorical = 0
        self._row = None
        self._query: Optional[int] = None
        self._c0 = self._c1 = 0

    # -- oracle hook ---------------------------------------------------------------------
    def begin_node(self, node: str, query: Optional[int] = None) -> None:
        self._row = self.row_of[self.node_ids[node]]
        self._query = query
        self._c0 = self._c1 = 0

    def min_margin(self) -> np.ndarray:
        """[B, S] smallest distance (CDF units) of any categorical draw to a class boundary."""
        return self.margin

    # -- helpers -------------------------------------------------------------------------
    @property
    def _shared(self) -> bool:
        return bool(self._row[S_FLAGS] & F_SHARED)

    def _elements(self, start: int, count: int, per_particle: int):
        """Element e of the current node's draw call -> (query, sample, dim) of the walk."""
        e = start + np.arange(count)
        p, d = e // per_particle, e % per_particle
        qi, s = p // self.S, p % self.S
        q = qi + (self._query or 0)
        return q, s, d

    def _words(self, q, s, d, stream: int, row=None):
        if self._row is None:
            raise RuntimeError("PhiloxDraws: draw before begin_node")
        row = self._row if row is None else row
        node_id = int(row[S_NODEID])
        sid = ((self.offset & 0xFF) << 24) | (node_id << 10) | (np.asarray(d, np.int64) << 2) | stream
        qkey = np.zeros_like(q) if (int(row[S_FLAGS]) & F_SHARED) else (self.q_base + q + 1)
        c1 = (qkey.astype(np.uint64) & MASK32) ^ np.uint64((self.seed >> 32) & 0xFFFFFFFF)
        key = (np.uint64(self.seed & 0xFFFFFFFF) + sid.astype(np.uint64)) & MASK32
        return philox2x32(s, c1, key)

    def _note_margin(self, q, s, margin) -> None:
        if self._shared:                                    # the same draw for every query
            for qq in range(self.B):
                np.minimum.at(self.margin, (np.full_like(s, qq), s), margin)
        else:
            np.minimum.at(self.margin, (q, s), margin)

    def _inv_cdf(self, probs: torch.Tensor, u: np.ndarray, q, s) -> torch.Tensor:
        p = probs.detach().double().cpu().numpy()
        k = p.shape[1]
        cdf = np.cumsum(p, axis=1)
        tot = cdf[:, -1]
        thr = u.astype(np.float64) * tot
        inner = cdf[:, : k - 1]
        idx = (inner <= thr[:, None]).sum(axis=1)           # smallest k with cdf[k] > thr, else K-1
        if k > 1:
            lo = np.take_along_axis(inner, np.clip(idx - 1, 0, k - 2)[:, None], 1)[:, 0]
            hi = np.take_along_axis(inner, np.clip(idx, 0, k - 2)[:, None], 1)[:, 0]
            lo_gap = np.where(idx > 0, np.abs(thr - lo), np.inf)
            hi_gap = np.where(idx < k - 1, np.abs(hi - thr), np.inf)
            margin = np.minimum(lo_gap, hi_gap) / np.where(tot > 0, tot, 1.0)
            self._note_margin(q, s, margin)
        self.n_categorical += len(idx)
        return torch.from_numpy(idx.astype(np.int64))

    # -- the reference's RNG calls -------------------------------------------------------
    def normal(self, shape) -> torch.Tensor:
        shape = tuple(int(x) for x in shape)
        count = int(np.prod(shape))
        per = shape[-1]
        q, s, d = self._elements(self._c1, count, per)
        self._c1 += count
        a, b = self._words(q, s, d, 0)
        cos, sin = box_muller_pair(a, b)
        out = cos.copy()
        fl = int(self._row[S_FLAGS])
        if self.lean and (fl & F_BM_SECOND):
            d0 = d == 0
            pa, pb = self._words(q[d0], s[d0], d[d0], 0, row=self.partner[int(self._row[S_NODEID])])
            out[d0] = box_muller_pair(pa, pb)[1]
        return torch.from_numpy(out.reshape(shape))

    def uniform(self, shape) -> torch.Tensor:               # softmax_nn within-bin uniform
        shape = tuple(int(x) for x in shape)
        count = int(np.prod(shape))
        q, s, d = self._elements(self._c1, count, shape[-1])
        self._c1 += count
        _, b = self._words(q, s, d, 1)
        return torch.from_numpy(u01(b).reshape(shape))

    def categorical(self, probs2d: torch.Tensor, replacement: bool = True) -> torch.Tensor:
        rows = int(probs2d.shape[0])
        per = int(self._row[S_OUTDIM]) if int(self._row[S_KIND]) == KIND_SOFTMAX else 1
        q, s, d = self._elements(self._c0, rows, per)
        self._c0 += rows
        a, _ = self._words(q, s, d, 1)
        return self._inv_cdf(probs2d, u01(a), q, s)

    def randint(self, n: int, count: int) -> torch.Tensor:  # root KDE: min(int(u * M), M - 1)
        q, s, d = self._elements(self._c0, int(count), 1)
        self._c0 += int(count)
        a, _ = self._words(q, s, d, 1)
        idx = np.minimum((u01(a) * np.float32(n)).astype(np.int64), n - 1)
        return torch.from_numpy(idx)

    def multinomial(self, probs2d: torch.Tensor, n: int) -> torch.Tensor:
        raise NotImplementedError("PhiloxDraws replays walk draws only (no resampling)")
