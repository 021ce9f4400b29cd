"""Plan packer: BNModel + query signature -> device step table, parameter blob, LDS slots.

The reference re-derives its topology per query signature in ``get_inference_state``
(reference ``vbn/inference/_core.py:57-109``: topo order, parent index tuples, column
slices, evidence/do masks) and re-reads CPD parameters inside every ATen call.  Here that
work is split in two device-resident objects:

* :class:`PackedModel` — once per model and device: every CPD's parameters packed into one
  fp32 blob in the fragment layouts the kernel reads (see ``csrc/vbn_walk_impl.h``), plus the
  host-side constants the reference recomputes per call (root loc/scale, mixture weights,
  KDE kernel scales), computed with the same torch fp32 ops so they are bit-identical.
* :class:`QueryPlan` — once per (query signature, engine mode): the ``vbn_step`` table
  (role / flags per node), parent-slot lists and output slots.  Node values live in LDS
  slots assigned by a liveness scan over the topological order, so a wave's LDS footprint
  is the peak number of simultaneously live columns, not the total DAG width.
"""
from __future__ import annotations

import hashlib
import math
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F

from .model import BNModel, CPDRecord

# ---- must match include/vbn_hip.h -------------------------------------------------------
KIND_ID = {"gaussian_nn": 0, "linear_gaussian": 1, "mdn": 2, "kde": 3, "softmax_nn": 4}
ROLE_SKIP, ROLE_LATENT, ROLE_FIXED, ROLE_PARAMS, ROLE_SELECT, ROLE_COLLECT = 0, 1, 2, 3, 4, 5
F_LOGP, F_ROOT, F_SHARED, F_STANDARDIZE, F_CLIP, F_F32L2, F_KDE_VALU = 1, 2, 4, 8, 16, 32, 64
F_KEEP, F_LPRESET, F_BM_FIRST, F_BM_SECOND, F_MLP_GENERIC = 128, 256, 512, 1024, 2048
ACT_ID = {"relu": 0, "tanh": 1, "gelu": 2, "elu": 3}
WITHIN_ID = {"uniform": 0, "triangular": 1, "gaussian": 2}
MODE_MCM, MODE_WEIGHTED, MODE_SAMPLE, MODE_GIBBS = 0, 1, 2, 3
STEP_INTS = 32
(S_KIND, S_ROLE, S_FLAGS, S_ACT, S_NIN, S_INOFF, S_OUTCOL, S_OUTDIM, S_FIXEDCOL, S_K, S_NOUT,
 S_NODEID, S_NOISE, S_AUX0, S_AUX1, S_AUX2, S_OFF_STD, S_OFF_W1, S_OFF_W2, S_OFF_B2, S_OFF_W3,
 S_OFF_B3, S_OFF_TAIL, S_OFF_PTS, S_OFF_W2H, S_OFF_KQ, S_OFF_KQY, S_OFF_KR, S_OFF_KV,
 S_WBLK_OFF, S_WBLK_LEN, S_RES7) = range(32)
WBLK_CHUNK = 256          # floats per LDS-DMA wave instruction (64 lanes x 16 B)
KDE_CHUNKS = 16
KDE_REC_TAIL = 16      # weight-0 record rows after the last point (csrc kde_scan: two trips of 4 ahead)
MLP_HIDDEN = (32, 32)
# heads at least this wide run on the split-f16 MFMA (csrc head_mfma; cfg3 walk 2.97 -> 2.74 ms,
# profiles/r03_bench/r03q_ab_cfg3.txt).  1 << 30 turns the MFMA head off.
HEAD_MFMA_MIN = 8
F_HEAD_MFMA = 4096
F_PRECOMP = 8192          # csrc VBN_F_PRECOMP: per-sample quantities read from the pre-pass
F_PRE_OUT = 16384         # csrc VBN_F_PRE_OUT: the pre-pass writes a node's per-sample quantities
F_PRECOMP_Q = 32768       # csrc VBN_F_PRECOMP_Q: with F_PRECOMP, per-QUERY quantities (precomp_q)
F_CLAMP_EV = 65536        # csrc VBN_F_CLAMP_EV: fixed value clamped in the kernel (clamp_evidence)
MAX_NODES = 1 << 14
MAX_NODE_DIMS = 1 << 8


def _row(r: int, h: int) -> int:
    """Row of the 32x32 MFMA accumulator held in register r by lane half h."""
    return (r & 3) + 8 * (r >> 2) + 4 * h


_ROWS = np.array([[_row(r, h) for r in range(16)] for h in range(2)])  # [2,16]


class _Blob:
    def __init__(self):
        self.parts: List[np.ndarray] = []
        self.size = 0

    def add(self, arr) -> int:
        a = np.ascontiguousarray(np.asarray(arr, dtype=np.float32).reshape(-1))
        off = self.size
        pad = (-a.size) % 4                      # keep every block 16-byte aligned
        if pad:
            a = np.concatenate([a, np.zeros(pad, np.float32)])
        self.parts.append(a)
        self.size += a.size
        return off

    def finish(self) -> np.ndarray:
        # one DMA chunk of slack: a weight block's last 1 KiB chunk may read past its end
        return np.concatenate(self.parts + [np.zeros(WBLK_CHUNK, np.float32)])


_KDE_C = math.sqrt(0.5 * math.log2(math.e))      # exp(-d^2 / 2) = exp2(-(c d)^2)


def _kde_cb(m: int) -> int:
    """16-point blocks per inverse-CDF chunk (a multiple of 4: whole pairs of the 32-point
    blocks of the MFMA pass; csrc kde_cb)."""
    nblk = (m + 15) // 16
    return ((nblk + KDE_CHUNKS - 1) // KDE_CHUNKS + 3) & ~3


def _kde_pack(feats: List[np.ndarray], records: bool = False) -> np.ndarray:
    """KDE point features y' (scaled) for the kernel (csrc/vbn_walk_impl.h, kde_mfma_sums).

    MFMA A-operand image: [KDE_CHUNKS * cb][4][16] fp32 (cb = _kde_cb(M) blocks per chunk),
    columns (y'_0 .. y'_{nf-1}, |y'|^2, 1) for nf <= 2 and (y'_0, y'_1, y'_2, |y'|^2) for
    nf == 3; padding points get |y'|^2 = 1e30, i.e. weight exp2(-1e30) = 0.
    ``records=True``: per-point rows (y'.., |y'|^2): [4 + 16 ceil(M/16) + 8][4] forward, then the
    points in reverse order [16 ceil(M/16) + 8][4], weight-0 rows around them (the inverse-CDF
    scan walks either array forward, two trips of 4 past a chunk end at most).
    """
    y = np.concatenate([f.reshape(f.shape[0], -1) for f in feats], axis=1).astype(np.float32)
    m, nf = y.shape
    if nf > 3:
        raise ValueError("kde MFMA pack supports at most 3 features")
    nblk = (m + 15) // 16
    rows = 4 + nblk * 16 + KDE_REC_TAIL if records else KDE_CHUNKS * _kde_cb(m) * 16
    a = np.zeros((rows, 4), np.float32)
    o = 4 if records else 0
    a[:, nf] = 1e30
    a[o:o + m, :nf] = y
    a[o:o + m, nf] = (y.astype(np.float64) ** 2).sum(axis=1).astype(np.float32)
    if records:
        rev = np.zeros((nblk * 16 + KDE_REC_TAIL, 4), np.float32)
        rev[:, nf] = 1e30
        rev[:m] = a[o:o + m][::-1]
        return np.concatenate([a, rev])
    if nf <= 2:
        a[:, nf + 1] = 1.0
    return a.reshape(rows // 16, 16, 4).transpose(0, 2, 1)


def _bf16_split3(v: np.ndarray):
    """f32 -> three bf16 (round to nearest even) whose sum is v exactly: hi = bf16(v),
    mid = bf16(v - hi), lo = v - hi - mid (8 significant bits left, exact); uint16 bits."""
    def rne(x):
        b = x.astype(np.float32).view(np.uint32).astype(np.uint64)
        return ((b + 0x7FFF + ((b >> 16) & 1)) >> 16).astype(np.uint16)

    def val(h):
        return (h.astype(np.uint32) << 16).view(np.float32)
    v = v.astype(np.float32)
    hi = rne(v)
    r1 = (v - val(hi)).astype(np.float32)
    mid = rne(r1)
    r2 = (r1 - val(mid)).astype(np.float32)
    lo = rne(r2)
    return hi, mid, lo


# bf16x3 slot pattern of one feature: A (point y') side and B (particle u = 2x') side, so the
# six products are u_h y_h, u_h y_m, u_m y_h, u_h y_l, u_l y_h, u_m y_m (csrc kde_bf16_sums)
_BF16_A = (0, 1, 0, 2, 0, 1)
_BF16_B = (0, 0, 1, 0, 2, 1)


def _kde_pack_b32(y: np.ndarray) -> np.ndarray:
    """Point pack of the bf16x3 pass (csrc kde_b32_sums): A operand of
    v_mfma_f32_32x32x16_bf16, rows = 32 points per block, K = 16 slots per point for one feature
    and 32 (two chained MFMAs) for 2-4: feature f at slots 6f .. 6f+5 (_BF16_A of its hi / mid /
    lo split), |y'|^2's hi / mid / lo at 6nf .. 6nf+2 (B side -1), 1.0 at 6nf+3 .. 6nf+5 (B
    side: the split of -|x'|^2), zero after.  Layout [block][K group g][half h][32 points][8
    slots] bf16: lane l = 32 h + n loads point n's slots 16 g + 8 h .. +7 as one 16-byte load;
    the points padded to KDE_CHUNKS * _kde_cb(M) * 16 (|y'|^2 = 1e30: weight 0), so a chunk is
    _kde_cb(M) / 2 blocks and its boundaries are the record scan's."""
    y = y.reshape(y.shape[0], -1).astype(np.float32)
    m, nf = y.shape
    if not 1 <= nf <= 4:
        raise ValueError("the bf16x3 KDE pack is for 1-4 features")
    kg = 1 if nf == 1 else 2
    rows = KDE_CHUNKS * _kde_cb(m) * 16
    feats = np.zeros((rows, nf), np.float32)
    feats[:m] = y
    sq = np.full(rows, 1e30, np.float32)
    sq[:m] = (y.astype(np.float64) ** 2).sum(axis=1).astype(np.float32)
    slots = np.zeros((rows, 16 * kg), np.uint16)
    for f in range(nf):
        sp = _bf16_split3(feats[:, f])
        for j in range(6):
            slots[:, 6 * f + j] = sp[_BF16_A[j]]
    for j, h in enumerate(_bf16_split3(sq)):
        slots[:, 6 * nf + j] = h
    slots[:, 6 * nf + 3:6 * nf + 6] = 0x3F80                   # bf16 1.0
    a = slots.reshape(rows // 32, 32, kg, 2, 8).transpose(0, 2, 3, 1, 4)   # [blk][g][h][32][8]
    return np.ascontiguousarray(a).reshape(-1).view(np.float32)


def _kde_pack_valu(y: np.ndarray) -> np.ndarray:
    """Point features y' for the VALU pass: [KDE_CHUNKS * csz / 8][nf][8] fp32 (csz = points
    per chunk, a multiple of 8; csrc kde_csz); padding points y' = 1e15 (weight 0)."""
    y = y.reshape(y.shape[0], -1).astype(np.float32)
    m, nf = y.shape
    csz = ((m + KDE_CHUNKS - 1) // KDE_CHUNKS + 7) & ~7
    a = np.full((KDE_CHUNKS * csz, nf), 1e15, np.float32)
    a[:m] = y
    return a.reshape(-1, 8, nf).transpose(0, 2, 1)


# ---- moment tables of one-feature KDE nodes (csrc kde_index_moments, round 6) ---------------
# Sampling needs, per particle u = 2 x' and chunk c, S_c(u) = sum_{j in c} exp2(u y'_j - |y'_j|^2)
# (the factored form of kde.py:172-177's softmax weights).  Around a grid centre u_g,
# exp2(u y') = exp2(u_g y') * exp(d ln2 y') with d = u - u_g, so
#   S_c(u) = sum_k d^k T[g][c][k],   T[g][c][k] = sum_{j in c} exp2(u_g y'_j - |y'_j|^2) (ln2 y'_j)^k / k!
# truncated after KDE_MT_TERMS terms: the remainder of each point's series is below
# |z|^K / K! e^|z| with |z| = |d| ln2 |y'_j| <= KDE_MT_Z, i.e. a relative error < 3e-8 on every
# weight, all of the same sign -- below the f32 rounding of the chunk sums.  The chunks are finer
# than the MFMA pass's 16 (KDE_MT_CHUNKS, ~M/64 points each), since a chunk costs 3 FMAs
# instead of its points' exps and the inverse-CDF scan then covers ~M/128 points instead of ~M/32.
KDE_MOMENTS = os.environ.get("VBN_KDE_MOMENTS", "1") != "0"      # A/B: 0 = MFMA pass 1 for every node
KDE_MT_TERMS = 4
KDE_MT_Z = 0.028                 # |d| ln2 max|y'| at the cell edge: 0.028^4 / 24 * e^0.028 < 3e-8
KDE_MT_CHUNKS = 64               # inverse-CDF chunks of a moment-table node (at most)
KDE_MT_MAX_CELLS = 16384         # table size bound (cells x 65 rows x 16 B: <= 17 MiB per node)
KDE_MT_EXP_MAX = 100.0           # largest log2 weight a cell may hold (f32 sums stay finite)
KDE_MT_EXP_MIN = -80.0           # every cell keeps a weight above 2^-80 (no all-underflow chunk set)
KDE_MT_HEADER = 8                # floats: u_lo, 1 / delta, delta, n_cells, n_chunks, chunk points
                                 # (the last three int32 bits), 0, 0


def kde_moment_cells(y: np.ndarray):
    """Grid of one-feature KDE parent points y' (float32, scaled): (u_lo, delta, inv_delta,
    n_cells) as float32 / int, the particle range u = 2 x' it covers being 2 [min y' - W,
    max y' + W] with W = max(span, 2) (a particle outside it takes the MFMA pass); None when
    the grid would exceed KDE_MT_MAX_CELLS or a cell's weights leave [2^-80, 2^100]."""
    y = np.asarray(y, np.float32).reshape(-1)
    y64 = y.astype(np.float64)
    sq = (y64 * y64).astype(np.float32).astype(np.float64)        # |y'|^2 as the records hold it
    ymax_abs = float(np.abs(y64).max())
    span = float(y64.max() - y64.min())
    w = max(span, 2.0)
    lo, hi = 2.0 * (float(y64.min()) - w), 2.0 * (float(y64.max()) + w)
    if ymax_abs == 0.0:
        delta = hi - lo
    else:
        delta = 2.0 * KDE_MT_Z / (math.log(2.0) * ymax_abs)
    delta32 = np.float32(delta)
    lo32 = np.float32(lo)
    n = int(math.ceil((hi - lo) / float(delta32))) + 1
    if n > KDE_MT_MAX_CELLS:
        return None
    centres = kde_moment_centres(lo32, delta32, n)
    # the largest log2 weight of each cell, u_g y' - |y'|^2 over the points (a max of lines in u)
    e_max = np.max(centres[:, None] * y64[None, :] - sq[None, :], axis=1)
    if e_max.max() > KDE_MT_EXP_MAX or e_max.min() < KDE_MT_EXP_MIN:
        return None
    return lo32, delta32, np.float32(1.0 / float(delta32)), n


def kde_moment_centres(lo32, delta32, n: int) -> np.ndarray:
    """Cell centres exactly as the kernel forms them: fmaf(g, delta, u_lo) in float32 (one
    rounding of the exact g * delta + u_lo, which float64 holds for g < 2^14)."""
    g = np.arange(n, dtype=np.float64)
    return (g * np.float64(delta32) + np.float64(lo32)).astype(np.float32).astype(np.float64)


def kde_moment_chunks(m: int) -> Tuple[int, int]:
    """(chunks, points per chunk) of a moment-table node of m points: ceil(m / 64) points per
    chunk, as many chunks as that takes (every chunk holds a point)."""
    per = -(-m // KDE_MT_CHUNKS)
    return -(-m // per), per


KDE_MT_GROUP = 8                 # chunks per group (the kernel locates a group, then its chunk)


def kde_moment_rows(n_chunks: int) -> int:
    """Rows per cell: the chunks, their groups of KDE_MT_GROUP, the whole point set."""
    return n_chunks + -(-n_chunks // KDE_MT_GROUP) + 1


def kde_moment_table(y: np.ndarray) -> Optional[np.ndarray]:
    """The moment table of one-feature KDE parent points y' (float32, scaled): header
    [u_lo, 1 / delta, delta, n_cells, n_chunks, chunk points (int32 bits), 0, 0], then per cell
    the n_chunks chunk rows, one row per group of KDE_MT_GROUP chunks and one row for the whole
    point set, KDE_MT_TERMS float32 each ([n_cells][kde_moment_rows(n_chunks)][4]; float64
    sums, one rounding).  None when kde_moment_cells declines the node."""
    cells = kde_moment_cells(y)
    if cells is None:
        return None
    lo32, delta32, inv32, n = cells
    y64 = np.asarray(y, np.float32).reshape(-1).astype(np.float64)
    sq = (y64 * y64).astype(np.float32).astype(np.float64)
    m = y64.size
    nch, per = kde_moment_chunks(m)
    centres = kde_moment_centres(lo32, delta32, n)
    pw = np.stack([(math.log(2.0) * y64) ** k / math.factorial(k) for k in range(KDE_MT_TERMS)], axis=1)
    ng = -(-nch // KDE_MT_GROUP)
    tab = np.zeros((n, kde_moment_rows(nch), KDE_MT_TERMS), np.float64)
    for j0 in range(0, m, 4096):                               # bounded [cells x points] blocks
        j1 = min(m, j0 + 4096)
        wts = np.exp2(centres[:, None] * y64[None, j0:j1] - sq[None, j0:j1])     # [n, pts]
        contrib = wts[:, :, None] * pw[None, j0:j1, :]                           # [n, pts, K]
        chunk = np.arange(j0, j1) // per
        for c in np.unique(chunk):
            tab[:, c, :] += contrib[:, chunk == c, :].sum(axis=1)
    for g in range(ng):
        tab[:, nch + g, :] = tab[:, g * KDE_MT_GROUP:min(nch, (g + 1) * KDE_MT_GROUP), :].sum(axis=1)
    tab[:, nch + ng, :] = tab[:, :nch, :].sum(axis=1)
    head = np.zeros(KDE_MT_HEADER, np.float32)
    head[:3] = [lo32, inv32, delta32]
    head[3:6] = np.array([n, nch, per], np.int32).view(np.float32)
    return np.concatenate([head, tab.astype(np.float32).reshape(-1)])


def _np(t: torch.Tensor) -> np.ndarray:
    return t.detach().to("cpu", torch.float32).numpy()


def _pack_mlp_generic(blob: _Blob, layers, offs: Dict[str, int]) -> Dict[str, int]:
    """Layer table + fragments of csrc mlp_generic (hidden_dims other than (32, 32)): per
    layer W fragments [ceil(out/32)][ceil(in/2)][64] and accumulator-init biases
    [ceil(out/32)][2][16]; the table [L, (in, out, off_w, off_b) x L] is int32 in the blob."""
    lane = np.arange(64)
    table = [len(layers)]
    for w, b in layers:
        w, b = _np(w), _np(b)
        out, nin = w.shape
        nblk, t1 = -(-out // 32), -(-nin // 2)
        wz = np.zeros((nblk * 32, 2 * t1), np.float32)
        wz[:out, :nin] = w
        frag = np.stack([np.stack([wz[32 * k + (lane & 31), 2 * t + (lane >> 5)] for t in range(t1)])
                         for k in range(nblk)])                                   # [nblk, t1, 64]
        bz = np.zeros(nblk * 32, np.float32)
        bz[:out] = b
        bias = np.stack([bz[32 * k + _ROWS] for k in range(nblk)])                # [nblk, 2, 16]
        table += [nin, out, blob.add(frag), blob.add(bias)]
    offs["w2"] = blob.add(np.asarray(table, np.int32).view(np.float32))
    offs["n_out"] = int(_np(layers[-1][0]).shape[0])
    offs["generic"] = 1
    offs["scratch"] = offs["n_out"] + 2 * max([int(w.shape[0]) for w, _ in layers[:-1]] + [1])
    return offs


def _pack_mlp(blob: _Blob, rec: CPDRecord, standardize: bool) -> Dict[str, int]:
    """MFMA fragment layouts of csrc/vbn_walk_impl.h mlp_forward (biases as accumulator init);
    other hidden_dims than (32, 32) get the generic layer-by-layer pack (mlp_generic)."""
    layers = rec.mlp_layers()
    hidden = tuple(int(w.shape[0]) for w, _ in layers[:-1])
    offs: Dict[str, int] = {}
    if standardize:
        inv = (np.float32(1.0) / _np(rec.state["std_x"]).astype(np.float32)).astype(np.float32)
        offs["std"] = blob.add(np.concatenate([_np(rec.state["mean_x"]), inv]))
    else:
        offs["std"] = 0
    if hidden != MLP_HIDDEN:
        return _pack_mlp_generic(blob, layers, offs)
    (w1, b1), (w2, b2), (w3, b3) = [(_np(w), _np(b)) for w, b in layers]
    nin = w1.shape[1]
    t1 = (nin + 1) // 2
    w1z = np.zeros((32, 2 * t1), np.float32)
    w1z[:, :nin] = w1
    lane = np.arange(64)
    w1f = np.stack([w1z[lane & 31, 2 * t + (lane >> 5)] for t in range(t1)])   # [t1, 64]
    w2f = np.zeros((16, 64), np.float32)
    for s in range(16):
        w2f[s] = w2[lane & 31, _ROWS[lane >> 5, s]]
    # weight block staged into LDS by the walk (one step ahead): W1 | biases | split-f16 W2 |
    # W3 | b3, contiguous, 16-byte aligned pieces (the exact-f32 W2 copy stays outside)
    offs["w1"] = blob.add(w1f)
    offs["wblk"] = offs["w1"]
    # accumulator init: [layer][group g][half h][register r] = b[row(r, h)] (one copy per group)
    offs["b2"] = blob.add(np.stack([np.stack([b[_ROWS]] * 2) for b in (b1, b2)]))  # [2, 2, 2, 16]
    # split-f16 fragments of v_mfma_f32_32x32x16_f16: k-step s, lane l, element j ->
    # W2[l&31][16s + 8(j>>2) + 4(l>>5) + (j&3)]; hi = f16(w), lo = f16(w - hi)
    # weights beyond the f16 split range: the node always takes the exact f32 layer-2 chain
    # (the split fragments are still packed, so the weight block layout does not change)
    offs["f32l2"] = int(np.abs(w2).max() > 32768.0)
    # layer-1 operand bound (csrc mlp_l1_act): with every operand |x| <= zlim, each layer-1
    # pre-activation |z| <= max|b1| + zlim max_r sum_k |W1[r, k]| and |act(z)| <= max(|z|, 1)
    # stay inside the split range, so the walk compares the operands (one per MFMA) instead
    # of every activation; 0.1 % margin for the f32 accumulation.  -1: no bound (always check)
    # relu nodes split the raw pre-activation with the ReLU folded in (csrc
    # layer2_split_relu), which needs z < 2048: the bound is taken against that
    rs = float(np.abs(w1.astype(np.float64)).sum(axis=1).max()) if w1.size else 0.0
    lim = 2048.0 if str(rec.hp("activation") or "relu") == "relu" else 32768.0
    room = lim * (1.0 - 1e-3) - float(np.abs(b1.astype(np.float64)).max())
    if room <= 1.0:
        offs["zlim"] = -1.0
    else:
        offs["zlim"] = float(np.float32(min(room / rs, 3.0e38))) if rs > 0 else 3.0e38
    j = np.arange(8)
    j3 = j
    frag = np.zeros((2, 64, 8), np.float32)
    for s in range(2):
        for ln in range(64):
            frag[s, ln] = w2[ln & 31, 16 * s + 8 * (j >> 2) + 4 * (ln >> 5) + (j & 3)]
    with np.errstate(over="ignore", invalid="ignore"):
        hi = frag.astype(np.float16)
        lo = (frag - hi.astype(np.float32)).astype(np.float16)
    halfs = np.concatenate([hi, lo]).reshape(-1)                               # [4, 64, 8] f16
    offs["w2h"] = blob.add(halfs.view(np.float32))
    # head: row j = W3[j][row(r, 0)] (r < 16) ++ W3[j][row(r, 1)] (lane half h reads 16 at 16 h)
    offs["w3"] = blob.add(np.concatenate([w3[:, _ROWS[0]], w3[:, _ROWS[1]]], axis=1))  # [n_out, 32]
    offs["b3"] = blob.add(b3)
    n_out = w3.shape[0]
    if HEAD_MFMA_MIN <= n_out <= 32 and np.abs(w3).max() <= 32768.0:
        # wide heads (mdn, softmax_nn) on the split-f16 MFMA like layer 2 (csrc head_mfma):
        # W3 padded to 32 output rows in the layer-2 fragment layout, then the bias as the
        # accumulator init [half h][16] = b3[row(r, h)] (0 beyond n_out); outside the block
        w3p = np.zeros((32, 32), np.float32)
        w3p[:n_out] = w3
        f3 = np.zeros((2, 64, 8), np.float32)
        for s_ in range(2):
            for ln in range(64):
                f3[s_, ln] = w3p[ln & 31, 16 * s_ + 8 * (j3 >> 2) + 4 * (ln >> 5) + (j3 & 3)]
        hi3 = f3.astype(np.float16)
        lo3 = (f3 - hi3.astype(np.float32)).astype(np.float16)
        b3p = np.zeros(32, np.float32)
        b3p[:n_out] = b3
        offs["w3h"] = blob.add(np.concatenate([hi3, lo3]).reshape(-1).view(np.float32))   # 1024 floats
        blob.add(b3p[_ROWS])                                                               # [2, 16]
    blen = offs["b3"] + b3.size - offs["wblk"]
    offs["wblk_len"] = -(-blen // WBLK_CHUNK) * WBLK_CHUNK
    offs["w2"] = blob.add(w2f.reshape(4, 4, 64).transpose(0, 2, 1))            # [4, 64, 4] (exact f32)
    offs["n_out"] = w3.shape[0]
    return offs


@dataclass
class NodePack:
    kind: int
    flags: int          # static flags (ROOT, STANDARDIZE, CLIP)
    act: int
    n_in: int
    out_dim: int
    k: int
    n_out: int
    aux0: int
    aux1: int
    offs: Dict[str, int]
    scratch: int = 0    # LDS scratch rows the node's MLP needs (head outputs + generic buffers)


def _pack_node(blob: _Blob, rec: CPDRecord) -> NodePack:
    kind = rec.kind
    D = rec.output_dim
    root = rec.is_root
    flags = F_ROOT if root else 0
    act = ACT_ID.get(str(rec.hp("activation") or "relu"), -1)
    if act < 0:
        raise ValueError(f"unknown activation {rec.hp('activation')}")
    st = rec.state
    offs: Dict[str, int] = {}
    k = n_out = aux0 = aux1 = 0
    if kind == "gaussian_nn":
        if root:
            loc = st["_loc"].view(1, 1, -1)
            scale = (F.softplus(st["_log_scale"]) + float(rec.hp("min_scale"))).view(1, 1, -1)
            std_y = st["std_y"].view(1, 1, -1)
            loc, scale = loc * std_y + st["mean_y"].view(1, 1, -1), scale * std_y
            loc, scale = loc.reshape(-1), scale.reshape(-1)
            offs["tail"] = blob.add(np.concatenate([_np(loc), _np(scale), _np(scale.log())]))
        else:
            flags |= F_STANDARDIZE
            offs.update(_pack_mlp(blob, rec, standardize=True))
            n_out = offs.pop("n_out")
            offs["tail"] = blob.add(np.concatenate([_np(st["std_y"]), _np(st["mean_y"]),
                                                    np.array([rec.hp("min_scale")], np.float32)]))
    elif kind == "linear_gaussian":
        var = st["_var"]
        scale = torch.sqrt(var.clamp(min=float(rec.hp("min_scale")) ** 2))
        w = st["_weight"]                                  # [n_in, D]
        offs["tail"] = blob.add(np.concatenate([_np(w.t().contiguous()).reshape(-1), _np(st["_bias"]),
                                                _np(scale), _np(torch.log(scale))]))
    elif kind == "mdn":
        k = int(rec.hp("n_components"))
        if root:
            pi = torch.softmax(st["_logits"], dim=-1).clamp_min(1e-5)
            pi = pi / pi.sum(dim=-1, keepdim=True).clamp_min(1e-12)
            scale = F.softplus(st["_log_scale"]) + float(rec.hp("min_scale"))
            log_scale = torch.log(scale)
            offs["tail"] = blob.add(np.concatenate([
                _np(pi), _np(torch.log(pi)), _np(st["_loc"]).reshape(-1), _np(scale).reshape(-1),
                _np(log_scale).reshape(-1), _np(torch.exp(2 * log_scale)).reshape(-1),
                _np(torch.softmax(st["_logits"], dim=-1))]))
        else:
            offs.update(_pack_mlp(blob, rec, standardize=False))
            n_out = offs.pop("n_out")
            if n_out != k * (2 * D) + k:
                raise ValueError("mdn head width mismatch")
            offs["tail"] = blob.add(np.array([rec.hp("min_scale")], np.float32))
    elif kind == "kde":
        pts_p = rec.extra["parents"].float()
        pts_y = rec.extra["targets"].float()
        m = int(pts_y.shape[0])
        dp = int(pts_p.shape[1]) if pts_p.dim() == 2 else 0
        if m == 0:
            raise RuntimeError("KDECPD is not fitted yet.")
        bw = float(rec.hp("bandwidth"))
        pbw = rec.hp("parent_bandwidth")
        pbw = bw if pbw is None else float(pbw)
        min_scale = float(rec.hp("min_scale"))
        s_p = max(pbw, 1e-3) + min_scale                  # kde.py:106
        s_y = max(bw, 1e-3) + min_scale
        noise_scale = max(bw, 1e-3) + min_scale            # kde.py:166,180
        cy = -0.5 * D * (math.log(2 * math.pi) + 2 * math.log(s_y))
        c_p = np.float32(_KDE_C / s_p)
        c_y = np.float32(_KDE_C / s_y)
        offs["tail"] = blob.add(np.array([1.0 / np.float32(s_p), 1.0 / np.float32(s_y),
                                          noise_scale, cy, math.log(float(m)), c_p, c_y, 0], np.float32))
        # MFMA packs (csrc/vbn_walk_impl.h, kde_b32_sums): bf16x3 point slots, [block][g][h][32][8]
        if 1 <= dp <= 3:
            offs["kq"] = blob.add(_kde_pack_b32(_np(pts_p) * c_p))
            offs["kr"] = blob.add(_kde_pack([_np(pts_p) * c_p], records=True))
            offs["kv"] = blob.add(_kde_pack_valu(_np(pts_p) * c_p))
            if dp == 1 and KDE_MOMENTS:               # pass 1 from a moment table (kde_index_moments)
                mt = kde_moment_table((_np(pts_p) * c_p).reshape(-1))
                if mt is not None:
                    offs["kmt"] = blob.add(mt)
        if dp + D <= 4:
            feats = np.concatenate(([_np(pts_p).reshape(m, -1) * c_p] if dp else [])
                                   + [_np(pts_y).reshape(m, -1) * c_y], axis=1)
            offs["kqy"] = blob.add(_kde_pack_b32(feats))
        stride = dp + D
        stride += (-stride) % 2 if stride > 1 else 0
        recs = np.zeros((m, stride), np.float32)
        if dp:
            recs[:, :dp] = _np(pts_p)
        recs[:, dp:dp + D] = _np(pts_y)
        offs["pts"] = blob.add(recs)
        k, aux0, aux1 = m, dp, stride
    elif kind == "softmax_nn":
        if str(rec.hp("mode_when_not_discrete") or "binned") != "binned":
            raise NotImplementedError("softmax_nn mode_when_not_discrete != 'binned'")
        if not bool(st["_bins_ready"]):
            raise RuntimeError("Bins not initialized. Call fit(...) before sampling.")
        k = int(rec.hp("n_classes"))
        aux0 = WITHIN_ID[str(rec.hp("within_bin"))]
        disc = st["_is_discrete"].bool()
        if D > 31:
            raise NotImplementedError("softmax_nn with more than 31 output dims")
        aux1 = int(sum(1 << d for d in range(D) if bool(disc[d])))
        if bool(rec.hp("within_bin_clip")):
            flags |= F_CLIP
        mbw = float(rec.hp("min_bin_width"))
        offs["tail"] = blob.add(np.concatenate([
            _np(st["_bin_edges"]).reshape(-1), _np(st["_sample_values"]).reshape(-1),
            _np(st["_class_values"]).reshape(-1),
            np.array([rec.hp("within_bin_scale"), mbw, mbw ** 2, 0.0], np.float32)]))
        if root:
            if bool(st["_root_ready"]):
                tab = torch.log_softmax(st["_root_log_probs"].view(D, k) / 1.0, dim=-1)
            else:
                tab = st["_logits"].view(D, k) / 1.0
            offs["pts"] = blob.add(_np(tab))
        else:
            offs.update(_pack_mlp(blob, rec, standardize=False))
            n_out = offs.pop("n_out")
    else:
        raise ValueError(kind)
    if offs.pop("generic", 0):
        flags |= F_MLP_GENERIC
    if offs.pop("f32l2", 0):
        flags |= F_F32L2
    scratch = offs.pop("scratch", n_out)
    return NodePack(kind=KIND_ID[kind], flags=flags, act=max(act, 0), n_in=rec.input_dim,
                    out_dim=D, k=k, n_out=n_out, aux0=aux0, aux1=aux1, offs=offs, scratch=scratch)


class PackedModel:
    """Device-resident parameter blob of a :class:`BNModel` (built once per model+device)."""

    def __init__(self, model: BNModel, device: torch.device):
        self.model = model
        self.device = torch.device(device)
        blob = _Blob()
        blob.add(np.zeros(4, np.float32))                 # offset 0 is never a real block
        self.nodes: Dict[str, NodePack] = {}
        # Philox stream ids pack (node, dim, stream) into 14 + 8 + 2 bits (csrc rng_words)
        if len(model.topo) >= MAX_NODES:
            raise NotImplementedError(f"{len(model.topo)} nodes: the walk keys RNG streams for < {MAX_NODES}")
        for node in model.topo:
            if model.out_dim(node) >= MAX_NODE_DIMS:
                raise NotImplementedError(f"node {node}: {model.out_dim(node)} dims (max {MAX_NODE_DIMS - 1})")
            rec = model.cpds[node]
            expect = sum(model.out_dim(p) for p in model.parents[node])
            if rec.input_dim != expect:
                raise ValueError(f"node {node}: CPD input_dim {rec.input_dim} != parents width {expect}")
            self.nodes[node] = _pack_node(blob, rec)
        host = torch.from_numpy(blob.finish())
        self.params = host.to(self.device)
        self.node_id = {n: i for i, n in enumerate(model.topo)}
        self.max_out = max([p.scratch for p in self.nodes.values()] + [1])
        self.has_kde = any(p.kind == KIND_ID["kde"] for p in self.nodes.values())
        self.dmax = max(model.out_dim(n) for n in model.topo)


@dataclass
class QueryPlan:
    steps: torch.Tensor        # int32 [n_steps, 32] (device)
    in_cols: torch.Tensor      # int32 (device)
    out_cols: torch.Tensor     # int32 (device)
    n_steps: int
    n_slots: int
    max_out: int
    fixed_nodes: List[str]     # order of columns in the fixed buffer
    fixed_ld: int
    noise_nodes: List[str]     # noise_idx order (latent nodes)
    out_nodes: List[str]
    mode: int
    slot_of: Dict[str, int]
    kind_mask: int = 63       # CPD kinds the walk evaluates (selects the kernel instantiation;
                              # | 32 non-relu activations, | 512 generic-MLP nodes)
    order: Optional[List[str]] = None   # the walk order of the steps (a topological order)
    wbuf: int = 0             # floats per LDS weight buffer (max wblk_len over the steps)
    # precompute (precompute_plans): the same walk with VBN_F_PRECOMP steps, the one-query
    # pre-pass walk whose out_x the per-sample ones read, and the one-wave-per-query pre-pass
    # whose out_x the per-query (VBN_F_PRECOMP_Q) ones read
    pc: Optional["QueryPlan"] = None
    pre: Optional["QueryPlan"] = None
    pre_q: Optional["QueryPlan"] = None


def barren_pruned(model: BNModel, keep: Sequence[str]) -> set:
    """Ancestors of ``keep`` (inclusive): every other node is barren for the query."""
    need = set()
    stack = list(keep)
    while stack:
        n = stack.pop()
        if n in need:
            continue
        need.add(n)
        stack.extend(model.parents[n])
    return need


def liveness_order(model: BNModel, *, fixed: Sequence[str], logp: Sequence[str], out_nodes: Sequence[str],
                   params: Sequence[str] = (), skip: Sequence[str] = (), seed: Optional[int] = None) -> List[str]:
    """A topological order of the non-skipped nodes that keeps few node values live at once
    (greedy list scheduling: among the ready nodes, the one whose step frees the most parent
    columns and holds the fewest new ones; ties in the model's order).  Node values live in LDS
    slots (build_plan's liveness scan), and a wave's LDS footprint bounds how many waves a CU
    holds: the 128-node cfg5 DAG peaks at 32 live columns in the model's order, 25 here."""
    skip_s, fixed_s, logp_s, params_s = set(skip), set(fixed), set(logp), set(params)
    nodes = [n for n in model.topo if n not in skip_s]
    rank = {n: i for i, n in enumerate(nodes)}
    # ties broken in the model's order, or (seed given) in a seeded random order: a restart of
    # the greedy, deterministic per seed
    tie = rank if seed is None else dict(zip(nodes, np.random.default_rng(seed).permutation(len(nodes)).tolist()))
    reads = {n: (n not in fixed_s) or (n in logp_s) or (n in params_s) for n in nodes}
    children = {n: [] for n in nodes}
    for n in nodes:
        for p in model.parents[n]:
            if p in rank:
                children[p].append(n)
    readers_left = {n: sum(1 for c in children[n] if reads[c]) for n in nodes}
    waiting = {n: sum(1 for p in model.parents[n] if p in rank) for n in nodes}
    outs = set(out_nodes)
    ready = [n for n in nodes if waiting[n] == 0]
    order: List[str] = []
    while ready:
        def cost(n):
            freed = sum(1 for p in model.parents[n] if p in rank and reads[n] and readers_left[p] == 1
                        and p not in outs)
            holds = 0 if (readers_left[n] == 0 and n not in outs) else 1
            return (holds - freed, tie[n])
        n = min(ready, key=cost)
        ready.remove(n)
        order.append(n)
        if reads[n]:
            for p in model.parents[n]:
                if p in rank:
                    readers_left[p] -= 1
        for c in children[n]:
            waiting[c] -= 1
            if waiting[c] == 0:
                ready.append(c)
    assert len(order) == len(nodes)
    return order


def build_plan(packed: PackedModel, *, latent: Sequence[str], fixed: Sequence[str],
               logp: Sequence[str], out_nodes: Sequence[str], shared_roots: bool, mode: int,
               skip: Sequence[str] = (), exact_f32: bool = False, kde_valu: bool = False,
               params: Sequence[str] = (), pre_out: Sequence[str] = (),
               order: Optional[Sequence[str]] = None, clamp: Sequence[str] = ()) -> QueryPlan:
    """Step table for one query signature.

    ``latent``: nodes sampled; ``fixed``: nodes read from the fixed buffer (evidence/do);
    ``logp``: nodes whose log p(value | parents) is accumulated; ``out_nodes``: nodes whose
    values are written per particle; ``skip``: nodes not walked at all; ``exact_f32``: run
    the MLPs' hidden layer on the exact f32 MFMA chain instead of the split-f16 product;
    ``kde_valu``: KDE pairwise distances on packed VALU instead of the 16x16x4 f32 MFMA tile.
    ``params``: nodes whose conditional parameters are written instead of a draw (role
    PARAMS; gaussian_nn / linear_gaussian: loc ++ scale, softmax_nn: class probabilities
    [D][C], mdn: softmax(logits) [K] ++ loc [K][D] ++ scale [K][D]) -- the Rao-Blackwellized
    target and CPDHandle.conditional.  ``pre_out``: latent nodes that write their per-sample
    quantities instead of a sample (VBN_F_PRE_OUT, the shared-sample pre-pass of
    :func:`precompute_plans`): NN CPDs their n_out MLP head outputs, KDE its 16 inverse-CDF
    chunk sums ++ the underflow shift.  ``order``: the walk order of the non-skipped nodes (a
    topological order; default the model's, reference ``vbn.py:670-675``) -- every draw is keyed
    by its node, so the order changes only the LDS slot assignment and the Box-Muller pairing
    (:func:`liveness_order`).  ``clamp``: fixed nodes whose values the kernel clamps as
    likelihood weighting's clamp_evidence does (VBN_F_CLAMP_EV; _core.py:112-114).
    """
    model = packed.model
    latent_s, fixed_s, logp_s, skip_s = set(latent), set(fixed), set(logp), set(skip)
    params_s = set(params)
    pre_s = set(pre_out)
    clamp_s = set(clamp)
    if order is None:
        order = [n for n in model.topo if n not in skip_s]
    else:
        order = list(order)
        if sorted(order) != sorted(n for n in model.topo if n not in skip_s):
            raise ValueError("order must list every non-skipped node once")
        seen = set()
        for n in order:
            if any(p not in seen and p not in skip_s for p in model.parents[n]):
                raise ValueError(f"order is not topological at node {n}")
            seen.add(n)
    for n in order:
        if n in params_s:
            if n in latent_s or n in fixed_s or n in logp_s:
                raise ValueError(f"params node {n} cannot be latent/fixed/logp")
            continue
        if (n in latent_s) == (n in fixed_s):
            raise ValueError(f"node {n} must be exactly one of latent/fixed")

    def width(n: str) -> int:
        if n in pre_s:
            return precompute_width(packed, n)
        if n not in params_s:
            return model.out_dim(n)
        rec = model.cpds[n]
        if rec.kind in ("gaussian_nn", "linear_gaussian"):
            return 2 * model.out_dim(n)                               # loc ++ scale
        if rec.kind == "softmax_nn":
            return model.out_dim(n) * int(rec.hp("n_classes"))        # class probabilities [D][C]
        if rec.kind == "mdn":
            return int(rec.hp("n_components")) * (1 + 2 * model.out_dim(n))  # weights, loc, scale
        raise ValueError(f"no parameter output for {rec.kind} node {n}")
    # liveness: last step index reading each node's columns
    pos = {n: i for i, n in enumerate(order)}
    last = {n: pos[n] for n in order}
    # a fixed node without log-prob only loads its value: it reads no parents
    reads = {n: (n in latent_s or n in logp_s or n in params_s) for n in order}
    for n in order:
        if not reads[n]:
            continue
        for p in model.parents[n]:
            if p not in pos:
                raise ValueError(f"node {n} needs skipped parent {p}")
            last[p] = max(last[p], pos[n])
    for n in out_nodes:
        last[n] = len(order) + 1
    free: List[int] = []
    n_slots = 0
    slot_of: Dict[str, int] = {}
    release: Dict[int, List[str]] = {}
    for i, n in enumerate(order):
        d = width(n)
        # contiguous run of d slots: take from the free list if a run exists
        base = None
        if d == 1 and free:
            free.sort()
            base = free.pop(0)
        elif d > 1:
            fs = sorted(free)
            for j in range(len(fs) - d + 1):
                if fs[j + d - 1] - fs[j] == d - 1:
                    base = fs[j]
                    for q in range(d):
                        free.remove(base + q)
                    break
        if base is None:
            base = n_slots
            n_slots += d
        slot_of[n] = base
        release.setdefault(last[n], []).append(n)
        for m in release.pop(i, []):
            if m != n or last[n] == i:
                free.extend(range(slot_of[m], slot_of[m] + width(m)))
    fixed_nodes = [n for n in order if n in fixed_s]
    fixed_col = {}
    c = 0
    for n in fixed_nodes:
        fixed_col[n] = c
        c += model.out_dim(n)
    noise_nodes = [n for n in order if n in latent_s]
    noise_idx = {n: i for i, n in enumerate(noise_nodes)}
    steps = np.zeros((len(order), STEP_INTS), np.int32)
    in_cols: List[int] = []
    for i, n in enumerate(order):
        npk = packed.nodes[n]
        row = steps[i]
        row[S_KIND] = npk.kind
        row[S_ROLE] = ROLE_PARAMS if n in params_s else (ROLE_LATENT if n in latent_s else ROLE_FIXED)
        fl = npk.flags
        if n in logp_s:
            fl |= F_LOGP
        if shared_roots and (npk.flags & F_ROOT):
            fl |= F_SHARED
        if exact_f32:
            fl |= F_F32L2
        if kde_valu and npk.kind == KIND_ID["kde"]:
            fl |= F_KDE_VALU
        if n in pre_s:
            fl |= F_PRE_OUT
        if n in clamp_s and n in fixed_s:
            fl |= F_CLAMP_EV
        row[S_FLAGS] = fl
        row[S_ACT] = npk.act
        row[S_NIN] = npk.n_in
        row[S_INOFF] = len(in_cols)
        if reads[n]:
            for p in model.parents[n]:
                in_cols.extend(range(slot_of[p], slot_of[p] + model.out_dim(p)))
        row[S_OUTCOL] = slot_of[n]
        row[S_OUTDIM] = npk.out_dim
        row[S_FIXEDCOL] = fixed_col.get(n, 0)
        row[S_K] = npk.k
        row[S_NOUT] = npk.n_out
        row[S_NODEID] = packed.node_id[n]
        row[S_NOISE] = noise_idx.get(n, 0)
        row[S_AUX0] = npk.aux0
        row[S_AUX1] = npk.aux1
        for key, idx in (("std", S_OFF_STD), ("w1", S_OFF_W1), ("w2", S_OFF_W2), ("b2", S_OFF_B2),
                         ("w3", S_OFF_W3), ("b3", S_OFF_B3), ("tail", S_OFF_TAIL), ("pts", S_OFF_PTS),
                         ("w2h", S_OFF_W2H)):
            row[idx] = npk.offs.get(key, 0)
        row[S_OFF_KQ] = npk.offs.get("kq", -1)
        if "zlim" in npk.offs:                   # NN steps: layer-1 operand bound (f32 bits)
            row[S_OFF_KQ] = np.float32(npk.offs["zlim"]).view(np.int32)
        row[S_OFF_KQY] = npk.offs.get("kqy", -1)
        if "w3h" in npk.offs:                    # NN steps: split-f16 head fragments
            row[S_OFF_KQY] = npk.offs["w3h"]
            fl |= F_HEAD_MFMA
            row[S_FLAGS] = fl
        row[S_OFF_KR] = npk.offs.get("kr", -1)
        row[S_OFF_KV] = npk.offs.get("kv", -1)
        row[S_RES7] = npk.offs.get("kmt", -1)   # kde: moment table of a one-feature node
        if "wblk" in npk.offs and (n in latent_s or n in logp_s or n in params_s):
            row[S_WBLK_OFF] = npk.offs["wblk"]
            row[S_WBLK_LEN] = npk.offs["wblk_len"]
    out_cols: List[int] = []
    for n in out_nodes:
        out_cols.extend(range(slot_of[n], slot_of[n] + width(n)))
    dev = packed.device

    def t(a):
        a = np.asarray(a, np.int32).reshape(-1) if len(a) else np.zeros(1, np.int32)
        return torch.from_numpy(np.ascontiguousarray(a)).to(dev)

    _pair_normals(steps)
    kind_mask = 0
    for n in order:
        if n in latent_s or n in logp_s or n in params_s:
            npk = packed.nodes[n]
            kind_mask |= 1 << npk.kind
            if npk.n_out and npk.act != ACT_ID["relu"]:
                kind_mask |= 32
            if npk.flags & F_MLP_GENERIC:
                kind_mask |= 512                 # csrc kind-set bit 9: the generic-MLP path
    max_out = max([packed.nodes[n].scratch for n in order] + [1])
    if any(packed.nodes[n].kind == KIND_ID["kde"] for n in order):
        max_out = max(max_out, KDE_CHUNKS)
    steps_t = torch.from_numpy(steps).to(dev) if len(order) else torch.zeros(1, STEP_INTS, dtype=torch.int32, device=dev)
    steps_t._vbn_wblk_max = int(steps[:, S_WBLK_LEN].max()) if len(order) else 0   # ops._check_wbuf
    ic_host = np.asarray(in_cols, np.int32).reshape(-1)
    # host copies for the plan-specialised walk (jit.py); the key names this exact table
    steps_t._vbn_host = (steps.copy(), ic_host.copy(),
                         hashlib.sha1(steps.tobytes() + b"|" + ic_host.tobytes()).hexdigest())
    return QueryPlan(
        steps=steps_t,
        in_cols=t(in_cols), out_cols=t(out_cols), n_steps=len(order), n_slots=max(n_slots, 1),
        max_out=max_out, fixed_nodes=fixed_nodes, fixed_ld=max(c, 1), noise_nodes=noise_nodes,
        out_nodes=list(out_nodes), mode=mode, slot_of=slot_of, kind_mask=kind_mask, order=list(order),
        wbuf=int(steps[:, S_WBLK_LEN].max()) if len(order) else 0)


def _pair_normals(steps: np.ndarray) -> None:
    """Pair consecutive one-dimensional normal draws (csrc draw_normal, lean walks only): the
    VBN_F_BM_FIRST step's Box-Muller pair gives r cos to itself and r sin, an independent N(0, 1),
    to the next VBN_F_BM_SECOND step.  Pairs never mix draws shared across queries (F_SHARED
    roots, Q5) with per-query ones, and one pair completes before the next starts (the kernel
    keeps a single spare).  Injected draws and the other walk forms ignore the flags."""
    # kinds whose LATENT step always draws exactly one dim-0 normal (softmax_nn draws one only
    # in its gaussian within-bin mode, so it is left out)
    gauss = (KIND_ID["gaussian_nn"], KIND_ID["linear_gaussian"], KIND_ID["mdn"], KIND_ID["kde"])
    pending = -1
    for i in range(len(steps)):
        r = steps[i]
        if r[S_ROLE] != ROLE_LATENT or r[S_KIND] not in gauss or r[S_OUTDIM] != 1:
            continue
        if pending >= 0 and (steps[pending][S_FLAGS] & F_SHARED) == (r[S_FLAGS] & F_SHARED):
            steps[pending][S_FLAGS] |= F_BM_FIRST
            r[S_FLAGS] |= F_BM_SECOND
            pending = -1
        else:
            pending = i


@dataclass
class GibbsPlan:
    init: QueryPlan            # ancestral start state (gibbs.py:29), every node kept in its own slots
    steps: torch.Tensor        # int32 [n_steps, 32]: one sweep (device)
    n_steps: int
    latent: List[str]          # sweep order; candidate noise index 2j, choice noise index 2j + 1
    target: str
    n_noise: int
    in_cols: torch.Tensor      # parent slots of every row (children read their parents too)
    kind_mask: int
    wbuf: int = 0              # floats per LDS weight buffer (max wblk_len over the sweep steps)


def build_gibbs_plan(packed: PackedModel, *, latent: Sequence[str], fixed: Sequence[str], target: str,
                     exact_f32: bool = False, kde_valu: bool = False) -> GibbsPlan:
    """One Gibbs sweep as a step table (GibbsSampler.sample, gibbs.py:36-87).

    Per latent node, in topological order: a LATENT step draws the chain's 8 candidates into
    the node's slot (one per lane) and starts the score with their log-prob (50-51); one
    FIXED + KEEP + LOGP step per child adds log p(child | candidate, other parents) from the
    child's current value (52-78); a SELECT step softmaxes the 8 scores, draws one and
    broadcasts it to the chain (79-82).  A COLLECT step at the end writes the target (83-87).
    Every node has its own slots for the whole walk (the sweep reads any node at any time).
    """
    model = packed.model
    order = list(model.topo)
    kw = dict(latent=latent, fixed=fixed, out_nodes=order, shared_roots=True,
              exact_f32=exact_f32, kde_valu=kde_valu)
    init = build_plan(packed, logp=[], mode=MODE_SAMPLE, **kw)
    full = build_plan(packed, logp=order, mode=MODE_SAMPLE, **kw)       # every row reads its parents
    assert init.slot_of == full.slot_of
    rows = full.steps.cpu().numpy()
    pos = {n: i for i, n in enumerate(order)}
    lat = [n for n in order if n in set(latent)]
    children = model.children()
    table: List[np.ndarray] = []
    for j, n in enumerate(lat):
        r = rows[pos[n]].copy()
        r[S_ROLE] = ROLE_LATENT
        # per-chain candidates, roots included: the reference's root candidates are [1, 8, D]
        # (gibbs.py:50), which it can only index at B = 1 (81); shared root candidates would
        # correlate every chain of the batch
        r[S_FLAGS] = (r[S_FLAGS] | F_LOGP | F_LPRESET) & ~F_SHARED
        r[S_NOISE] = 2 * j
        table.append(r)
        for c in children[n]:
            r = rows[pos[c]].copy()
            r[S_ROLE] = ROLE_FIXED
            r[S_FLAGS] = (r[S_FLAGS] | F_LOGP | F_KEEP) & ~F_SHARED
            table.append(r)
        r = rows[pos[n]].copy()
        r[S_ROLE] = ROLE_SELECT
        r[S_FLAGS] = 0
        r[S_NOISE] = 2 * j + 1
        table.append(r)
    r = rows[pos[target]].copy()
    r[S_ROLE] = ROLE_COLLECT
    r[S_FLAGS] = 0
    table.append(r)
    tab = np.ascontiguousarray(np.stack(table))
    tab[:, S_FLAGS] &= ~(F_BM_FIRST | F_BM_SECOND)                          # walk-only pairing
    sel = (tab[:, S_ROLE] == ROLE_SELECT) | (tab[:, S_ROLE] == ROLE_COLLECT)
    tab[sel, S_WBLK_OFF] = 0                                              # no MLP on these rows
    tab[sel, S_WBLK_LEN] = 0
    steps = torch.from_numpy(tab).to(packed.device)
    steps._vbn_wblk_max = int(tab[:, S_WBLK_LEN].max())                  # ops._check_wbuf
    ic_host = full.steps._vbn_host[1]
    steps._vbn_host = (tab.copy(), ic_host.copy(),                         # jit.py (sweep kernels)
                       hashlib.sha1(b"gibbs|" + tab.tobytes() + b"|" + ic_host.tobytes()).hexdigest())
    return GibbsPlan(init=init, steps=steps, n_steps=len(table), latent=lat, target=target,
                     n_noise=max(2 * len(lat), 1), in_cols=full.in_cols, kind_mask=full.kind_mask,
                     wbuf=int(tab[:, S_WBLK_LEN].max()))


def gibbs_levels(tab: np.ndarray, in_cols: np.ndarray, n_waves: int) -> List[List[List[Tuple[int, int]]]]:
    """Wave-parallel schedule of one Gibbs sweep table (csrc vbn_walk_plan.h, chain workgroups).

    A node update -- its LATENT step, one FIXED + KEEP step per child, its SELECT step -- reads
    the slots of its Markov blanket (parents, children, the children's other parents) and
    writes its own.  Two updates that touch no slot the other writes commute, so running them
    at the same time on different waves gives bit-for-bit the sequential sweep (same draws,
    which are keyed by node and sweep, and the same operations on the same values).  Level of
    an update = 1 + the highest level of an earlier update it conflicts with; the updates of a
    level are spread over ``n_waves`` waves (longest first, by step count), and the COLLECT
    steps form a last level on wave 0.

    Returns ``levels[l][w]`` = the (begin, end) step ranges wave w runs in level l, in sweep
    order.  A child's FIXED + KEEP step writes back the value it read (the same bits), which is
    a read for this analysis.
    """
    groups, level, collect = _gibbs_update_levels(tab, in_cols)
    n_lv = max(level) + 1 if level else 0
    out: List[List[List[Tuple[int, int]]]] = []
    for lv in range(n_lv):
        mem = [g for g in range(len(groups)) if level[g] == lv]
        load = [0] * n_waves
        assign: List[List[int]] = [[] for _ in range(n_waves)]
        for g in sorted(mem, key=lambda g: (-(groups[g][1] - groups[g][0]), g)):
            w = min(range(n_waves), key=lambda w: (load[w], w))
            assign[w].append(g)
            load[w] += groups[g][1] - groups[g][0]
        out.append([[groups[g] for g in sorted(a)] for a in assign])
    if collect:
        out.append([[(c, c + 1) for c in collect]] + [[] for _ in range(n_waves - 1)])
    return out


def _gibbs_update_levels(tab: np.ndarray, in_cols: np.ndarray):
    """(groups, level, collect) of a Gibbs sweep table: the (begin, end) step range of every node
    update, its level (gibbs_levels), and the COLLECT steps."""
    n = len(tab)
    groups: List[Tuple[int, int]] = []
    collect: List[int] = []
    i = 0
    while i < n:
        role = int(tab[i, S_ROLE])
        if role == ROLE_COLLECT:
            collect.append(i)
            i += 1
            continue
        if role != ROLE_LATENT:
            raise ValueError(f"gibbs_levels: step {i} (role {role}) outside a LATENT .. SELECT group")
        j = i + 1
        while j < n and int(tab[j, S_ROLE]) != ROLE_SELECT:
            if int(tab[j, S_ROLE]) != ROLE_FIXED or not int(tab[j, S_FLAGS]) & F_KEEP:
                raise ValueError(f"gibbs_levels: step {j} is not a child log-prob step")
            j += 1
        if j == n:
            raise ValueError("gibbs_levels: LATENT step without its SELECT")
        groups.append((i, j + 1))
        i = j + 1

    def cols(r):
        return set(range(int(r[S_OUTCOL]), int(r[S_OUTCOL]) + int(r[S_OUTDIM])))

    reads, writes = [], []
    for b, e in groups:
        rd, wr = set(), cols(tab[b])
        for k in range(b, e):
            r = tab[k]
            rd |= set(int(c) for c in in_cols[int(r[S_INOFF]):int(r[S_INOFF]) + int(r[S_NIN])])
            if int(r[S_ROLE]) == ROLE_FIXED:
                rd |= cols(r)
        reads.append(rd)
        writes.append(wr)
    level = []
    for g in range(len(groups)):
        lv = 0
        for h in range(g):
            if writes[h] & (reads[g] | writes[g]) or reads[h] & writes[g]:
                lv = max(lv, level[h] + 1)
        level.append(lv)
    return groups, level, collect


# Relative costs of the sweep's operations for gibbs_schedule: a step with an MLP (or KDE
# scan), a root step (a table lookup and one draw), a SELECT, a workgroup barrier.
_GIBBS_COST_MLP, _GIBBS_COST_ROOT, _GIBBS_COST_SELECT, _GIBBS_COST_BARRIER = 1.0, 0.2, 0.15, 0.1


def _gibbs_step_cost(r) -> float:
    if int(r[S_ROLE]) == ROLE_SELECT:
        return _GIBBS_COST_SELECT
    heavy = int(r[S_WBLK_LEN]) > 0 or int(r[S_KIND]) == KIND_ID["kde"]
    return _GIBBS_COST_MLP if heavy else _GIBBS_COST_ROOT


def _lpt(items: Sequence[Tuple[float, object]], n_waves: int):
    """Longest-processing-time assignment of (cost, item) to n_waves waves: (per-wave items in
    input order, makespan)."""
    load = [0.0] * n_waves
    assign: List[List[int]] = [[] for _ in range(n_waves)]
    for k in sorted(range(len(items)), key=lambda k: (-items[k][0], k)):
        w = min(range(n_waves), key=lambda w: (load[w], w))
        assign[w].append(k)
        load[w] += items[k][0]
    return [[items[k][1] for k in sorted(a)] for a in assign], max(load) if items else 0.0


def gibbs_step_deps(tab: np.ndarray, in_cols: np.ndarray):
    """Step-level ordering constraints of a Gibbs sweep table: {step: set of steps that must run
    before it} over the LATENT / child / SELECT steps (COLLECT steps excluded).

    Inside an update, its children follow its LATENT step and its SELECT follows both.  Between
    updates h < g (sweep order), with slot(u) the slots update u writes (candidates at its LATENT
    step, the choice at its SELECT): a step of g that reads slot(h) runs after h's SELECT, and a
    step of h that reads slot(g) runs before g's LATENT -- so every read sees the value the
    sequential sweep gives it (a child's KEEP write-back rewrites the bits it read: a read)."""
    groups, _, _ = _gibbs_update_levels(tab, in_cols)

    def cols(r):
        return set(range(int(r[S_OUTCOL]), int(r[S_OUTCOL]) + int(r[S_OUTDIM])))

    def reads(i):
        r = tab[i]
        if int(r[S_ROLE]) == ROLE_SELECT:
            return set()
        rd = set(int(c) for c in in_cols[int(r[S_INOFF]):int(r[S_INOFF]) + int(r[S_NIN])])
        return rd | cols(r) if int(r[S_ROLE]) == ROLE_FIXED else rd

    rd = {i: reads(i) for b, e in groups for i in range(b, e)}
    deps = {i: set() for i in rd}
    for b, e in groups:
        for i in range(b + 1, e):
            deps[i].add(b)
        deps[e - 1] |= set(range(b + 1, e - 1))
    for g, (b, e) in enumerate(groups):
        wg = cols(tab[b])
        for bh, eh in groups[:g]:
            wh = cols(tab[bh])
            for i in range(b, e):
                if rd[i] & wh:
                    deps[i].add(eh - 1)
            for i in range(bh, eh):
                if rd[i] & wg:
                    deps[b].add(i)
    return deps


def _gibbs_schedule_dag(tab: np.ndarray, in_cols: np.ndarray, n_waves: int):
    """Phases of any ready steps (gibbs_step_deps), not whole levels: each phase fills the waves
    with the ready steps of the longest remaining path first, up to a per-wave budget; the budget
    with the shortest modelled sweep wins.  Every LATENT / child step scores into its own row."""
    deps = gibbs_step_deps(tab, in_cols)
    cost = {i: _gibbs_step_cost(tab[i]) for i in deps}
    succ = {i: [] for i in deps}
    for j, d in deps.items():
        for i in d:
            succ[i].append(j)
    cp: Dict[int, float] = {}
    for i in sorted(deps, reverse=True):          # a step's successors come later in the table
        cp[i] = cost[i] + max((cp[j] for j in succ[i]), default=0.0)
    groups, _, collect = _gibbs_update_levels(tab, in_cols)
    row_of, n_rows, sel_rows = {}, 0, {}
    for b, e in groups:
        rows = []
        for i in range(b, e - 1):
            row_of[i] = n_rows
            rows.append(n_rows)
            n_rows += 1
        sel_rows[e - 1] = tuple(rows)
    best = None
    env = os.environ.get("VBN_GIBBS_DAG_BUDGET")            # ablation: one per-wave budget
    for budget in ((float(env),) if env else (0.8, 1.0, 1.2, 1.4, 2.0, 3.0, float("inf"))):
        done, phases, t = set(), [], 0.0
        while len(done) < len(deps):
            ready = sorted((i for i in deps if i not in done and deps[i] <= done), key=lambda i: (-cp[i], i))
            load = [0.0] * n_waves
            waves: List[List[int]] = [[] for _ in range(n_waves)]
            for i in ready:
                w = min(range(n_waves), key=lambda w: (load[w], w))
                if load[w] > 0 and load[w] + cost[i] > budget + 1e-9:
                    continue
                load[w] += cost[i]
                waves[w].append(i)
            done |= {i for ws in waves for i in ws}
            t += max(load) + _GIBBS_COST_BARRIER
            phases.append([[("select", i, sel_rows[i]) if i in sel_rows else ("lpout", i, row_of[i])
                            for i in sorted(ws)] for ws in waves])
        if best is None or t < best[0] - 1e-9:
            best = (t, phases)
    phases = best[1]
    if collect:
        phases.append([[("run", c) for c in collect]] + [[] for _ in range(n_waves - 1)])
    return phases, n_rows


def gibbs_schedule(tab: np.ndarray, in_cols: np.ndarray, n_waves: int, split=None):
    """Phased wave schedule of one Gibbs sweep table (csrc vbn_walk_plan.h, chain workgroups).

    The levels are those of gibbs_levels.  A level runs in one of two forms, whichever the cost
    model (_GIBBS_COST_*) says is shorter (``split`` forces one):

    * whole updates: each wave runs whole LATENT .. SELECT groups, the score in its register,
      then one barrier;
    * split updates, for levels whose updates have uneven child counts: phase A runs the LATENT
      steps, phase B every child log-prob step of the level, phase C the SELECT steps, each
      phase balanced over the waves with a barrier after it.  A LATENT or child step starts its
      own score at 0 and stores it in a score row (LDS); the SELECT step adds the rows in sweep
      order -- ((lp_latent + lp_child1) + lp_child2) ..., the same additions as the sequential
      sweep (each child adds one term), so the chains stay bit-identical.

    ``split="levels"`` keeps the per-level choice without the step-level form.
    ``split="dag"`` (and the default, when its modelled sweep is shorter) drops the levels:
    _gibbs_schedule_dag fills each phase with any steps whose constraints (gibbs_step_deps)
    are met, longest remaining path first.

    Returns (phases, n_rows): ``phases`` is a list of per-wave op lists, a barrier after each
    phase; an op is ("run", i) -- step i with the register score --, ("lpout", i, row) or
    ("select", i, rows).  ``n_rows`` is the number of score rows the split steps need.
    """
    if split == "dag":
        return _gibbs_schedule_dag(tab, in_cols, n_waves)
    try_dag = split is None
    if split == "levels":                 # the level forms only, chosen per level by the model
        split = None
    groups, level, collect = _gibbs_update_levels(tab, in_cols)
    n_lv = max(level) + 1 if level else 0
    phases: List[List[List[tuple]]] = []
    n_rows = 0
    for lv in range(n_lv):
        mem = [g for g in range(len(groups)) if level[g] == lv]
        whole_items = [(sum(_gibbs_step_cost(tab[i]) for i in range(*groups[g])), g) for g in mem]
        whole, t_whole = _lpt(whole_items, n_waves)
        t_whole += _GIBBS_COST_BARRIER
        lat, kids, sel = [], [], []
        row = 0
        for g in mem:
            b, e = groups[g]
            rows = list(range(row, row + e - 1 - b))
            row += e - 1 - b
            lat.append((_gibbs_step_cost(tab[b]), ("lpout", b, rows[0])))
            kids += [(_gibbs_step_cost(tab[i]), ("lpout", i, rows[i - b])) for i in range(b + 1, e - 1)]
            sel.append((_gibbs_step_cost(tab[e - 1]), ("select", e - 1, tuple(rows))))
        parts = [_lpt(ph, n_waves) for ph in (lat, kids, sel) if ph]
        t_split = sum(t for _, t in parts) + _GIBBS_COST_BARRIER * len(parts)
        use_split = split if split is not None else t_split < t_whole
        if use_split:
            phases += [p for p, _ in parts]
            n_rows = max(n_rows, row)
        else:
            phases.append([[("run", i) for g in sorted(a) for i in range(*groups[g])] for a in whole])
    if collect:
        phases.append([[("run", c) for c in collect]] + [[] for _ in range(n_waves - 1)])
    if try_dag and n_waves > 1:
        dag = _gibbs_schedule_dag(tab, in_cols, n_waves)
        if gibbs_schedule_cost(dag[0], tab) < gibbs_schedule_cost(phases, tab) - 1e-9:
            return dag
    return phases, n_rows


def gibbs_schedule_cost(phases, tab: np.ndarray) -> float:
    """Modelled sweep time of a gibbs_schedule (the longest wave of each phase, plus barriers)."""
    return sum(max(sum(_gibbs_step_cost(tab[op[1]]) for op in ops) for ops in ph) + _GIBBS_COST_BARRIER
               for ph in phases)



def precompute_width(packed: PackedModel, n: str) -> int:
    """Per-sample quantities of a precomputed node: NN CPDs their MLP head outputs, KDE its 16
    inverse-CDF chunk sums ++ the underflow shift."""
    npk = packed.nodes[n]
    return KDE_CHUNKS + 1 if npk.kind == KIND_ID["kde"] else int(npk.n_out)


def precompute_plans(packed: PackedModel, plan: QueryPlan, *, skip: Sequence[str] = (),
                     exact_f32: bool = False, kde_valu: bool = False, per_query: bool = True
                     ) -> Optional[Tuple[QueryPlan, Optional[QueryPlan], Optional[QueryPlan]]]:
    """Per-sample and per-query precompute of a walk (SURVEY §7 hard part 5).

    A node's MLP head outputs (gaussian_nn, mdn, softmax_nn; latent, or evidence with a
    log-prob) or its KDE inverse-CDF chunk sums (latent kde) depend only on its parents'
    values, which the reference broadcasts and recomputes for every particle
    (``core/utils.py:64-69``, ``gaussian_nn.py:215-241``, ``kde.py:131-146``).  Two cases are
    functions of fewer than B x S inputs:

    * **per sample** -- parents all latent roots with draws shared by every query (MCM / LW /
      ancestral, Q5): a one-query pre-pass walk (the same root steps -- same flags, so the same
      Philox draws and Box-Muller pairs -- then those nodes with VBN_F_PRE_OUT) computes them
      once per sample; the main walk's steps read row s (VBN_F_PRECOMP);
    * **per query** -- parents all evidence / do values (every engine, IS included): a pre-pass
      of one wave per query (B x 64 particles, every lane of a wave the same inputs) computes
      them once per query; the main walk's steps read row b (VBN_F_PRECOMP | VBN_F_PRECOMP_Q,
      wave-uniform scalar loads).

    Either way the main walk then runs the node's epilogue and its own per-particle draws as
    before.  Same device functions on the same values: the outputs are bit-identical to the
    plain walk when every wave holds one query (S a multiple of 64: the MLP's wave-uniform
    exact-path decision then sees the same inputs in the pre-pass wave and in the main wave;
    run_walk checks).  Returns (main plan, per-sample pre-pass or None, per-query pre-pass or
    None), or None when no node qualifies.
    """
    model = packed.model
    rows = plan.steps._vbn_host[0].copy()
    order = list(plan.order) if plan.order is not None else [n for n in model.topo if n not in set(skip)]
    assert len(order) == len(rows)
    at = {n: i for i, n in enumerate(order)}
    roots = [n for n in order if rows[at[n]][S_ROLE] == ROLE_LATENT and rows[at[n]][S_FLAGS] & F_SHARED]
    root_s = set(roots)
    fixed = [n for n in order if rows[at[n]][S_ROLE] == ROLE_FIXED]
    fixed_s = set(fixed)
    nn_kinds = (KIND_ID["gaussian_nn"], KIND_ID["mdn"], KIND_ID["softmax_nn"])

    def qualifies(n: str) -> bool:
        r = rows[at[n]]
        if r[S_FLAGS] & (F_ROOT | F_SHARED) or not model.parents[n]:
            return False
        kind, role = int(r[S_KIND]), int(r[S_ROLE])
        if kind in nn_kinds and not r[S_FLAGS] & F_MLP_GENERIC:
            return role == ROLE_LATENT or (role == ROLE_FIXED and bool(r[S_FLAGS] & F_LOGP))
        # a KDE node with a moment table computes its chunk sums from the table in a few FMAs;
        # precomputing them would only force the pre-pass's 16 coarse chunks on its scan
        return (kind == KIND_ID["kde"] and role == ROLE_LATENT and not r[S_FLAGS] & F_KDE_VALU
                and r[S_OFF_KQ] >= 0 and r[S_RES7] < 0)

    cand_s = [n for n in order if qualifies(n) and all(p in root_s for p in model.parents[n])]
    cand_q = [n for n in order if per_query and qualifies(n) and all(p in fixed_s for p in model.parents[n])]
    # an evidence candidate's pre-pass slot holds its head outputs, not its value: one that is a
    # parent of another candidate stays per particle
    cand_q = [n for n in cand_q if not (n in fixed_s and any(n in model.parents[m] for m in cand_q))]
    if not cand_s and not cand_q:
        return None
    pre = pre_q = None
    if cand_s:
        keep = root_s | set(cand_s)
        porder = [n for n in order if n in keep]         # the main walk's order: its Box-Muller pairs
        pre = build_plan(packed, latent=roots + cand_s, fixed=[], logp=[], out_nodes=cand_s, shared_roots=True,
                         mode=MODE_SAMPLE, skip=[n for n in model.topo if n not in keep], exact_f32=exact_f32,
                         pre_out=cand_s, order=porder)
        prow = pre.steps._vbn_host[0].copy()
        for i, n in enumerate(porder):               # the main walk's Box-Muller pairs (roots pair
            prow[i][S_FLAGS] &= ~(F_BM_FIRST | F_BM_SECOND)        # with roots only) and no others
            if n in root_s:
                prow[i][S_FLAGS] |= rows[at[n]][S_FLAGS] & (F_BM_FIRST | F_BM_SECOND)
        pre = _with_steps(pre, prow, packed.device)
    if cand_q:
        # the main walk's fixed nodes, reading the main walk's fixed buffer (its columns), then
        # the candidates writing their quantities (an evidence candidate is one of them)
        cq = set(cand_q)
        keep = fixed_s | cq
        qorder = [n for n in order if n in keep]
        pre_q = build_plan(packed, latent=cand_q, fixed=[n for n in fixed if n not in cq], logp=[],
                           out_nodes=cand_q, shared_roots=False, mode=MODE_SAMPLE,
                           skip=[n for n in model.topo if n not in keep], exact_f32=exact_f32, pre_out=cand_q,
                           order=qorder)
        qrow = pre_q.steps._vbn_host[0].copy()
        qrow[:, S_FLAGS] &= ~(F_BM_FIRST | F_BM_SECOND)          # PRE_OUT steps draw no normals
        for i, n in enumerate(qorder):
            if n not in cq:
                qrow[i][S_FIXEDCOL] = rows[at[n]][S_FIXEDCOL]
                qrow[i][S_FLAGS] |= rows[at[n]][S_FLAGS] & F_CLAMP_EV    # LW: clamped evidence
        import dataclasses
        pre_q = dataclasses.replace(_with_steps(pre_q, qrow, packed.device), fixed_nodes=list(plan.fixed_nodes),
                                    fixed_ld=plan.fixed_ld)
    for cands, extra in ((cand_s, 0), (cand_q, F_PRECOMP_Q)):
        stride = sum(precompute_width(packed, n) for n in cands)
        if extra and 64 * stride < (1 << 15):
            # the per-query pre-pass writes 64 identical rows per query: the walk reads row
            # 64 b of its out_x in place (stride 64 x width, engines.run_walk), no gather copy
            stride *= 64
        assert stride < (1 << 15)
        col = 0
        for n in cands:
            r = rows[at[n]]
            r[S_FLAGS] |= F_PRECOMP | extra
            r[S_AUX2] = col | (stride << 16)
            col += precompute_width(packed, n)
            r[S_WBLK_OFF] = 0                        # no MLP runs: nothing to stage
            r[S_WBLK_LEN] = 0
    return _with_steps(plan, rows, packed.device), pre, pre_q


def _with_steps(plan: QueryPlan, rows: np.ndarray, device) -> QueryPlan:
    """A copy of ``plan`` with another step table (same slots, parent lists and outputs)."""
    import dataclasses
    steps_t = torch.from_numpy(np.ascontiguousarray(rows)).to(device)
    steps_t._vbn_wblk_max = int(rows[:, S_WBLK_LEN].max()) if len(rows) else 0
    pc = (rows[:, S_FLAGS] & F_PRECOMP) != 0
    pq = (rows[:, S_FLAGS] & F_PRECOMP_Q) != 0
    for m, attr in ((pc & ~pq, "_vbn_precomp_stride"), (pq, "_vbn_precomp_q_stride")):
        if m.any():                                  # ops.walk checks the precomp tensors' widths
            setattr(steps_t, attr, int(rows[m, S_AUX2][0]) >> 16)
    ic_host = plan.steps._vbn_host[1]
    steps_t._vbn_host = (rows.copy(), ic_host.copy(),
                         hashlib.sha1(rows.tobytes() + b"|" + ic_host.tobytes()).hexdigest())
    return dataclasses.replace(plan, steps=steps_t, wbuf=steps_t._vbn_wblk_max, pc=None, pre=None, pre_q=None)
