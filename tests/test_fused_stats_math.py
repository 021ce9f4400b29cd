"""Host replica of the fused posterior summary's arithmetic (csrc vbn_walk_impl.h stats_partials:
per-64-particle float64 rows; vbn_walk.hip vbn_stats_merge_kernel: Chan's pairwise merge) against
the oracle's VBN._posterior_stats (vbn.py:483-504) -- the decomposition itself, on CPU, including
zero-weight waves, all-zero rows (uniform weights) and NaN samples.  The GPU kernels are checked
against the same oracle in tests/test_gpu_fused_stats.py."""
import numpy as np
import pytest
import torch

from oracle import vbn_oracle as O


def _partials(pdf, x):
    """stats_partials for every wave: rows [B, S/64, 2 + 4 D]."""
    b, s, d = x.shape
    w = np.nan_to_num(pdf.astype(np.float64), nan=0.0, posinf=0.0, neginf=0.0).clip(min=0.0)
    w = w.reshape(b, s // 64, 64)
    xx = x.astype(np.float64).reshape(b, s // 64, 64, d)
    W = w.sum(-1)
    Q = (w * w).sum(-1)
    rows = [W[..., None], Q[..., None]]
    for k in range(d):
        xk = xx[..., k]
        sx = (w * xk).sum(-1)
        with np.errstate(invalid="ignore", divide="ignore"):
            mw = np.where(W > 0, sx / np.where(W > 0, W, 1.0), sx)
        m2w = (w * (xk - mw[..., None]) ** 2).sum(-1)
        mu = xk.sum(-1) / 64.0
        m2u = ((xk - mu[..., None]) ** 2).sum(-1)
        rows += [mw[..., None], m2w[..., None], mu[..., None], m2u[..., None]]
    return np.concatenate(rows, -1)


def _merge(part, d, eps):
    """vbn_stats_merge_kernel."""
    b, n_parts, _ = part.shape
    W = part[..., 0].sum(-1)
    Q = part[..., 1].sum(-1)
    S = 64.0 * n_parts
    mean = np.zeros((b, d), np.float32)
    std = np.zeros((b, d), np.float32)
    ess = np.zeros(b, np.float32)
    for i in range(b):
        ok = W[i] > eps
        if ok:
            ess[i] = 1.0 / max(np.float32(Q[i] / (W[i] * W[i])), np.float32(eps))
        else:
            uni = np.float32(1.0) / np.float32(64 * n_parts)
            ess[i] = np.float32(1.0) / max(np.float32(64 * n_parts) * (uni * uni), np.float32(eps))
        for k in range(d):
            o = 2 + 4 * k + (0 if ok else 2)
            wk = part[i, :, 0] if ok else np.full(n_parts, 64.0)
            m = (wk * part[i, :, o]).sum() / (W[i] if ok else S)
            m2 = (part[i, :, o + 1] + wk * (part[i, :, o] - m) ** 2).sum()
            mean[i, k] = m
            std[i, k] = np.sqrt(max(np.float32(m2 / (W[i] if ok else S)), np.float32(0.0)))
    return mean, std, ess


@pytest.mark.parametrize("s,d", [(64, 1), (1024, 1), (2048, 3)])
def test_wave_partials_merge_to_the_reference_summary(s, d):
    g = torch.Generator().manual_seed(s + d)
    b = 6
    pdf = torch.rand(b, s, generator=g) * 2.0
    x = torch.randn(b, s, d, generator=g) * 3.0 + 5.0          # |mean| >> std: cancellation test
    pdf[1, :64] = 0.0                                           # a zero-weight wave
    pdf[2] = 0.0                                                # all zero: uniform weights
    pdf[3, 5] = float("nan")                                    # nan -> 0
    pdf[3, 6] = float("inf")                                    # inf -> 0
    pdf[4] = torch.exp(torch.randn(s, generator=g) * 20.0)      # wide dynamic range
    x[5, s - 1, 0] = float("nan")                               # a NaN sample with weight
    pdf[0, 3] = 0.0
    x[0, 3, 0] = float("nan")                                   # a NaN sample with weight 0
    mean, std, ess = _merge(_partials(pdf.numpy(), x.numpy()), d, 1e-12)
    ref = O.posterior_stats(pdf.double(), x.double(), 1e-12)
    torch.testing.assert_close(torch.from_numpy(mean).double(), ref["mean"], rtol=1e-5, atol=1e-6, equal_nan=True)
    torch.testing.assert_close(torch.from_numpy(std).double(), ref["std"], rtol=1e-5, atol=1e-6, equal_nan=True)
    torch.testing.assert_close(torch.from_numpy(ess).double(), ref["ess"], rtol=1e-5, atol=1e-6, equal_nan=True)
    assert torch.isnan(torch.from_numpy(mean)[0, 0]) and torch.isnan(ref["mean"][0, 0])
