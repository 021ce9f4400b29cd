"""Discrete weighted posterior of a target (the benchmark adapter's consumer).

Mirrors the reference's ``_estimate_discrete_posterior`` / ``_estimate_discrete_posterior_batch``
(benchmarking/models/vbn.py:202-242, normalisation ``_normalize_probs`` 116-121): the weights
and samples ``VBN.infer_posterior`` returns are binned on the GPU in one launch
(``vbn_hip::discrete_posterior``), one lane per query in sample order, so the float64 bins are
the reference's bit for bit and the normalisation uses numpy's pairwise sum.  Same argument
handling, same error types and messages; the lists are built from one device-to-host copy.
``discrete_posterior`` keeps the result on the device ([B, k] float64).
"""
from __future__ import annotations

from typing import List, Tuple

import torch

from . import ops


def _raise_bad(bad: torch.Tensor) -> None:
    nz = torch.nonzero(bad).flatten()
    if nz.numel():
        code = int(bad[int(nz[0])])
        if code == 1:
            raise ValueError("cannot convert float NaN to integer")
        raise OverflowError("cannot convert float infinity to integer")


def _check_k(k) -> int:
    k = int(k)
    if k < 0:
        raise ValueError("negative dimensions are not allowed")
    return k


def _device_pair(samples: torch.Tensor, weights: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    dev = weights.device if weights.is_cuda else (samples.device if samples.is_cuda else None)
    if dev is None:
        raise RuntimeError("discrete_posterior: the HIP path needs GPU tensors (no CPU fallback)")
    return samples.to(dev), weights.to(dev)


def discrete_posterior(samples: torch.Tensor, weights: torch.Tensor, k: int) -> torch.Tensor:
    """Batch form on the device: samples [B,S] or [B,S,D] (feature 0), weights [B,S] ->
    probs [B,k] float64 (benchmarking/models/vbn.py:226-242 without the list conversion)."""
    if samples.dim() == 3:
        samples = samples[:, :, 0]
    if samples.dim() != 2:
        raise ValueError(f"Expected samples with 2D shape, got {tuple(samples.shape)}")
    if weights.dim() != 2:
        raise ValueError(f"Expected weights with 2D shape, got {tuple(weights.shape)}")
    if samples.shape[0] != weights.shape[0]:
        raise ValueError("Samples/weights batch size mismatch")
    k = _check_k(k)
    b = samples.shape[0]
    if samples.shape[1] != weights.shape[1]:          # zip() pairs the shorter length
        n = min(samples.shape[1], weights.shape[1])
        samples, weights = samples[:, :n], weights[:, :n]
    if k == 0:
        return torch.empty(b, 0, dtype=torch.float64, device=weights.device)
    samples, weights = _device_pair(samples.detach(), weights.detach())
    probs, bad = ops.discrete_posterior(samples, weights, k)
    _raise_bad(bad)
    return probs


def estimate_discrete_posterior_batch(samples: torch.Tensor, weights: torch.Tensor, k: int) -> List[List[float]]:
    """reference benchmarking/models/vbn.py:226-242."""
    return discrete_posterior(samples, weights, k).cpu().tolist()


def estimate_discrete_posterior(samples: torch.Tensor, weights: torch.Tensor, k: int) -> List[float]:
    """reference benchmarking/models/vbn.py:202-223: the first query of a batch, flattened."""
    if samples.dim() == 3:
        samples = samples[:, :, 0]
    if samples.dim() == 2:
        samples = samples[0]
    if weights.dim() == 2:
        weights = weights[0]
    vals = samples.reshape(1, -1)
    wts = weights.reshape(1, -1)
    return estimate_discrete_posterior_batch(vals, wts, k)[0]
