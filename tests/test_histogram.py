"""Discrete weighted histogram: oracle pin and the kernel's algorithm on CPU.

* The oracle restatement (oracle/vbn_oracle.py estimate_discrete_posterior_batch) reproduces
  the reference adapter's outputs recorded in tests/golden/discrete_hist.pt bit for bit,
  including the exception types of its two error cases.
* The kernel's numpy pairwise sum (csrc/vbn_walk.hip np_pairwise_sum) restated here on the
  host equals ``np.ndarray.sum`` bit for bit, so the device normalisation is numpy's.
"""
import math
import os

import numpy as np
import pytest
import torch

from oracle import vbn_oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = os.path.join(HERE, "golden", "discrete_hist.pt")


def _cases():
    return torch.load(FIX, weights_only=True)["cases"]


@pytest.mark.parametrize("case", _cases(), ids=lambda c: c["name"])
def test_oracle_matches_reference_fixture(case):
    if case.get("error"):
        with pytest.raises((ValueError, OverflowError)) as ei:
            O.estimate_discrete_posterior_batch(case["samples"], case["weights"], case["k"])
        assert type(ei.value).__name__ == case["error"]
        return
    got = torch.tensor(O.estimate_discrete_posterior_batch(case["samples"], case["weights"], case["k"]),
                       dtype=torch.float64)
    assert torch.equal(got, case["probs"])


def _pairwise(a, n, st=1, depth=24):
    """Host replica of the kernel's np_pairwise_sum<24>."""
    if n < 8:
        r = 0.0
        for i in range(n):
            r += a[i * st]
        return r
    if n <= 128 or depth == 0:
        r = [a[j * st] for j in range(8)]
        i = 8
        while i < n - (n % 8):
            for j in range(8):
                r[j] += a[(i + j) * st]
            i += 8
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
        while i < n:
            res += a[i * st]
            i += 1
        return res
    n2 = n // 2
    n2 -= n2 % 8
    return _pairwise(a, n2, st, depth - 1) + _pairwise(a[n2 * st:], n - n2, st, depth - 1)


@pytest.mark.parametrize("n", [0, 1, 5, 7, 8, 9, 15, 16, 17, 100, 127, 128, 129, 200, 255, 256, 257, 1000, 4099])
def test_kernel_pairwise_sum_is_numpys(n):
    rng = np.random.default_rng(n)
    a = rng.standard_normal(n) * np.power(10.0, rng.integers(-12, 12, n))
    want = float(a.sum())
    got = 0.0 + _pairwise([float(x) for x in a], n)
    assert got == want or (math.isnan(got) and math.isnan(want))
