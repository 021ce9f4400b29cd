#!/usr/bin/env python3
"""Golden fixtures for the discrete weighted histogram (build container only).

Runs the reference benchmark adapter's ``_estimate_discrete_posterior_batch``
(benchmarking/models/vbn.py:226-242) on seeded synthetic samples / weights: half-integer
samples (round half to even), values outside [0, k), NaN / inf / negative weights, all-NaN and
negative-total rows (uniform), weights spanning 1e-30 .. 1e30 (the float64 summation order
matters), 3-D samples, k above and below the kernel's 128-bin LDS limit, and the two error
cases (NaN / inf sample with a finite weight).

Writes ``tests/golden/discrete_hist.pt`` (tensors and builtins only).
Usage: python tests/golden/make_golden_histogram.py [--out tests/golden]
"""
from __future__ import annotations

import argparse
import os
import sys

# one OpenMP / MKL thread, fixed before torch loads: the reference's fits (linear_gaussian's
# lstsq, the NN epochs) then reproduce bit for bit from run to run (under the default thread
# pool the ridge weights drifted by up to 2.4e-7 between regenerations)
os.environ["OMP_NUM_THREADS"] = "1"
os.environ["MKL_NUM_THREADS"] = "1"

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("VBN_REFERENCE", "/root/reference")


def _cases():
    g = torch.Generator().manual_seed(2024)
    out = []

    def add(name, samples, weights, k):
        out.append({"name": name, "samples": samples, "weights": weights, "k": k})

    # plain: half-integers included, some values outside the support
    s = (torch.randint(-4, 14, (4, 1000), generator=g).float() / 2.0)
    w = torch.rand(4, 1000, generator=g)
    add("halves", s, w, 5)
    # non-finite / negative weights, a row of NaN weights, a row summing to <= 0
    s = torch.rand(5, 700, generator=g) * 7.0 - 1.0
    w = torch.randn(5, 700, generator=g).abs()
    w[0, ::7] = float("nan")
    w[1, ::11] = float("inf")
    w[1, 3::13] = float("-inf")
    w[2] = float("nan")
    w[3] = -w[3]
    w[4, ::2] = -w[4, ::2]
    add("nonfinite_weights", s, w, 6)
    # weights across many decades: the float64 summation order shows
    s = torch.randint(0, 3, (3, 4096), generator=g).float() + (torch.rand(3, 4096, generator=g) - 0.5) * 0.9
    e = torch.randint(-30, 31, (3, 4096), generator=g).float()
    w = (torch.rand(3, 4096, generator=g) + 0.5) * torch.pow(10.0, e)
    add("decades", s, w, 3)
    # 3-D samples (feature 0 is binned)
    s = torch.rand(2, 512, 3, generator=g) * 4.0
    w = torch.rand(2, 512, generator=g)
    add("three_d", s, w, 4)
    # many bins (above the 128-bin LDS limit) and exactly at it
    s = torch.rand(3, 3000, generator=g) * 210.0 - 5.0
    w = torch.rand(3, 3000, generator=g) * 3.0
    add("k200", s, w, 200)
    s = torch.rand(2, 2000, generator=g) * 130.0
    w = torch.rand(2, 2000, generator=g)
    add("k128", s, w, 128)
    add("k9", torch.rand(2, 300, generator=g) * 9.0, torch.rand(2, 300, generator=g), 9)
    add("k1", torch.rand(2, 64, generator=g) * 2.0 - 0.5, torch.rand(2, 64, generator=g), 1)
    # a larger batch (many lanes / workgroups)
    s = torch.randint(0, 8, (300, 256), generator=g).float()
    w = torch.rand(300, 256, generator=g)
    add("batch300", s, w, 8)
    # float64 inputs: half-integers off by 1e-12 bin by their own value (a float32
    # cast would round them onto the half and to even), weights 1 + O(1e-12) sum in float64
    base = torch.randint(0, 6, (3, 800), generator=g).double() + 0.5
    off = torch.where(torch.rand(3, 800, generator=g, dtype=torch.float64) < 0.5, 1e-12, -1e-12)
    w = 1.0 + torch.rand(3, 800, generator=g, dtype=torch.float64) * 1e-12
    add("f64_both", base + off, w, 6)
    add("f64_samples_f32_weights", base - off, torch.rand(3, 800, generator=g), 6)
    add("f32_samples_f64_weights", torch.randint(0, 4, (2, 500), generator=g).float(),
        torch.rand(2, 500, generator=g, dtype=torch.float64) * 1e-300, 4)
    return out


def _error_cases():
    s = torch.tensor([[0.0, 1.0, float("nan"), 2.0], [1.0, 1.0, 1.0, 1.0]])
    w = torch.ones(2, 4)
    e1 = {"name": "nan_sample", "samples": s, "weights": w, "k": 3}
    s2 = torch.tensor([[0.0, 1.0, 2.0], [1.0, float("inf"), 0.0]])
    e2 = {"name": "inf_sample", "samples": s2, "weights": torch.ones(2, 3), "k": 3}
    s3 = torch.tensor([[0.0, float("nan"), 2.0]])
    e3 = {"name": "nan_sample_nan_weight", "samples": s3, "weights": torch.tensor([[1.0, float("nan"), 1.0]]),
          "k": 3}
    return [e1, e2, e3]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=HERE)
    args = ap.parse_args()
    if not os.path.isdir(os.path.join(REF, "benchmarking")):
        print(f"reference not found at {REF}; nothing to do")
        return 0
    sys.path.insert(0, REF)
    from benchmarking.models.vbn import _estimate_discrete_posterior_batch as ref

    cases = []
    for c in _cases():
        probs = ref(c["samples"], c["weights"], c["k"])
        c["probs"] = torch.tensor(probs, dtype=torch.float64)
        cases.append(c)
    for c in _error_cases():
        try:
            probs = ref(c["samples"], c["weights"], c["k"])
            c["error"] = ""
            c["probs"] = torch.tensor(probs, dtype=torch.float64)
        except Exception as ex:  # noqa: BLE001 -- the exception type is the recorded output
            c["error"] = type(ex).__name__
            c["message"] = str(ex)
        cases.append(c)
    path = os.path.join(args.out, "discrete_hist.pt")
    torch.save({"cases": cases}, path)
    print(f"wrote {path}: {len(cases)} cases")
    return 0


if __name__ == "__main__":
    sys.exit(main())
