#!/usr/bin/env python3
"""Precompile the Gibbs sweep units the GPU tests and the Gibbs bench load (CPU, hiprtc) into the
package's plan cache, so `pytest -m gpu` on a fresh box does not spend minutes in hiprtc.

    python scripts/precompile_gibbs_tests.py

The kind set of each launch is the library's own (`vbn_hip_walk_kind_set` on the arguments
`ops.gibbs_walk` builds, | 256 without injected draws) and the schedule is `plan.gibbs_schedule`
with the test's `VBN_GIBBS_SPLIT`, so the source -- and the cache key -- are the ones
`jit.module_for` computes.  A unit the tests no longer load only costs disk.
"""
from __future__ import annotations

import ctypes
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

SPLIT = {"": None, "0": False, "1": True, "dag": "dag", "levels": "levels"}

# (wave_particles, chain_waves, VBN_GIBBS_SPLIT): tests/test_gpu_jit.py
# test_chain_workgroup_gibbs_bit_identical + test_specialised_gibbs_sweeps_bit_identical (auto
# chain waves: 8) + the Gibbs bench (full wave, 8 waves)
CFG2_CASES = [(32, 1, ""), (32, 2, ""), (32, 4, ""), (64, 1, ""), (64, 2, ""), (64, 4, ""), (32, 2, "1"),
              (64, 4, "1"), (32, 4, "0"), (64, 8, ""), (32, 8, "1"), (64, 0, ""), (32, 0, ""), (64, 8, "levels"),
              (32, 2, "dag"), (32, 8, ""), (64, 8, "0")]


def _kind_set(gp, pk, n_chains, wp, noise):
    from vectorizedbayesiannetwork_amd import _lib
    from vectorizedbayesiannetwork_amd.plan import MODE_GIBBS
    import torch
    lib = _lib.load()
    dummy = torch.zeros(16)
    a = _lib.VbnWalkArgs()
    a.steps = gp.steps.data_ptr()
    a.in_cols = gp.in_cols.data_ptr()
    a.params = a.fixed = a.out_x = a.state = dummy.data_ptr()
    a.out_cols = gp.in_cols.data_ptr()
    a.noise = dummy.data_ptr() if noise else None
    a.n_queries, a.n_samples, a.n_steps = n_chains, 8, gp.n_steps
    a.state_flags, a.n_slots, a.max_out, a.fixed_ld = 1, gp.init.n_slots, gp.init.max_out, gp.init.fixed_ld
    a.noise_b, a.dmax, a.n_out_cols, a.mode, a.kind_mask = n_chains, pk.dmax, 1, MODE_GIBBS, gp.kind_mask
    a.gibbs_iters, a.gibbs_burn_in, a.gibbs_thin, a.n_noise = 4, 1, 1, gp.n_noise
    a.wbuf_floats, a.wave_particles = gp.wbuf, wp
    km = lib.vbn_hip_walk_kind_set(ctypes.byref(a))
    if km <= 0:
        raise RuntimeError(f"kind set: error {km}")
    return km | (0 if noise else 256)              # ops._plan_module


def _units():
    """(label, steps, in_cols, kind set, chain waves, split) of every unit to compile."""
    import torch
    import bench
    from conftest import load_golden
    from vectorizedbayesiannetwork_amd import plan as P
    from vectorizedbayesiannetwork_amd.model import model_from_checkpoint
    out = []
    cfg, model, target, ev = bench.build_model("cfg2")
    pk = P.PackedModel(model, torch.device("cpu"))
    gp = P.build_gibbs_plan(pk, latent=[n for n in model.topo if n not in ev],
                            fixed=[n for n in model.topo if n in ev], target=target)
    rows, ic, _ = gp.steps._vbn_host
    for wp, cw, split in CFG2_CASES:
        out.append((f"cfg2 wp{wp} cw{cw} split'{split}'", rows, ic, _kind_set(gp, pk, 13, wp, False), cw, split))
    # recorded draws (injected noise): the oracle tests, chain_waves 4, full wave
    for name in ("ext_gibbs_mix10", "ext_gibbs_kde6"):
        fx = load_golden(name)
        m = model_from_checkpoint(fx["model"])
        pkm = P.PackedModel(m, torch.device("cpu"))
        for case in fx["cases"][:2]:
            q = case["query"]
            fixed = set(q["evidence"]) | set(q["do"])
            g = P.build_gibbs_plan(pkm, latent=[n for n in m.topo if n not in fixed],
                                   fixed=[n for n in m.topo if n in fixed], target=q["target"])
            r, i, _ = g.steps._vbn_host
            km = _kind_set(g, pkm, 4, 64, True)
            for split in ("", "1"):
                out.append((f"{name} {q['target']} split'{split}'", r, i, km, 4, split))
    return out


def _compile(unit):
    label, rows, ic, km, cw, split = unit
    from vectorizedbayesiannetwork_amd import jit
    from vectorizedbayesiannetwork_amd.plan import gibbs_schedule
    schedule = gibbs_schedule(rows, ic, cw, split=SPLIT[split]) if cw > 0 else None
    src = jit.plan_source(rows, ic, km, schedule)
    key = jit._source_key(src)
    if jit._cached_code(key) is not None:
        return f"{label}: {key} (cached)"
    t0 = time.perf_counter()
    jit._compile_store(src, key)
    return f"{label}: {key} (compiled in {time.perf_counter() - t0:.1f} s)"


def main():
    units = _units()
    seen, uniq = set(), []
    for u in units:                                # identical sources compile once
        k = (u[1].tobytes(), u[2].tobytes(), u[3], u[4], u[5] if u[4] > 0 else "")
        if k not in seen:
            seen.add(k)
            uniq.append(u)
    with ProcessPoolExecutor(max(1, min(8, os.cpu_count() or 1))) as ex:
        for line in ex.map(_compile, uniq):
            print(line, flush=True)


if __name__ == "__main__":
    main()
