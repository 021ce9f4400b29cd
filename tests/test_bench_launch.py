"""bench.py's rank launch: ``--gpus N`` without a launcher starts N rank
processes (torch.distributed.run children, 127.0.0.1 rendezvous), the JSON line reports the
process group's size and the ranks it saw, and a launcher whose WORLD_SIZE disagrees with
``--gpus`` is refused.  ``--stub`` runs the launch / rank / reporting path with no GPU work
(gloo), so these run on CPU."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _run(args, env_extra=None, timeout=240):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    env["OMP_NUM_THREADS"] = "1"
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True,
                          timeout=timeout, env=env, cwd=REPO)


def _json(r):
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, (r.stdout, r.stderr[-2000:])
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [1, 2])
def test_gpus_n_launches_n_ranks(n):
    r = _run(["--gpus", str(n), "--stub", "--steps", "1", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-3000:]
    out = _json(r)
    assert out["n_gpus"] == n
    assert out["ranks_seen"] == list(range(n))


def test_world_size_mismatch_is_refused():
    r = _run(["--gpus", "1", "--stub"], env_extra={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE=2" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_gpus_must_be_positive():
    r = _run(["--gpus", "0", "--stub"])
    assert r.returncode != 0
