"""bench.py's own multi-rank launch, on the CPU.

`bench.py --gpus N` with no launcher around it must start N rank processes
itself (python_ldpc_app/main.py:248-291 starts its own worker pool), report
the ranks that answered on the communicator, and fail loudly -- never report
one rank for --gpus N.  --stub replaces the GPU rank body with a gloo group
that only counts the ranks, so the launcher logic runs here."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def run(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "LDPC_RDV_KEY")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True,
                          timeout=timeout)


@pytest.mark.parametrize("n", [2, 3])
def test_self_launch_starts_n_ranks(n):
    r = run(["--gpus", str(n), "--stub"])
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # only rank 0 prints its line (gloo's own chatter aside)
    out = json.loads(lines[0])
    assert out["stub"] and out["n_gpus"] == n and out["ranks_seen"] == n and out["world_size"] == n
    assert out["rdv_key_set"]  # one rendezvous key per launch (ldpc_amd.comm)


def test_one_gpu_runs_in_process():
    r = run(["--gpus", "1", "--stub"], {"WORLD_SIZE": "1", "RANK": "0", "MASTER_PORT": "0"})
    # a launcher-provided world of 1: no children, no rendezvous key
    assert r.returncode == 0, r.stderr
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["ranks_seen"] == 1 and not out["rdv_key_set"]


def test_launcher_world_mismatch_fails():
    r = run(["--gpus", "8", "--stub"], {"WORLD_SIZE": "1", "RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=1" in (r.stderr + r.stdout)


def test_failing_rank_fails_the_launch():
    # no GPU here: every real rank exits with "no HIP device"; the launch must
    # exit non-zero instead of printing a one-rank line
    r = run(["--gpus", "2", "--cpu-seconds", "0"], {"HIP_VISIBLE_DEVICES": ""})
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
