"""bench.py --gpus N without a torch.distributed launcher spawns the N rank
processes itself; rehearsed on the CPU with gloo (GPUFLOW_BENCH_SELFTEST):
rendezvous, the counter-block all-reduce, the timing max and the single JSON
line of rank 0."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(n):
    env = dict(os.environ, GPUFLOW_BENCH_SELFTEST="1")
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n)], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def test_launcher_spawns_world_2_and_all_reduces():
    r = _run(2)
    assert r["n_gpus"] == 2
    # each rank counts 1000 + rank packets and rank + 1 policy drops; rank 1 takes 0.6 s
    assert r["verdicts"]["drop_reasons"] == {"133": 3}
    assert r["ms_per_step"] == 600.0
    assert abs(r["value"] - 2001 / 0.6 / 1e6) < 1e-6


def test_launcher_single_rank():
    r = _run(1)
    assert r["n_gpus"] == 1 and r["verdicts"]["drop_reasons"] == {"133": 1}
