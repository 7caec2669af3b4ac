"""bench.py --gpus N started with no launcher (the way the driver's N = 1 line is started, with a
larger N): the script runs torch.distributed.run itself as a child process, every rank joins one
process group, and rank 0 prints the JSON line with the world size the group saw. CPU only:
--dry-run stops after the rendezvous (gloo), before any GPU call."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_gpus2_without_launcher_starts_two_ranks():
    env = dict(os.environ, AK_BENCH_BACKEND="gloo")
    env.pop("RANK", None)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rows", "200000", "--no-cpu",
                        "--dry-run"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["world_size"] == 2 and rec["requested_gpus"] == 2
    assert "launching 2 ranks" in p.stderr
