"""bench.py's multi-GPU launch path on CPU (VERDICT r02 "bench.py --gpus N is parsed and
ignored"): `python bench.py --gpus 2` without a launcher must start two ranks itself, and a
launcher whose WORLD_SIZE disagrees with --gpus must make it exit non-zero -- it can never
print n_gpus: 1 for a 2-GPU request.  --plumbing runs the launch / barrier / all-reduce path
on gloo without a GPU or a solve."""
import json
import os
import subprocess
import sys

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _env():
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e["OMP_NUM_THREADS"] = "1"
    return e


def test_bench_gpus2_spawns_two_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--plumbing", "--steps", "3", "--warmup", "1"],
                       capture_output=True, text=True, timeout=240, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout                      # rank 0 only
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["ranks_reporting"] == 2 and line["plumbing"] is True
    assert "rank 0/2 reporting" in r.stderr and "rank 1/2 reporting" in r.stderr


def test_bench_world_size_mismatch_exits_nonzero():
    e = _env()
    e.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--plumbing"], capture_output=True, text=True,
                       timeout=120, env=e, cwd=ROOT)
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr
    assert '"n_gpus"' not in r.stdout
