"""bench.py's multi-GPU launcher on CPU (--dry-run: gloo, stand-in workload).

`python bench.py --gpus N` outside torch.distributed.run starts N rank
processes itself; these tests run that path with N = 2 and check the JSON
line's n_gpus, that every rank took part in the reductions, that a failing
rank ends the job with its exit code instead of a hang, and that --gpus must
agree with a WORLD_SIZE set by torch.distributed.run."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(OMP_NUM_THREADS="1", **kw)
    return env


def _run(args, **env):
    return subprocess.run([sys.executable, BENCH, *args], env=_env(**env), capture_output=True, text=True,
                          timeout=180, cwd="/tmp")


def test_dry_run_two_ranks_prints_one_line_with_n_gpus():
    p = _run(["--gpus", "2", "--dry-run", "--steps", "2", "--warmup", "1"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["ranks_seen"] == 2
    assert d["steps"] == 2 and d["scaling"] == "weak"
    # whole-job rate: both ranks' steps over the slowest rank's time
    assert abs(d["value"] - 2 * d["steps"] / (d["ms_per_step"] * d["steps"] / 1e3)) < 1e-3 * d["value"] + 1e-3


def test_dry_run_single_rank():
    p = _run(["--dry-run", "--steps", "1", "--warmup", "0"])
    assert p.returncode == 0, p.stderr[-2000:]
    assert json.loads(p.stdout.strip().splitlines()[-1])["n_gpus"] == 1


def test_failing_rank_stops_the_job():
    p = _run(["--gpus", "2", "--dry-run", "--steps", "2", "--warmup", "1"], FCS_BENCH_DRY_FAIL_RANK="1")
    assert p.returncode == 3
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_gpus_must_match_world_size():
    p = _run(["--gpus", "2", "--dry-run"], WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    assert p.returncode != 0 and "WORLD_SIZE=1" in p.stderr
