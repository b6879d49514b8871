"""bench.py's multi-rank launcher on the CPU (gloo): `bench.py --gpus N` run without a torchrun environment must start
N ranks itself (the driver's `--gpus 8` leg would otherwise record a silent 1-rank number), and a --gpus / WORLD_SIZE
mismatch must fail.  --check-launch builds the process group and runs one all-reduce, no GPU work."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, **env_over):
    env = dict(os.environ, CFM_DIST_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_over)
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=180)


def _json_lines(out):
    return [json.loads(s) for s in out.splitlines() if s.strip().startswith("{")]


def test_bench_gpus_2_spawns_two_ranks():
    r = _run(["--gpus", "2", "--check-launch"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout           # one line: rank 0's
    res = lines[0]
    assert res["n_gpus"] == 2 and res["world_size_reported"] == 2 and res["ranks_in_allreduce"] == 2
    assert res["dist_backend"] == "gloo"


def test_bench_gpus_1_stays_single_process():
    r = _run(["--check-launch"])
    assert r.returncode == 0, r.stderr[-2000:]
    res = _json_lines(r.stdout)[0]
    assert res["n_gpus"] == 1 and res["dist_backend"] is None
    assert "launching" not in r.stderr


def test_bench_gpus_mismatch_exits_nonzero():
    r = _run(["--gpus", "2", "--check-launch"], WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2
    assert "WORLD_SIZE=1" in r.stderr
    assert not _json_lines(r.stdout)
