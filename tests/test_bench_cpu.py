"""CPU: bench.py's multi-process launcher and reporting path with the --stub workload (gloo).
`python bench.py --gpus 2` must start the ranks itself (torchrun child, 127.0.0.1) and report
n_gpus == 2 with the whole-job aggregate; a torchrun environment whose WORLD_SIZE disagrees
with --gpus is an error."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], capture_output=True, text=True,
                          timeout=240, env=e, cwd=REPO)


def test_bench_launcher_spawns_ranks():
    r = _run(["--stub", "--gpus", "2", "--steps", "2", "--warmup", "1", "--batch", "3", "--new-tokens", "5"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout          # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 6 and d["config"]["parallelism"] == "dp2"
    # 2 ranks x 3 utterances x 5 frames x 9 codebooks per step
    assert abs(d["value"] - 2 * 2 * 3 * 5 * 9 / (d["ms_per_step"] * d["steps"] / 1e3)) / d["value"] < 0.01


def test_bench_single_process_stub():
    r = _run(["--stub", "--steps", "1", "--warmup", "0", "--batch", "2", "--new-tokens", "4"])
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert d["n_gpus"] == 1


def test_bench_world_size_mismatch_is_an_error():
    r = _run(["--stub", "--gpus", "4", "--steps", "1"], env={"WORLD_SIZE": "2"})
    assert r.returncode != 0 and "WORLD_SIZE=2" in (r.stderr + r.stdout)
