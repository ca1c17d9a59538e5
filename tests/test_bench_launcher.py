"""CPU: bench.py's multi-rank launcher: `--gpus N`
without torchrun spawns N ranks itself and the emitted line reports them;
a --gpus / WORLD_SIZE mismatch fails loudly. The step is the --dry-run
stand-in (gloo, no GPU)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run"] + args,
                          capture_output=True, text=True, timeout=240, env=e)


@pytest.mark.timeout(300)
def test_bench_spawns_two_ranks():
    r = _run(["--gpus", "2", "--steps", "5", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(line) == 1
    d = json.loads(line[0])
    assert d["n_gpus"] == 2 and d["world_size"] == 2 and d["backend"] == "gloo" and d["dry_run"]
    # at N > 1 the run measures configs[1] (headline) and configs[3]'s 64/GPU bf16 share
    wl = {w["config"]: w for w in d["workloads"]}
    assert wl["configs[1]"]["global_batch"] == 16 and wl["configs[1]"]["dtype"] == "f32"
    assert wl["configs[3]"]["global_batch"] == 128 and wl["configs[3]"]["dtype"] == "bf16"


def test_bench_rejects_world_mismatch():
    r = _run(["--gpus", "1"], env={"WORLD_SIZE": "2"})
    assert r.returncode != 0 and "WORLD_SIZE=2" in (r.stderr + r.stdout)
