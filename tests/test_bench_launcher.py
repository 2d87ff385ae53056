"""bench.py --gpus N (the driver's SCALE runs): without a launcher around it the
bench starts N ranks itself (torch.distributed.run, one process per GPU); every rank sees
world_size == N and rank 0 prints the one JSON line.  CPU: the ranks run the launcher
self-test (a gloo group, no GPU work)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_launches_n_ranks(n):
    r = _run(["--gpus", str(n), "--launcher-selftest"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout            # rank 0 prints exactly one line
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["world_env"] == n
    assert sorted(tuple(x) for x in d["ranks"]) == [(i, str(i)) for i in range(n)]


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "2", "--launcher-selftest"], {"WORLD_SIZE": "1", "RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE=1 but --gpus 2" in r.stderr


def test_more_ranks_than_gpus_exits_nonzero():
    """The launching parent makes no HIP call; each rank compares its LOCAL_RANK with its own
    device count (stubbed to 1 here) and the one past it exits 2, which torch.distributed.run
    propagates as a failed job — never a silent run on fewer ranks."""
    r = _run(["--gpus", "2", "--launcher-selftest"], {"M3S_BENCH_DEVICES_STUB": "1"})
    assert r.returncode != 0
    assert "LOCAL_RANK=1 but only 1 GPU(s) visible" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_launcher_parent_makes_no_device_call():
    """`launch_ranks` (bench.py) must not touch torch.cuda / HIP before starting the ranks."""
    import ast
    src = open(os.path.join(ROOT, "bench.py")).read()
    fn = next(n for n in ast.walk(ast.parse(src))
              if isinstance(n, ast.FunctionDef) and n.name == "launch_ranks")
    body = ast.get_source_segment(src, fn)
    doc = ast.get_docstring(fn) or ""
    assert "torch.cuda" not in body.replace(doc, "")
