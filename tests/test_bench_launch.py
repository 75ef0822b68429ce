"""bench.py --gpus N without a launcher starts its own N ranks (CPU tests).

The driver may run `python3 bench.py --gpus 8` on an 8-GPU node with no
torch.distributed.run around it: bench.py then spawns N fresh child
processes of itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, as
torch.distributed.run sets them) before anything touches the GPU, relays rank
0's JSON line and exits non-zero when a rank fails or the job times out.
"""
import json
import os
import subprocess
import sys
import textwrap
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402  (imports no torch at module level)


def test_spawn_plan_env():
    plan = bench.spawn_plan(["--gpus", "4", "--steps", "20"], 4, 29555, base_env={"PATH": "/bin", "X": "1"})
    assert len(plan) == 4
    for r, (cmd, env) in enumerate(plan):
        assert cmd[0] == sys.executable and cmd[-4:] == ["--gpus", "4", "--steps", "20"]
        assert os.path.basename(cmd[2]) == "bench.py"
        assert env["RANK"] == env["LOCAL_RANK"] == str(r)
        assert env["WORLD_SIZE"] == env["LOCAL_WORLD_SIZE"] == "4"
        assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "29555"
        assert env["X"] == "1" and env["PATH"] == "/bin"     # the caller's environment is kept


def _child(tmp_path, body):
    p = tmp_path / "child.py"
    p.write_text(textwrap.dedent(body))
    return str(p)


def _plan(script, n):
    return bench.spawn_plan([], n, bench.free_port(), script=script)


class _Out:
    def __init__(self):
        self.text = ""

    def write(self, s):
        self.text += s

    def flush(self):
        pass


def test_launch_relays_rank0_only(tmp_path):
    script = _child(tmp_path, """
        import json, os
        print("[Gloo] Rank 0 is connected to 2 peer ranks", flush=True)    # not JSON: goes to stderr
        print(json.dumps({k: os.environ[k] for k in ("RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}),
              flush=True)
    """)
    out = _Out()
    assert bench.launch_ranks(_plan(script, 3), timeout_s=60, out=out) == 0
    lines = [json.loads(x) for x in out.text.splitlines()]
    assert len(lines) == 1 and lines[0]["RANK"] == "0" and lines[0]["WORLD_SIZE"] == "3"


def test_launch_failure_ends_the_others(tmp_path):
    script = _child(tmp_path, """
        import os, sys, time
        if os.environ["RANK"] == "1":
            sys.exit(3)
        time.sleep(120)
    """)
    t0 = time.monotonic()
    assert bench.launch_ranks(_plan(script, 3), timeout_s=100, out=_Out()) == 3
    assert time.monotonic() - t0 < 30


def test_launch_timeout(tmp_path):
    script = _child(tmp_path, """
        import time
        time.sleep(120)
    """)
    t0 = time.monotonic()
    assert bench.launch_ranks(_plan(script, 2), timeout_s=2, out=_Out()) == 124
    assert time.monotonic() - t0 < 30


def test_bench_self_launches_before_torch(tmp_path):
    """bench.main() with --gpus 2 and no WORLD_SIZE hands off to launch_ranks
    without importing torch (the parent must never touch the GPU)."""
    code = textwrap.dedent(f"""
        import json, sys
        sys.path.insert(0, {ROOT!r})
        import bench
        seen = {{}}
        def fake(plan, timeout_s):
            seen["n"] = len(plan)
            seen["ranks"] = [e["RANK"] for _, e in plan]
            seen["argv"] = plan[0][0][3:]
            seen["torch"] = "torch" in sys.modules
            return 7
        bench.launch_ranks = fake
        sys.argv = ["bench.py", "--gpus", "2", "--steps", "20", "--warmup", "5"]
        try:
            bench.main()
        except SystemExit as e:
            seen["exit"] = e.code
        print(json.dumps(seen))
    """)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stderr
    seen = json.loads(r.stdout.strip().splitlines()[-1])
    assert seen == {"n": 2, "ranks": ["0", "1"], "argv": ["--gpus", "2", "--steps", "20", "--warmup", "5"],
                    "torch": False, "exit": 7}


@pytest.mark.timeout(300)
def test_bench_ranks_fail_loudly_without_gpus():
    """On a machine without GPUs the spawned ranks fail and so does the job
    (no silent one-GPU measurement)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
                        "--launch-timeout", "240"], capture_output=True, text=True, env=env, timeout=280, cwd=ROOT)
    assert r.returncode != 0
    assert r.stdout.strip() == ""
    assert "launcher: starting 2 ranks" in r.stderr
