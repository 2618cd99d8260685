"""grace_amd.launcher / bench.py self-launch: N ranks from one command, the
torchrun env contract, rank 0's JSON relayed once, and a failing or hung rank ending the whole
launch non-zero with no process left behind.  CPU only (gloo where a rendezvous is needed)."""
import json
import os
import subprocess
import sys
import textwrap
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _alive(pid: int) -> bool:
    try:
        with open(f"/proc/{pid}/status") as f:
            for line in f:
                if line.startswith("State:"):
                    return "Z" not in line.split()[1]
    except FileNotFoundError:
        return False
    return False


def _script(tmp_path, body: str) -> str:
    p = tmp_path / "rank_script.py"
    p.write_text(textwrap.dedent(body))
    return str(p)


def _launch(script, n, timeout=60.0, grace=3.0, extra=()):
    cmd = [sys.executable, "-m", "grace_amd.launcher", "-np", str(n), "--timeout", str(timeout),
           "--grace", str(grace), script, *extra]
    return subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout + 60)


def test_env_contract_and_single_json_line(tmp_path):
    s = _script(tmp_path, """
        import json, os
        keys = ["RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"]
        env = {k: os.environ[k] for k in keys}
        print("progress line from rank", env["RANK"], flush=True)
        print(json.dumps({"metric": "m", "value": 1.0, "env": env}), flush=True)
    """)
    r = _launch(s, 3)
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout  # only rank 0's JSON, once; progress lines go to stderr
    out = json.loads(lines[0])
    assert out["env"]["RANK"] == "0" and out["env"]["WORLD_SIZE"] == "3" and out["env"]["MASTER_ADDR"] == "127.0.0.1"
    assert out["launcher"]["nproc"] == 3 and out["launcher"]["exit_codes"] == [0, 0, 0]
    assert "progress line from rank 0" in r.stderr and "progress line from rank 2" in r.stderr


def test_failing_rank_ends_the_launch_without_orphans(tmp_path):
    pids = tmp_path / "pids"
    s = _script(tmp_path, f"""
        import os, subprocess, sys, time
        r = int(os.environ["RANK"])
        kid = subprocess.Popen(["sleep", "300"])  # a grandchild in the rank's process group
        with open({str(pids)!r} + f".{{r}}", "w") as f:
            f.write(f"{{os.getpid()}} {{kid.pid}}")
        if r == 1:
            sys.exit(1)
        time.sleep(300)  # the survivors would hang forever without the launcher
    """)
    t0 = time.monotonic()
    r = _launch(s, 3, timeout=120, grace=2)
    took = time.monotonic() - t0
    assert r.returncode == 1, (r.returncode, r.stderr)
    assert took < 60, took
    assert r.stdout.strip() == ""
    assert "rank 1 exited with 1" in r.stderr
    for q in range(3):
        for pid in map(int, open(f"{pids}.{q}").read().split()):
            assert not _alive(pid), f"rank {q} left process {pid} running"


def test_timeout_kills_every_rank(tmp_path):
    s = _script(tmp_path, """
        import json, time
        print(json.dumps({"metric": "m", "value": 1.0}), flush=True)
        time.sleep(300)
    """)
    r = _launch(s, 2, timeout=3, grace=1)
    assert r.returncode == 124, r.stderr
    assert r.stdout.strip() == ""  # a failed launch withholds rank 0's number
    assert "timeout" in r.stderr


def test_gloo_rendezvous_through_the_launcher(tmp_path):
    s = _script(tmp_path, """
        import json, os, sys
        sys.path.insert(0, os.environ["GRACE_ROOT"])
        import torch, torch.distributed as dist
        dist.init_process_group("gloo")
        t = torch.tensor([dist.get_rank() + 1.0])
        dist.all_reduce(t)
        if dist.get_rank() == 0:
            print(json.dumps({"metric": "m", "value": float(t), "world_seen": dist.get_world_size()}), flush=True)
        dist.destroy_process_group()
    """)
    os.environ["GRACE_ROOT"] = ROOT
    r = _launch(s, 2, timeout=120)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip())
    assert out["world_seen"] == 2 and out["value"] == 3.0


@pytest.mark.skipif(__import__("torch").cuda.is_available(), reason="CPU-host check (a GPU box would run it)")
def test_bench_self_launch_fails_loudly_without_gpus():
    """``bench.py --gpus 2`` outside torchrun launches 2 ranks (no torch import in the parent); on
    a host without GPUs every rank refuses, so the launch exits non-zero with no JSON line."""
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--launch-timeout", "120"], cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert r.stdout.strip() == ""
    assert "[launcher]" in r.stderr and ("needs a GPU" in r.stderr or "visible GPU" in r.stderr)
