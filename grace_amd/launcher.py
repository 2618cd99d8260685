"""``grace_amd.launcher``: start N ranks of a script on one node, one process per GPU.

The reference is driven by a launcher that spawns the ranks (``horovodrun -np 2 ...`` /
``mpirun -np 2 ...``, /root/reference/TRAINING.md:69-85) and its harness reports "Total img/sec
on N GPU(s)" from rank 0 (/root/reference/examples/torch/pytorch_synthetic_benchmark.py:194-198).
This module is that launcher for the torch.distributed env:// rendezvous (RCCL over xGMI):

    python -m grace_amd.launcher -np 8 bench.py --gpus 8 --steps 20
    # or from a script that was started without torchrun (bench.py --gpus 8 does this):
    from grace_amd.launcher import launch
    sys.exit(launch([sys.executable, __file__, *sys.argv[1:]], nproc=8))

Rules (the MI355X pool's, and what a launcher must guarantee):

* STDLIB ONLY: the parent never imports torch, so it never initialises the GPU; every rank is a
  fresh child process started with ``subprocess`` (fork + exec in the CHILD, before any HIP call
  anywhere), never ``os.exec*`` of the parent.
* Each child gets ``RANK`` / ``LOCAL_RANK`` / ``WORLD_SIZE`` / ``LOCAL_WORLD_SIZE`` /
  ``MASTER_ADDR`` (127.0.0.1) / a free ``MASTER_PORT`` -- the same contract as
  ``torch.distributed.run``, so a script works under either.
* Each child runs in its own session (process group).  When one rank exits non-zero, the
  launcher waits ``grace_s`` for the others (their collectives should fail on their own), then
  SIGTERMs and finally SIGKILLs every surviving rank's whole process group; a launch that
  exceeds ``timeout_s`` is killed the same way (exit 124).  SIGTERM / SIGINT to the launcher
  are forwarded the same way.  No orphans: the launcher returns only after every child is reaped.
* Rank 0's stdout is relayed: a JSON object line (the benchmark contract) is held back and
  printed ONCE at the end, with a ``launcher`` record added (ranks, exit codes, wall time);
  every other line of any rank goes to stderr, so the launcher's stdout carries only that line.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import threading
import time
from typing import Dict, List, Optional


def free_port(addr: str = "127.0.0.1") -> int:
    """A TCP port that was free a moment ago on ``addr`` (the OS picks it)."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((addr, 0))
        return int(s.getsockname()[1])


def rank_env(rank: int, nproc: int, addr: str, port: int, base: Optional[Dict[str, str]] = None) -> Dict[str, str]:
    env = dict(os.environ if base is None else base)
    env.update({
        "RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(nproc),
        "LOCAL_WORLD_SIZE": str(nproc), "GROUP_RANK": "0", "NODE_RANK": "0",
        "MASTER_ADDR": addr, "MASTER_PORT": str(port), "GRACE_LAUNCHER": "1",
        "PYTHONUNBUFFERED": "1",
    })
    return env


def _killpg(p: subprocess.Popen, sig: int) -> None:
    try:
        os.killpg(p.pid, sig)  # the child leads its own session: pgid == pid
    except (ProcessLookupError, PermissionError):
        pass


class _Relay(threading.Thread):
    """Forward rank 0's stdout: the LAST JSON object line is kept for the final print, the rest
    goes to stderr as it arrives (progress stays visible)."""

    def __init__(self, stream):
        super().__init__(daemon=True, name="grace-launcher-relay")
        self.stream = stream
        self.result: Optional[dict] = None

    def run(self):
        for raw in iter(self.stream.readline, b""):
            line = raw.decode("utf-8", "replace").rstrip("\n")
            obj = None
            if line.startswith("{"):
                try:
                    obj = json.loads(line)
                except ValueError:
                    obj = None
            if isinstance(obj, dict):
                self.result = obj
            else:
                sys.stderr.write(line + "\n")
                sys.stderr.flush()


def launch(cmd: List[str], nproc: int, timeout_s: float = 3000.0, grace_s: float = 20.0,
           master_addr: str = "127.0.0.1", master_port: Optional[int] = None, relay_json: bool = True,
           poll_s: float = 0.2) -> int:
    """Run ``cmd`` as ``nproc`` ranks; returns the exit code the launcher should exit with:
    0 when every rank exited 0, else the first failing rank's code (124 on timeout, 1 when a
    rank died from a signal)."""
    if nproc < 1:
        raise ValueError("nproc must be >= 1")
    port = master_port or free_port(master_addr)
    procs: List[subprocess.Popen] = []
    relay = None
    t0 = time.monotonic()
    state = {"signal": None}

    def on_signal(signum, _frame):
        state["signal"] = signum

    old = {s: signal.signal(s, on_signal) for s in (signal.SIGTERM, signal.SIGINT)}
    try:
        for r in range(nproc):
            out = subprocess.PIPE if (r == 0 and relay_json) else sys.stderr.fileno()
            procs.append(subprocess.Popen(cmd, env=rank_env(r, nproc, master_addr, port), stdout=out,
                                          start_new_session=True))
        if relay_json:
            relay = _Relay(procs[0].stdout)
            relay.start()
        codes: List[Optional[int]] = [None] * nproc
        failed_at = None
        why = None
        while True:
            for r, p in enumerate(procs):
                if codes[r] is None:
                    codes[r] = p.poll()
            if all(c is not None for c in codes):
                break
            now = time.monotonic()
            bad = [r for r, c in enumerate(codes) if c not in (None, 0)]
            if bad and failed_at is None:
                failed_at = now
                why = f"rank {bad[0]} exited with {codes[bad[0]]}"
            if state["signal"] is not None and why is None:
                why = f"launcher received signal {state['signal']}"
                failed_at = now - grace_s  # no grace: stop now
            if why is None and now - t0 > timeout_s:
                why = f"timeout after {timeout_s:.0f}s"
                failed_at = now - grace_s
            if failed_at is not None and now - failed_at >= grace_s:
                sys.stderr.write(f"[launcher] {why}: terminating the remaining ranks\n")
                _stop_all(procs)
                for r, p in enumerate(procs):
                    codes[r] = p.wait()
                break
            time.sleep(poll_s)
        if relay is not None:
            relay.join(timeout=10)
        wall = time.monotonic() - t0
        if why is not None and why.startswith("timeout"):
            rc = 124
        else:
            bad = [c for c in codes if c != 0]
            rc = 0 if not bad else (bad[0] if bad[0] > 0 else 1)
        if state["signal"] is not None and rc == 0:
            rc = 128 + int(state["signal"])
        if relay is not None and relay.result is not None:
            res = dict(relay.result)
            res["launcher"] = {"kind": "grace_amd.launcher (subprocess per rank, env:// rendezvous)",
                               "nproc": nproc, "master": f"{master_addr}:{port}", "exit_codes": codes,
                               "wall_s": round(wall, 2)}
            if rc == 0:
                print(json.dumps(res), flush=True)
            else:  # a failed launch must not hand a sweep a throughput number
                sys.stderr.write("[launcher] rank 0 result withheld (launch failed): " + json.dumps(res) + "\n")
        if rc != 0:
            sys.stderr.write(f"[launcher] failed: {why or 'a rank exited non-zero'}; exit codes {codes}\n")
        return rc
    finally:
        _stop_all(procs)
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                _killpg(p, signal.SIGKILL)
                p.wait()
        for s, h in old.items():
            signal.signal(s, h)


def _stop_all(procs: List[subprocess.Popen], term_wait_s: float = 10.0) -> None:
    live = [p for p in procs if p.poll() is None]
    for p in live:
        _killpg(p, signal.SIGTERM)
    deadline = time.monotonic() + term_wait_s
    for p in live:
        try:
            p.wait(timeout=max(0.0, deadline - time.monotonic()))
        except subprocess.TimeoutExpired:
            pass
    for p in live:
        if p.poll() is None:
            _killpg(p, signal.SIGKILL)
    # a rank's own children (e.g. data-loader workers) share its process group and can outlive it
    for p in procs:
        if _pg_alive(p.pid):
            _killpg(p, signal.SIGKILL)


def _pg_alive(pgid: int) -> bool:
    try:
        os.killpg(pgid, 0)
        return True
    except (ProcessLookupError, PermissionError):
        return False


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m grace_amd.launcher", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("-np", "--nproc", type=int, required=True, help="ranks (one per GPU)")
    ap.add_argument("--timeout", type=float, default=3000.0, help="kill every rank after this many seconds")
    ap.add_argument("--grace", type=float, default=20.0,
                    help="seconds the other ranks get to exit after one failed, before they are killed")
    ap.add_argument("--master-addr", default="127.0.0.1")
    ap.add_argument("--master-port", type=int, default=0, help="0 = a free port")
    ap.add_argument("--no-relay", action="store_true", help="rank 0 prints directly (no JSON relay)")
    ap.add_argument("script")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    cmd = [sys.executable, "-u", a.script, *a.args]
    return launch(cmd, a.nproc, timeout_s=a.timeout, grace_s=a.grace, master_addr=a.master_addr,
                  master_port=a.master_port or None, relay_json=not a.no_relay)


if __name__ == "__main__":
    sys.exit(main())
