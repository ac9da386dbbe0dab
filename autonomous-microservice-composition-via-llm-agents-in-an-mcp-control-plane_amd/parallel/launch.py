"""Self-launch of one rank per GPU (one process per GPU, RCCL
over xGMI; the reference serves everything from one process,
control_plane.py:135-138,157).

``python bench.py --gpus 8`` must measure the whole node even when no
external launcher (torchrun) started it.  ``self_launch`` is called by an
entry point BEFORE anything touches the GPU: when the process is not a rank
already (no ``WORLD_SIZE`` in the environment) and more than one rank is
wanted, it starts ``n`` fresh child processes of the same script with the
torch.distributed env:// variables (``RANK``, ``LOCAL_RANK``,
``WORLD_SIZE``, ``LOCAL_WORLD_SIZE``, ``MASTER_ADDR=127.0.0.1``,
``MASTER_PORT``) set, waits for all of them and returns the exit code for
the parent to exit with.  The parent never initialises HIP (it only imports
modules and spawns children), so no process that touched the GPU ever
``exec``s another program.  A child that fails makes the parent stop the
others (only the PIDs it started) and return that child's code.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import time
from typing import List, Optional, Sequence

CHILD_ENV = "MCP_RANK_CHILD"


def is_rank_process() -> bool:
    """True inside torchrun / a self-launched child (env:// variables set)."""
    return "WORLD_SIZE" in os.environ


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(script: str, argv: Sequence[str], n: int, extra_env: Optional[dict] = None,
                poll_s: float = 0.2, timeout_s: Optional[float] = None) -> int:
    """Start ``n`` ranks of ``script argv`` and wait.  Returns 0 when every
    rank exits 0, else the first non-zero exit code seen (the other ranks are
    terminated, then killed if they do not exit)."""
    port = free_port()
    procs: List[subprocess.Popen] = []
    for r in range(n):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n),
                    "LOCAL_WORLD_SIZE": str(n), "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                    "MASTER_PORT": str(port), CHILD_ENV: "1"})
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if extra_env:
            env.update(extra_env)
        procs.append(subprocess.Popen([sys.executable, script, *argv], env=env))
    t0 = time.monotonic()
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            if all(c == 0 for c in codes):
                return 0
            if timeout_s is not None and time.monotonic() - t0 > timeout_s:
                rc = 124
                break
            time.sleep(poll_s)
    except KeyboardInterrupt:
        rc = 130
    for p in procs:
        if p.poll() is None:
            p.terminate()
    deadline = time.monotonic() + 20
    for p in procs:
        try:
            p.wait(timeout=max(0.1, deadline - time.monotonic()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    return rc


def self_launch(n: int, script: Optional[str] = None, argv: Optional[Sequence[str]] = None,
                extra_env: Optional[dict] = None) -> Optional[int]:
    """Entry-point helper.  Returns None when this process should run the
    work itself (already a rank, or ``n <= 1``); otherwise spawns ``n`` ranks
    and returns the exit code to exit with."""
    if n <= 1 or is_rank_process():
        return None
    script = os.path.abspath(script or sys.argv[0])
    argv = list(sys.argv[1:] if argv is None else argv)
    return spawn_ranks(script, argv, n, extra_env)


def check_devices(world_local: int, local_rank: int) -> None:
    """In a rank: fail fast (exit 3) when this node has fewer GPUs than
    ranks.  ``torch.cuda.device_count()`` does not initialise HIP."""
    import torch
    n = torch.cuda.device_count()
    if n < world_local or local_rank >= n:
        print(f"[rank {os.environ.get('RANK', '?')}] needs {world_local} GPUs on this node, "
              f"found {n}", file=sys.stderr, flush=True)
        sys.exit(3)
