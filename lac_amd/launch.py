"""One process per GPU for ``bench.py --gpus N`` (the metric is
reported at 1, 2, 4 and 8 GPUs; the reference itself is single-stream,
``/root/reference/arith_code.py:401-420``).

When ``--gpus N > 1`` is given and no launcher has set ``WORLD_SIZE``, the bench's
parent process starts ``python -m torch.distributed.run --nproc-per-node N`` as a
child -- before it makes any GPU call, so no GPU-initialised process ever execs
-- relays the ranks' stdout line by line (rank 0 prints the one JSON line),
passes stderr through, and exits with the launcher's status: a failing rank fails
the run.  The children see RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* from
torch.distributed.run exactly as under the driver's own multi-GPU command.

Ranks never share a GPU under nccl (RCCL refuses it); ``check_devices`` refuses
N above the visible device count unless the backend is gloo (one-GPU rehearsals).
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys


class LaunchError(RuntimeError):
    pass


def free_port(host: str = "127.0.0.1") -> int:
    s = socket.socket()
    s.bind((host, 0))
    p = s.getsockname()[1]
    s.close()
    return p


def check_devices(nproc: int, backend: str, ndev: int) -> None:
    """Refuse more nccl ranks than GPUs (never fall back to fewer ranks)."""
    if nproc < 1:
        raise LaunchError(f"--gpus {nproc}: need at least one rank")
    if backend == "nccl" and nproc > ndev:
        raise LaunchError(f"--gpus {nproc} with backend nccl needs {nproc} GPUs, {ndev} visible "
                          f"(ranks sharing a GPU only for rehearsals: LAC_DIST_BACKEND=gloo)")


def command(nproc: int, script: str, argv, port: int) -> list:
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), script, *argv]


def run_ranks(nproc: int, script: str, argv, env=None, out=None) -> tuple:
    """Run ``script argv`` on ``nproc`` ranks; returns (exit status, JSON objects seen
    on the ranks' stdout).  Every stdout line is relayed to ``out`` (default
    sys.stdout) as it arrives; stderr is inherited."""
    out = out if out is not None else sys.stdout
    e = dict(os.environ if env is None else env)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK"):
        e.pop(k, None)
    e.setdefault("MASTER_ADDR", "127.0.0.1")
    cmd = command(nproc, script, argv, free_port())
    p = subprocess.Popen(cmd, env=e, stdout=subprocess.PIPE, text=True, bufsize=1)
    lines = []
    for line in p.stdout:
        out.write(line)
        out.flush()
        s = line.strip()
        if s.startswith("{"):
            try:
                lines.append(json.loads(s))
            except ValueError:
                pass
    rc = p.wait()
    return rc, lines


def relay(nproc: int, script: str, argv) -> int:
    """bench.py's parent: run the ranks and check that exactly one JSON result line came
    back; returns the process exit status."""
    rc, lines = run_ranks(nproc, script, argv)
    results = [d for d in lines if "metric" in d]
    if rc != 0:
        print(f"[launch] torch.distributed.run exited {rc}: a rank failed", file=sys.stderr, flush=True)
        return rc
    if len(results) != 1:
        print(f"[launch] expected one JSON result line from rank 0, got {len(results)}", file=sys.stderr,
              flush=True)
        return 3
    if results[0].get("n_gpus") != nproc:
        print(f"[launch] result line reports n_gpus={results[0].get('n_gpus')}, launched {nproc}",
              file=sys.stderr, flush=True)
        return 3
    return 0
