"""Self-launching SPMD jobs: one process per MI355X (or per gloo CPU worker).

Reference: a local Flink environment runs ``parallelism`` real subtasks
(``A/common/MLEnvironment.java:115-138``).  The MI355X equivalent is P processes, each owning one GPU and
joined by ``torch.distributed`` (RCCL over xGMI for device tensors, gloo for host objects).  ``torchrun``
does this from the outside; this module does it from the inside so that ``python bench.py --gpus 8`` or
``useLocalEnv(8, spawn=True)`` starts the whole job by itself:

* :func:`launch_script` — run ``argv`` as P child processes with ``RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*``
  set, wait for all of them, kill the rest if one fails or the timeout passes, return the first non-zero
  exit code (0 when every rank succeeded);
* :func:`launch` — run a picklable function ``fn(*args)`` on P ranks (spawned interpreters) and return the
  per-rank results in rank order.

The parent never initialises the GPU: it only counts devices through the environment, never calls
``torch.cuda``, so the children are started from a process with no HIP context (a requirement of the
pool's process guard, and the same rule torchrun follows).  Children are started as ordinary child
processes (``subprocess`` / ``multiprocessing`` spawn); nothing is exec'd over a running interpreter.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
import traceback
from typing import Any, Callable, Dict, List, Optional, Sequence

__all__ = ["free_port", "rank_env", "launch_script", "launch", "in_launched_job"]


def free_port(host: str = "127.0.0.1") -> int:
    """A TCP port that was free a moment ago (bind to 0 and release)."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        s.bind((host, 0))
        return int(s.getsockname()[1])


def in_launched_job() -> bool:
    """True inside a rank of an SPMD job (torchrun or this launcher)."""
    return "WORLD_SIZE" in os.environ and "RANK" in os.environ


def rank_env(rank: int, world: int, port: int, base: Optional[Dict[str, str]] = None,
             addr: str = "127.0.0.1") -> Dict[str, str]:
    env = dict(os.environ if base is None else base)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": addr, "MASTER_PORT": str(port),
                "GROUP_RANK": "0", "ROLE_RANK": str(rank)})
    # dmabuf IPC is the only mode the host driver supports for RCCL / tensor sharing between processes
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def _terminate(procs: Sequence[subprocess.Popen], grace_s: float = 10.0):
    for p in procs:
        if p.poll() is None:
            try:
                p.send_signal(signal.SIGTERM)
            except OSError:
                pass
    deadline = time.time() + grace_s
    for p in procs:
        while p.poll() is None and time.time() < deadline:
            time.sleep(0.05)
        if p.poll() is None:
            try:
                p.kill()
            except OSError:
                pass
            p.wait()


def launch_script(nprocs: int, argv: Sequence[str], timeout_s: Optional[float] = None,
                  extra_env: Optional[Dict[str, str]] = None, port: Optional[int] = None,
                  quiet_ranks: bool = False) -> int:
    """Run ``argv`` as ``nprocs`` ranks of one job; return 0 iff every rank exited 0.

    Rank 0's stdout/stderr are the parent's (so its JSON line reaches the caller unchanged); other ranks
    share stderr and, with ``quiet_ranks``, have their stdout discarded."""
    nprocs = int(nprocs)
    if nprocs < 1:
        raise ValueError("nprocs must be >= 1")
    port = port or free_port()
    procs: List[subprocess.Popen] = []
    for r in range(nprocs):
        env = rank_env(r, nprocs, port)
        if extra_env:
            env.update(extra_env)
        out = subprocess.DEVNULL if (quiet_ranks and r > 0) else None
        procs.append(subprocess.Popen(list(argv), env=env, stdout=out))
    t0 = time.time()
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                print(f"[launch] a rank exited with {rc}; stopping the job", file=sys.stderr, flush=True)
                break
            if all(c == 0 for c in codes):
                return 0
            if timeout_s is not None and time.time() - t0 > timeout_s:
                print(f"[launch] job exceeded {timeout_s:.0f}s; stopping it", file=sys.stderr, flush=True)
                rc = 124
                break
            time.sleep(0.05)
    except KeyboardInterrupt:
        rc = 130
    _terminate(procs)
    return rc if rc != 0 else 1


def _child(fn: Callable, args: tuple, rank: int, world: int, port: int, q, env_extra: Dict[str, str]):
    os.environ.update(rank_env(rank, world, port, base={}))
    os.environ.update(env_extra)
    try:
        res = fn(*args)
        q.put((rank, True, res))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, False, f"{type(e).__name__}: {e}\n{traceback.format_exc()}"))
        raise SystemExit(1)
    finally:
        try:
            from . import comm
            comm.shutdown()
        except Exception:  # noqa: BLE001
            pass


def launch(nprocs: int, fn: Callable, *args, timeout_s: Optional[float] = 600.0,
           env: Optional[Dict[str, str]] = None) -> List[Any]:
    """Run ``fn(*args)`` on ``nprocs`` spawned ranks; returns the results in rank order.

    ``fn`` must be importable by name (module-level).  Inside ``fn``, ``useLocalEnv()`` attaches to the
    job (world size ``nprocs``).  Any rank failing raises ``RuntimeError`` with that rank's traceback."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_child, args=(fn, args, r, nprocs, port, q, dict(env or {})))
             for r in range(nprocs)]
    for p in procs:
        p.start()
    results: Dict[int, Any] = {}
    errors: Dict[int, str] = {}
    t0 = time.time()
    while len(results) + len(errors) < nprocs:
        try:
            rank, ok, val = q.get(timeout=0.2)
            (results if ok else errors)[rank] = val
            if not ok:
                break
        except Exception:  # queue.Empty
            pass
        dead = [p for p in procs if p.exitcode not in (None, 0)]
        if dead and q.empty():
            time.sleep(0.5)
            if q.empty():
                errors.setdefault(-1, f"rank process exited with code {dead[0].exitcode}")
                break
        if timeout_s is not None and time.time() - t0 > timeout_s:
            errors[-1] = f"timeout after {timeout_s}s"
            break
    for p in procs:
        p.join(timeout=5 if not errors else 0.5)
    for p in procs:
        if p.is_alive():
            p.terminate()
            p.join(5)
            if p.is_alive():
                p.kill()
                p.join()
    if errors:
        k = sorted(errors)[0]
        raise RuntimeError(f"rank {k} failed: {errors[k]}")
    return [results[r] for r in range(nprocs)]
