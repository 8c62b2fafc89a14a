"""Session / environment: ``MLEnvironment`` and ``MLEnvironmentFactory``.

Reference: ``A/common/MLEnvironment.java`` (holds Flink batch/stream environments; local env with
parallelism = #cores, ``:115-138``) and ``A/common/MLEnvironmentFactory.java`` (id -> env registry,
default id 0).  Here an environment describes the SPMD job this process belongs to:

* ``rank`` / ``world_size`` — one process per MI355X (or per CPU worker under gloo);
* ``local_tasks`` — logical BSP tasks per process (lets a single process reproduce Flink's
  P-subtask semantics, e.g. ``useLocalEnv(4)`` on one CPU process);
* ``device`` — where this rank's tensors live (``cuda:<LOCAL_RANK>`` on a GPU box);
* the per-environment ``LazyObjectsManager`` (lazy print / collect sinks).
"""
from __future__ import annotations

import os
import threading
from typing import Dict, Optional

import torch

from ..parallel import comm
from .lazy import LazyObjectsManager

__all__ = ["MLEnvironment", "MLEnvironmentFactory", "useLocalEnv", "useRemoteEnv", "resetEnv", "getMLEnv",
           "DEFAULT_ML_ENVIRONMENT_ID"]

DEFAULT_ML_ENVIRONMENT_ID = 0


class MLEnvironment:
    def __init__(self, parallelism: Optional[int] = None, device: Optional[str] = None,
                 compute_dtype: torch.dtype = torch.float64):
        comm.init_distributed()
        self.rank = comm.get_rank()
        self.world_size = comm.get_world_size()
        if device is None:
            env_dev = os.environ.get("ALINK_DEVICE")
            if env_dev:
                device = env_dev
            else:
                device = str(comm.device_for_rank()) if torch.cuda.is_available() else "cpu"
        self.device = torch.device(device)
        if parallelism is None or parallelism <= 0:
            parallelism = self.world_size
        self.local_tasks = max(1, parallelism // self.world_size)
        self.compute_dtype = compute_dtype
        self.lazy = LazyObjectsManager()
        self.tables: Dict[str, object] = {}  # registered table names (sqlQuery)

    @property
    def parallelism(self) -> int:
        return self.world_size * self.local_tasks

    def getParallelism(self):
        return self.parallelism

    def setParallelism(self, p: int):
        self.local_tasks = max(1, int(p) // self.world_size)

    def getLazyObjectsManager(self):
        return self.lazy

    @property
    def is_gpu(self) -> bool:
        return self.device.type == "cuda"

    def __repr__(self):
        return (f"MLEnvironment(rank={self.rank}, world_size={self.world_size}, local_tasks={self.local_tasks}, "
                f"device={self.device})")


class MLEnvironmentFactory:
    _lock = threading.Lock()
    _envs: Dict[int, MLEnvironment] = {}
    _next_id = 1

    @classmethod
    def get(cls, env_id: int = DEFAULT_ML_ENVIRONMENT_ID) -> MLEnvironment:
        with cls._lock:
            if env_id not in cls._envs:
                if env_id == DEFAULT_ML_ENVIRONMENT_ID:
                    cls._envs[env_id] = MLEnvironment()
                else:
                    raise KeyError(f"Cannot find MLEnvironment for MLEnvironmentId {env_id}. "
                                   "Did you get the MLEnvironmentId by calling getNewMLEnvironmentId?")
            return cls._envs[env_id]

    @classmethod
    def getDefault(cls) -> MLEnvironment:
        return cls.get(DEFAULT_ML_ENVIRONMENT_ID)

    @classmethod
    def getNewMLEnvironmentId(cls) -> int:
        return cls.registerMLEnvironment(MLEnvironment())

    @classmethod
    def registerMLEnvironment(cls, env: MLEnvironment) -> int:
        with cls._lock:
            i = cls._next_id
            cls._next_id += 1
            cls._envs[i] = env
            return i

    @classmethod
    def setDefault(cls, env: MLEnvironment):
        with cls._lock:
            cls._envs[DEFAULT_ML_ENVIRONMENT_ID] = env

    @classmethod
    def remove(cls, env_id: int):
        with cls._lock:
            if env_id == DEFAULT_ML_ENVIRONMENT_ID:
                cls._envs.pop(env_id, None)
                return None
            return cls._envs.pop(env_id, None)


def useLocalEnv(parallelism: int = 1, device: Optional[str] = None, spawn: bool = False,
                timeout_s: Optional[float] = None, **kwargs) -> MLEnvironment:
    """PyAlink entry point: create (and make default) an environment with the given parallelism.

    ``spawn=True`` outside an SPMD job makes the call self-launching (the reference's local env runs
    ``parallelism`` real subtasks): the current script is started again as ``parallelism`` ranks (one
    process per GPU, ``parallel/launch.py``), this process waits for them and exits with their status.
    Call it before anything touches the GPU."""
    if spawn and parallelism > 1:
        from ..parallel.launch import in_launched_job, launch_script
        import sys
        if not in_launched_job():
            sys.exit(launch_script(parallelism, [sys.executable] + sys.argv, timeout_s=timeout_s))
    env = MLEnvironment(parallelism=parallelism, device=device, **kwargs)
    MLEnvironmentFactory.setDefault(env)
    return env


def useRemoteEnv(host=None, port=None, parallelism: int = 1, **kwargs) -> MLEnvironment:
    """On this platform a "remote" job is an SPMD launch (torchrun); this attaches to it."""
    return useLocalEnv(parallelism=parallelism, **kwargs)


def resetEnv():
    MLEnvironmentFactory.remove(DEFAULT_ML_ENVIRONMENT_ID)


def getMLEnv() -> MLEnvironment:
    return MLEnvironmentFactory.getDefault()
