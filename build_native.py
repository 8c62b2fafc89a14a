#!/usr/bin/env python3
"""Build the native parts of alink_amd in-tree.

* ``alink_amd/ops/libalink_hip.so``   — HIP/CDNA4 kernels, ``hipcc --offload-arch=gfx950`` (C ABI, ctypes)
* ``alink_amd/_native/libalink_native.so`` — host C++ runtime (CSV/libsvm/vector parsing, murmur3
  feature hashing, sample-sort helpers), ``g++ -O3`` (C ABI, ctypes)

Incremental: a target is rebuilt only when a source is newer than it.  Usage:
    python build_native.py [--force] [--only hip|host]
"""
from __future__ import annotations

import argparse
import glob
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
HIP_SRC = sorted(glob.glob(os.path.join(ROOT, "alink_amd", "ops", "csrc", "*.hip")))
HIP_OUT = os.path.join(ROOT, "alink_amd", "ops", "libalink_hip.so")
HOST_SRC = sorted(glob.glob(os.path.join(ROOT, "alink_amd", "_native", "csrc", "*.cpp")))
HOST_OUT = os.path.join(ROOT, "alink_amd", "_native", "libalink_native.so")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")


def _stale(out, srcs, extra=()):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in list(srcs) + list(extra))


def _run(cmd):
    print("+", " ".join(cmd), flush=True)
    subprocess.check_call(cmd)


def build_hip(force=False):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    headers = glob.glob(os.path.join(ROOT, "alink_amd", "ops", "csrc", "*.h"))
    if not force and not _stale(HIP_OUT, HIP_SRC, headers):
        return HIP_OUT
    objs = []
    tmp = os.path.join(ROOT, "build", "hip")
    os.makedirs(tmp, exist_ok=True)
    for s in HIP_SRC:
        o = os.path.join(tmp, os.path.basename(s) + ".o")
        if force or _stale(o, [s], headers):
            _run([hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-mcode-object-version=5",
                  "-Wno-unused-command-line-argument", "-c", s, "-o", o])
        objs.append(o)
    _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", HIP_OUT] + objs)
    return HIP_OUT


def build_host(force=False):
    if not HOST_SRC:
        return None
    headers = glob.glob(os.path.join(ROOT, "alink_amd", "_native", "csrc", "*.h"))
    if not force and not _stale(HOST_OUT, HOST_SRC, headers):
        return HOST_OUT
    cxx = shutil.which("g++") or "c++"
    _run([cxx, "-O3", "-std=c++17", "-fPIC", "-shared", "-march=x86-64-v2", "-fopenmp", "-o", HOST_OUT]
         + HOST_SRC)
    return HOST_OUT


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--only", choices=["hip", "host"], default=None)
    a = ap.parse_args(argv)
    if a.only in (None, "host"):
        build_host(a.force)
    if a.only in (None, "hip"):
        build_hip(a.force)


if __name__ == "__main__":
    main(sys.argv[1:])
