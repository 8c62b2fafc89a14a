#!/usr/bin/env python3
"""AddressSanitizer + UBSan run of the host C++ runtime (SURVEY §5.2 race / memory-safety tooling).

Builds ``alink_amd/_native/csrc/*.cpp`` with ``-fsanitize=address,undefined`` into ``build/asan/`` and runs the
REAL Python wrappers (``alink_amd._native``: CSV parser incl. quoted / malformed / ragged lines, Guava murmur3 on
empty and non-BMP strings, dense vector parsing, the three FTRL CSR kernels incl. out-of-range indices) in a
child process with the sanitizer runtimes preloaded, so any heap overflow or UB in the C++ or in the buffer
sizing of the ctypes callers aborts the child.  Host code only: GPU sanitizer runs are not available on this
pool.  Usage: ``python tools/asan_host.py`` (exit 0 = clean).
"""
import glob
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "build", "asan", "libalink_native_asan.so")


def build() -> str:
    srcs = sorted(glob.glob(os.path.join(ROOT, "alink_amd", "_native", "csrc", "*.cpp")))
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    cxx = shutil.which("g++") or "c++"
    cmd = [cxx, "-O1", "-g", "-std=c++17", "-fPIC", "-shared", "-fopenmp", "-fno-omit-frame-pointer",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-o", OUT] + srcs
    subprocess.check_call(cmd)
    return OUT


def runtime_libs():
    libs = []
    for name in ("libasan.so", "libubsan.so"):
        p = subprocess.check_output(["g++", "-print-file-name=" + name]).decode().strip()
        if not os.path.isabs(p) or not os.path.exists(p):
            return None
        libs.append(os.path.realpath(p))
    return libs


EXERCISE = r'''
import numpy as np
import alink_amd._native as N
assert N.lib is not None, "asan build not loaded"
# CSV: quoted fields with escaped quotes, empty fields, ragged / long lines, unicode
lines = ['1,"a ""q"" b",2.5,true', '2,,,', '3,"unterminated,4.0,false', '', '4,x,1e308,TRUE',
         '5,' + 'y' * 5000 + ',-0.0,false', '6,"",nan,false', '7,é€😀,3,false']
for skip in (True, False):
    try:
        N.parse_csv_lines(lines, [2, 0, 1, 3], ",", '"', skip)
    except RuntimeError:
        pass
try:
    N.parse_csv_lines(['1,2', 'bad,3'], [2, 2], ",", "", True)
except RuntimeError:
    pass
N.parse_csv_lines([], [2, 0], ",", '"', True)
# murmur3: empty, odd length, surrogate pairs, long
h = N.murmur3_utf16(["", "a", "ab", "abc", "😀x", "z" * 10001])
assert h.shape == (6,)
N.murmur3_utf16([])
# dense vectors: short / long / malformed rows
N.parse_dense_vectors(["1 2 3", "4,5,6", "7 8", "1 2 3 4 5"], 3)
N.parse_dense_vectors(["", "x y z"], 3)
N.parse_dense_vectors([], 4)
# FTRL CSR kernels
rng = np.random.default_rng(0)
nrows, dim = 64, 50
nnz = rng.integers(0, 6, nrows)
indptr = np.concatenate([[0], np.cumsum(nnz)]).astype(np.int64)
idx = rng.integers(0, dim, indptr[-1]).astype(np.int32)
val = rng.normal(size=indptr[-1])
y = rng.integers(0, 2, nrows).astype(np.float64)
w, n, z = np.zeros(dim), np.zeros(dim), np.zeros(dim)
N.ftrl_update_csr(indptr, idx, val, y, w, n, z, 0.1, 1.0, 0.01, 0.01)
bad = idx.copy()
if len(bad):
    bad[0] = dim + 7
    try:
        N.ftrl_update_csr(indptr, bad, val, y, w, n, z, 0.1, 1.0, 0.01, 0.01)
        raise SystemExit("out-of-range index accepted")
    except ValueError:
        pass
m = N.ftrl_partial_margin(indptr, idx, val, w[10:30].copy(), 10, 30)
assert m.shape == (nrows,)
ws, ns, zs = w[10:30].copy(), n[10:30].copy(), z[10:30].copy()
N.ftrl_shard_update(indptr, idx, val, rng.normal(size=nrows), ws, ns, zs, 10, 30, 0.1, 1.0, 0.01, 0.01)
# round-6 entry points: CSV over spans, JSON top-level members, packed column join, Java float rows
data = np.frombuffer(b'1,"a""b",2\n\n3,,x\n4,"unterminated', dtype=np.uint8)
st = np.array([0, 11, 12, 18], dtype=np.int64)
en = np.array([10, 11, 17, 31], dtype=np.int64)
for blocks in (False, True):
    try:
        N.parse_csv_spans(data, st, en, [2, 0, 0], ",", '"', blocks=blocks)
    except RuntimeError:
        pass
docs = [b'{"a": 1, "b": "x"}', b'{"a": [1, {"q": "]"}], "b": "\\"}', b'{"a":', b'{"a": "unterminated',
        b'', b'{"a": -0, "b": 1e400}', b'{"a"', b'{' * 3000]
jd = np.frombuffer(b"".join(docs), dtype=np.uint8)
jo = np.zeros(len(docs) + 1, dtype=np.int64)
jo[1:] = np.cumsum([len(d) for d in docs])
N.json_top_values(jd, jo, ["a", "b", ""])
N.json_top_values(jd, jo, [])
c1 = (np.frombuffer(b"abcde", dtype=np.uint8), np.array([0, 2, 2, 5], dtype=np.int64))
c2 = (np.zeros(0, dtype=np.uint8), np.zeros(4, dtype=np.int64))
assert bytes(N.join_packed_columns([c1, c2], ",", "\r\n")) == b"ab,\r\n,\r\ncde,\r\n"
N.java_float_rows(np.array([[1.5, -0.0, 3e38], [1e-45, np.nan, np.inf]], dtype=np.float32), " ")
print("ASAN_EXERCISE_OK")
'''


# canary: a deliberately undersized output buffer MUST be reported (proves the sanitizer is live in the child)
CANARY = r'''
import ctypes, numpy as np
import alink_amd._native as N
buf = b"1 2 3,4 5 6"
off = np.array([0, 5, 11], dtype=np.int64)
out = np.zeros(2, dtype=np.float64)          # needs 2 x 3
N.lib.alink_parse_dense_vectors(ctypes.c_char_p(buf), N._ptr(off), ctypes.c_int64(2), ctypes.c_int64(3), N._ptr(out))
print("CANARY_NOT_CAUGHT")
'''


def run() -> int:
    libs = runtime_libs()
    if libs is None:
        print("sanitizer runtimes not found; skipped")
        return 77
    so = build()
    env = dict(os.environ)
    env["LD_PRELOAD"] = ":".join(libs)
    env["ALINK_NATIVE_LIB"] = so
    env["ASAN_OPTIONS"] = "detect_leaks=0:halt_on_error=1:abort_on_error=0:exitcode=23"
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1:exitcode=24"
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env["OMP_NUM_THREADS"] = "4"
    p = subprocess.run([sys.executable, "-c", EXERCISE], env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=600)
    sys.stdout.write(p.stdout[-4000:])
    sys.stderr.write(p.stderr[-8000:])
    if not (p.returncode == 0 and "ASAN_EXERCISE_OK" in p.stdout):
        return p.returncode or 1
    c = subprocess.run([sys.executable, "-c", CANARY], env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=300)
    if c.returncode != 23 or "heap-buffer-overflow" not in c.stderr:
        print("sanitizer canary NOT caught:", c.returncode, c.stdout[-500:], c.stderr[-1500:])
        return 25
    print("ASAN_CANARY_CAUGHT")
    return 0


if __name__ == "__main__":
    sys.exit(run())
