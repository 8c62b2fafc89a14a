#!/usr/bin/env python3
"""Host <-> device transfer / synchronisation sites of the FTRL stream pipeline, per micro-batch: every
``item`` / ``tolist`` / ``int`` / ``float`` / ``bool`` / ``cpu`` of a device tensor (a device-to-host copy, i.e. a
stream synchronisation), every ``to`` / ``torch.tensor`` / ``torch.as_tensor`` that moves host data to the device
(host-to-device copy), counted by the framework source line that issued it, during ``StreamOperator.execute``
of ``tools/ftrl_pipeline_bench.py``.

    python tools/ftrl_sync_count.py [--rows 1048576] [--batch 65536] [--mode SHARDED]
"""
import argparse
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

COUNT = collections.Counter()
ACTIVE = [False]


def _site():
    for fr in reversed(traceback.extract_stack(limit=12)[:-2]):
        if "alink_amd" in fr.filename:
            return f"{fr.filename.split('alink_amd/')[-1]}:{fr.lineno}"
    return "other"


def _patch_d2h(name):
    orig = getattr(torch.Tensor, name)

    def f(self, *a, **k):
        if ACTIVE[0] and self.is_cuda:
            COUNT[("D2H " + name, _site())] += 1
        return orig(self, *a, **k)
    setattr(torch.Tensor, name, f)


def _patch_to():
    orig = torch.Tensor.to

    def f(self, *a, **k):
        if ACTIVE[0] and not self.is_cuda:
            dev = k.get("device", a[0] if a and isinstance(a[0], (str, torch.device)) else None)
            if dev is not None and torch.device(dev).type == "cuda":
                COUNT[("H2D to", _site())] += 1
        return orig(self, *a, **k)
    torch.Tensor.to = f


def _patch_ctor(name):
    orig = getattr(torch, name)

    def f(data, *a, **k):
        dev = k.get("device")
        if ACTIVE[0] and dev is not None and torch.device(dev).type == "cuda" and not (
                isinstance(data, torch.Tensor) and data.is_cuda):
            COUNT[("H2D " + name, _site())] += 1
        return orig(data, *a, **k)
    setattr(torch, name, f)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1 << 20)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--mode", default="SHARDED")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    for n in ("item", "tolist", "__int__", "__float__", "__bool__", "cpu", "numpy", "__index__"):
        _patch_d2h(n)
    _patch_to()
    for n in ("tensor", "as_tensor"):
        _patch_ctor(n)
    import ftrl_pipeline_bench as B
    from alink_amd.operator.stream.base import StreamOperator
    orig = StreamOperator.execute

    def run(*x, **k):
        ACTIVE[0] = True
        try:
            return orig(*x, **k)
        finally:
            ACTIVE[0] = False
    StreamOperator.execute = staticmethod(run)
    sys.argv = ["ftrl_pipeline_bench.py", "--rows", str(a.rows), "--batch", str(a.batch), "--mode", a.mode,
                "--init-rows", "20000"]
    B.main()
    nb = -(-a.rows // a.batch)
    total = sum(COUNT.values())
    print(f"== {total / nb:.1f} host<->device transfers per micro-batch ({nb} micro-batches)")
    for (kind, site), c in COUNT.most_common(a.top):
        print(f"{c / nb:8.2f}/batch  {kind:16s} {site}")


if __name__ == "__main__":
    main()
