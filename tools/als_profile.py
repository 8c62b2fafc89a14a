"""cProfile of one ALS training call on the GPU (host-side breakdown): python tools/als_profile.py [ratings]"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    from alink_amd import useLocalEnv
    from alink_amd.common.params import Params
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.models.recommendation.als import train_als
    env = useLocalEnv(1)
    dev = env.device
    g = torch.Generator(device=dev).manual_seed(0)
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    u = torch.randint(0, R // 10, (R,), generator=g, device=dev)
    it = ((R // 100) * torch.rand(R, generator=g, device=dev) ** 3).long()
    rt = torch.randint(1, 6, (R,), generator=g, device=dev).double()
    mt = MTable(TableSchema(["u", "i", "r"], [Types.LONG, Types.LONG, Types.DOUBLE]),
                [Column(u), Column(it), Column(rt)])
    p = Params().set("userCol", "u").set("itemCol", "i").set("rateCol", "r").set("rank", 64).set("numIter", 1) \
        .set("lambda", 0.1)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t = time.perf_counter()
    pr.enable()
    train_als(mt, p, env)
    torch.cuda.synchronize()
    pr.disable()
    print("total", time.perf_counter() - t, flush=True)
    pstats.Stats(pr).sort_stats("cumtime").print_stats(25)


if __name__ == "__main__":
    main()
