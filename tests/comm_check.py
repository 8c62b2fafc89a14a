"""Every ``parallel/comm.py`` wrapper, checked against the values each rank can compute locally.

Run as ``python tests/comm_check.py RANK WORLD PORT OUTDIR [TAG]`` (one process per rank).  With WORLD=1 the
script sets ``ALINK_COMM_FORCE_COLLECTIVE=1`` so the 1-rank group takes every wrapper's real collective branch:
on a GPU box that is the RCCL (``nccl``) branch — the code an 8-GPU job runs, which RCCL will not let two ranks
of one device execute ("Duplicate GPU detected") — and on the host the gloo branch.  Rank r's inputs are
deterministic functions of r, so the expected result of every collective is known on every rank for any world
size.  Writes ``OUTDIR/comm_<TAG>_<WORLD>_<RANK>.json`` with one entry per check.
"""
import json
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _x(r, n, dtype, salt=0):
    import torch
    g = torch.Generator().manual_seed(1009 * salt + 17 * r + 3)
    return (torch.randn(n, generator=g, dtype=torch.float64) * (r + 1)).to(dtype)


def _fold(parts, op):
    import torch
    acc = parts[0].clone()
    for p in parts[1:]:
        acc = acc + p if op == "sum" else (torch.maximum(acc, p) if op == "max" else torch.minimum(acc, p))
    return acc


def checks(out):
    import numpy as np
    import torch
    from alink_amd.common.strings import StringBlock
    from alink_amd.parallel import comm
    comm.init_distributed()
    ws, me = comm.get_world_size(), comm.get_rank()
    gpu = torch.cuda.is_available() and os.environ.get("ALINK_DEVICE", "") != "cpu"
    dev = comm.device_for_rank() if gpu else torch.device("cpu")
    res = {}
    out["backend"] = comm._backend()
    out["is_distributed"] = comm.is_distributed()
    out["world"] = ws

    def ok(name, cond):
        res[name] = bool(cond)

    def close(a, b, tol=1e-9):
        a, b = a.detach().cpu().double(), b.detach().cpu().double()
        return a.shape == b.shape and bool(torch.allclose(a, b, rtol=tol, atol=tol))

    # ---- all_reduce: device (small -> one-shot on RCCL jobs, large -> RCCL) and host tensors ----
    for dtype in (torch.float32, torch.float64):
        tol = 1e-5 if dtype == torch.float32 else 1e-12
        for op in ("sum", "max", "min"):
            for n, where in ((1000, "dev_small"), (300_000, "dev_large"), (777, "host")):
                x = _x(me, n, dtype, salt=n)
                t = x.clone() if where == "host" else x.to(dev)
                comm.all_reduce(t, op)
                ref = _fold([_x(r, n, dtype, salt=n) for r in range(ws)], op)
                ok(f"all_reduce.{where}.{str(dtype)[6:]}.{op}", close(t, ref, tol) and
                   (t.device.type == ("cpu" if where == "host" else dev.type)))
    t = _x(me, 50, torch.float64).to(dev)
    comm.all_reduce(t, "prod")
    ref = _x(0, 50, torch.float64)
    for r in range(1, ws):
        ref = ref * _x(r, 50, torch.float64)
    ok("all_reduce.prod", close(t, ref))
    # ---- all_reduce_coalesced ----
    a, b = _x(me, 10, torch.float64).to(dev), _x(me, 7, torch.float64, 1).to(dev)
    comm.all_reduce_coalesced([a, b])
    ok("all_reduce_coalesced", close(a, _fold([_x(r, 10, torch.float64) for r in range(ws)], "sum")) and
       close(b, _fold([_x(r, 7, torch.float64, 1) for r in range(ws)], "sum")))
    # ---- reduce_scatter (+ async): dim 0 = ws * 5 rows ----
    full = [_x(r, ws * 5 * 3, torch.float64, 2).view(ws * 5, 3) for r in range(ws)]
    want = _fold(full, "sum")[me * 5:(me + 1) * 5]
    for where in ("dev", "host"):
        src = full[me].clone() if where == "host" else full[me].to(dev)
        got = comm.reduce_scatter(src)
        ok(f"reduce_scatter.{where}", close(got, want) and got.device.type == src.device.type)
        got = comm.reduce_scatter_async(src.clone()).wait()
        ok(f"reduce_scatter_async.{where}", close(got, want) and got.device.type == src.device.type)
    # non-divisible dim 0: blocks of ceil(n / ws) rows, the last ones shorter or empty, no row dropped
    for n in (ws * 5 + 2, ws + 1):
        full = [_x(r, n * 3, torch.float64, 6).view(n, 3) for r in range(ws)]
        lo, hi = comm.scatter_block(n, ws, me)
        want = _fold(full, "sum")[lo:hi]
        for where in ("dev", "host"):
            src = full[me].clone() if where == "host" else full[me].to(dev)
            got = comm.reduce_scatter(src)
            ok(f"reduce_scatter.uneven{n}.{where}", got.shape == want.shape and close(got, want))
            got = comm.reduce_scatter_async(src.clone()).wait()
            ok(f"reduce_scatter_async.uneven{n}.{where}", got.shape == want.shape and close(got, want))
        blocks = comm.all_gather_object((lo, hi))
        ok(f"reduce_scatter.uneven{n}.cover", [b for blk in blocks for b in blk][0] == 0 and blocks[-1][1] == n
           and all(blocks[i][1] == blocks[i + 1][0] for i in range(ws - 1)))
    mx = [_x(r, ws * 4, torch.float32, 3).view(ws * 4, 1) for r in range(ws)]
    got = comm.reduce_scatter(mx[me].to(dev), "max")
    ok("reduce_scatter.max", close(got, _fold(mx, "max")[me * 4:(me + 1) * 4], 1e-6))
    # ---- all_reduce_async ----
    for where in ("dev", "host"):
        x = _x(me, 4096, torch.float64, 4)
        t = x.clone() if where == "host" else x.to(dev)
        p = comm.all_reduce_async(t)
        got = p.wait()
        ok(f"all_reduce_async.{where}", got is t and close(t, _fold([_x(r, 4096, torch.float64, 4)
                                                                       for r in range(ws)], "sum")))
    # ---- all_gather_tensor / varlen (+ async) / arrays ----
    for where in ("dev", "host"):
        x = _x(me, 6, torch.float64, 5).view(3, 2)
        got = comm.all_gather_tensor(x if where == "host" else x.to(dev))
        ok(f"all_gather_tensor.{where}", close(got, torch.cat([_x(r, 6, torch.float64, 5).view(3, 2)
                                                                for r in range(ws)])))
    lens = [2 + 3 * r for r in range(ws)]
    vx = [torch.arange(lens[r] * 2, dtype=torch.int64).view(lens[r], 2) + 100 * r for r in range(ws)]
    got = comm.all_gather_varlen(vx[me].to(dev))
    ok("all_gather_varlen", torch.equal(got.cpu(), torch.cat(vx)))
    got = comm.all_gather_varlen(vx[me].to(dev), lens=lens)
    ok("all_gather_varlen.known_lens", torch.equal(got.cpu(), torch.cat(vx)))
    got = comm.host_all_gather(torch.tensor([[me, 2 * me, 7]], dtype=torch.int64))
    ok("host_all_gather", torch.equal(got, torch.tensor([[r, 2 * r, 7] for r in range(ws)], dtype=torch.int64)))
    got = comm.all_gather_varlen_async(vx[me].to(dev)).wait()
    ok("all_gather_varlen_async", torch.equal(got.cpu(), torch.cat(vx)))
    got = comm.all_gather_varlen_async(vx[me].clone()).wait()
    ok("all_gather_varlen_async.host", torch.equal(got, torch.cat(vx)) and not got.is_cuda)
    arrs = comm.all_gather_arrays([np.arange(r + 1, dtype=np.float64) for r in range(me, me + 2)])
    ok("all_gather_arrays", all(np.array_equal(arrs[r][j], np.arange(r + j + 1, dtype=np.float64))
                                for r in range(ws) for j in range(2)))
    # ---- all-to-all: tensors (device + host, 2-D), bytes, strings, objects ----
    for where in ("dev", "host"):
        send = [torch.full((me + j + 1, 2), float(10 * me + j), dtype=torch.float64) for j in range(ws)]
        send = send if where == "host" else [s.to(dev) for s in send]
        got = comm.all_to_all_tensors(send)
        ok(f"all_to_all_tensors.{where}", len(got) == ws and all(
            torch.equal(got[i].cpu(), torch.full((i + me + 1, 2), float(10 * i + me), dtype=torch.float64))
            for i in range(ws)) and got[0].device.type == send[0].device.type)
    got = comm.all_to_all_bytes([f"{me}->{j}".encode() * (j + 1) for j in range(ws)])
    ok("all_to_all_bytes", got == [f"{i}->{me}".encode() * (me + 1) for i in range(ws)])
    blocks = [StringBlock.from_list([f"r{me}j{j}", None, "é" * (j + 1)]) for j in range(ws)]
    got = comm.all_to_all_strings(blocks)
    ok("all_to_all_strings", [b.to_list() for b in got] == [[f"r{i}j{me}", None, "é" * (me + 1)]
                                                           for i in range(ws)])
    got = comm.all_to_all_objects([{"src": me, "dst": j} for j in range(ws)])
    ok("all_to_all_objects", got == [{"src": i, "dst": me} for i in range(ws)])
    got = comm.all_to_all_objects([[f"s{me}", None] for j in range(ws)])
    ok("all_to_all_objects.strings", got == [[f"s{i}", None] for i in range(ws)])
    # ---- objects + barrier ----
    ok("all_gather_object", comm.all_gather_object(("rank", me)) == [("rank", r) for r in range(ws)])
    ok("broadcast_object", comm.broadcast_object({"v": me * 7} if me == 0 else None) == {"v": 0})
    comm.barrier()
    ok("barrier", True)
    if gpu:
        torch.cuda.synchronize(dev)
    out["checks"] = res
    out["stats"] = comm.STATS.as_dict()
    from alink_amd.parallel import oneshot
    out["oneshot_instance"] = oneshot._INSTANCE is not None
    out["oneshot_setup_error"] = oneshot.SETUP_ERROR


def run(rank, world, port, outdir, tag="default"):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    if world == 1:
        os.environ["ALINK_COMM_FORCE_COLLECTIVE"] = "1"
    out = {}
    try:
        checks(out)
    except Exception:
        out["error"] = traceback.format_exc()
    try:
        from alink_amd.parallel import comm
        comm.shutdown()
    except Exception:
        out["shutdown_error"] = traceback.format_exc()
    with open(os.path.join(outdir, f"comm_{tag}_{world}_{rank}.json"), "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    run(int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], *(sys.argv[5:6] or []))
