"""One-shot all-reduce kernel (ops/csrc/allreduce.hip) on one GPU: P local staging areas stand in for the P
ranks' IPC-mapped buffers; every virtual rank copies + signals (phase 1), then each waits + sums (phase 2)."""
import pytest
import torch

from alink_amd.parallel.oneshot import OneShot

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("P", [1, 2, 3, 8, 12])
@pytest.mark.parametrize("dtype,op", [(torch.float64, "sum"), (torch.float32, "sum"), (torch.float64, "max"),
                                      (torch.float32, "min")])
def test_oneshot_reduction_matches_torch(P, dtype, op):
    cap = 1 << 19
    bases = [OneShot.alloc(cap, P) for _ in range(P)]
    views = [OneShot("cuda", P, r, cap, bases, [], []) for r in range(P)]
    try:
        for call in range(4):                      # slots alternate with the sequence number
            n = [1, 1000, 5000, 60000][call]       # last: several elements per thread (P <= 8: unrolled loads)
            xs = [torch.randn(n, device="cuda", dtype=dtype) for _ in range(P)]
            outs = [torch.empty_like(x) for x in xs]
            seq = call + 1
            for r in range(P):
                views[r].launch(xs[r], outs[r], op, phases=1, seq=seq)
            for r in range(P):
                views[r].launch(xs[r], outs[r], op, phases=2, seq=seq)
            torch.cuda.synchronize()
            st = torch.stack(xs)
            ref = st.sum(0) if op == "sum" else (st.max(0).values if op == "max" else st.min(0).values)
            if op == "sum":
                # rank-order summation: identical to a sequential fold
                acc = xs[0].clone()
                for x in xs[1:]:
                    acc = acc + x
                ref = acc
            for r in range(P):
                assert torch.equal(outs[r], ref), (r, call)
            assert all(int(v.err.item()) == 0 for v in views)
    finally:
        views[0].owned = bases
        views[0].close()


def test_oneshot_missing_peer_times_out_with_nan(monkeypatch):
    import alink_amd.parallel.oneshot as O
    monkeypatch.setattr(O, "TIMEOUT_S", 0.05)
    cap = 1 << 12
    bases = [OneShot.alloc(cap, 2) for _ in range(2)]
    v = OneShot("cuda", 2, 0, cap, bases, bases, [])
    x = torch.ones(100, dtype=torch.float64, device="cuda")
    out = torch.empty_like(x)
    v.launch(x, out, "sum", phases=3, seq=1)     # peer 1 never signals
    torch.cuda.synchronize()
    assert int(v.err.item()) == 1 and bool(torch.isnan(out).all())
    # the mapped host word carries the failure too: the next call's check raises without a device copy
    with pytest.raises(RuntimeError, match="timed out"):
        v.check()
    assert int(v.err.item()) == 0                    # re-armed after raising
    # in-place all_reduce_ of a non-contiguous tensor (staged through a contiguous copy) on a healthy 1-rank view
    one = OneShot("cuda", 1, 0, cap, [bases[0]], [], [])
    y = torch.arange(24, dtype=torch.float64, device="cuda").view(4, 6).t()
    ref = y.clone()
    one.all_reduce_(y)
    torch.cuda.synchronize()
    assert torch.equal(y, ref)
    one.close()
    v.close()
