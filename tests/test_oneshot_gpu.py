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


def _fold_sum(xs):
    acc = xs[0].clone()
    for x in xs[1:]:
        acc = acc + x
    return acc


def test_oneshot_peer_already_signalled_next_call():
    """Wrap-safe poll: peers 1 and 2 finish call s and signal call s+1 before rank 0's wave first polls for
    s (a preempted wave, ranks time-sharing a GPU).  Rank 0's flags then read s+1, never s; it must still
    complete call s from the untouched slot s&1, and then call s+1."""
    P, cap = 3, 1 << 16
    bases = [OneShot.alloc(cap, P) for _ in range(P)]
    views = [OneShot("cuda", P, r, cap, bases, [], []) for r in range(P)]
    try:
        n = 4000
        s = 7
        xa = [torch.randn(n, device="cuda", dtype=torch.float64) for _ in range(P)]
        xb = [torch.randn(n, device="cuda", dtype=torch.float64) for _ in range(P)]
        oa = [torch.empty_like(x) for x in xa]
        ob = [torch.empty_like(x) for x in xb]
        for r in range(P):
            views[r].launch(xa[r], oa[r], "sum", phases=1, seq=s)
        for r in (1, 2):
            views[r].launch(xa[r], oa[r], "sum", phases=2, seq=s)
            views[r].launch(xb[r], ob[r], "sum", phases=1, seq=s + 1)      # now one call ahead of rank 0
        views[0].launch(xa[0], oa[0], "sum", phases=2, seq=s)
        torch.cuda.synchronize()
        assert int(views[0].err.item()) == 0
        views[0].launch(xb[0], ob[0], "sum", phases=1, seq=s + 1)
        for r in range(P):
            views[r].launch(xb[r], ob[r], "sum", phases=2, seq=s + 1)
        torch.cuda.synchronize()
        ra, rb = _fold_sum(xa), _fold_sum(xb)
        for r in range(P):
            assert torch.equal(oa[r], ra) and torch.equal(ob[r], rb), r
        assert all(int(v.err.item()) == 0 for v in views)
    finally:
        views[0].owned = bases
        views[0].close()


def test_oneshot_sequence_number_wraps():
    """Sequence numbers are 32-bit: calls 2^32-2, 2^32-1, 0, 1 reduce correctly (the slot alternates with the
    low bit, the arrival test is modular)."""
    P, cap = 2, 1 << 14
    bases = [OneShot.alloc(cap, P) for _ in range(P)]
    views = [OneShot("cuda", P, r, cap, bases, [], []) for r in range(P)]
    try:
        for s in (0xFFFFFFFE, 0xFFFFFFFF, 0x100000000, 0x100000001):
            xs = [torch.randn(300, device="cuda", dtype=torch.float32) for _ in range(P)]
            outs = [torch.empty_like(x) for x in xs]
            for r in range(P):
                views[r].launch(xs[r], outs[r], "sum", phases=1, seq=s)
            for r in range(P):
                views[r].launch(xs[r], outs[r], "sum", phases=2, seq=s)
            torch.cuda.synchronize()
            ref = _fold_sum(xs)
            assert all(torch.equal(o, ref) for o in outs), hex(s)
        assert all(int(v.err.item()) == 0 for v in views)
    finally:
        views[0].owned = bases
        views[0].close()


def test_timeout_on_the_last_reduction_raises_at_shutdown(monkeypatch):
    """A peer that never arrives for the job's LAST one-shot reduction (no later call would check the error word)
    makes comm.shutdown() raise after its cleanup instead of letting a NaN model pass silently."""
    import alink_amd.parallel.oneshot as O
    from alink_amd.parallel import comm
    monkeypatch.setattr(O, "TIMEOUT_S", 0.05)
    cap = 1 << 12
    bases = [OneShot.alloc(cap, 2) for _ in range(2)]
    v = OneShot("cuda", 2, 0, cap, bases, bases, [])
    x = torch.ones(64, dtype=torch.float64, device="cuda")
    v.all_reduce_(x)                                   # peer 1 never signals
    monkeypatch.setattr(O, "_INSTANCE", v)
    with pytest.raises(RuntimeError, match="timed out"):
        comm.shutdown()
    assert O._INSTANCE is None                         # cleaned up before raising
