"""Comm-stream discipline (parallel/comm.py _on_comm_stream): RCCL collectives issued from the dedicated comm
stream with event waits both ways, on a 1-rank RCCL process group (the one configuration a 1-GPU box can run)."""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nccl_group():
    import torch.distributed as dist
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    yield dist
    dist.destroy_process_group()


def test_collectives_on_comm_stream_order_with_compute(nccl_group):
    from alink_amd.parallel import comm
    dist = nccl_group
    dev = torch.device("cuda", 0)
    cs = comm.comm_stream(dev)
    assert cs != torch.cuda.current_stream(dev)
    for _ in range(20):
        x = torch.randn(1 << 20, device=dev)
        y = x * 3.0                                   # producer on the compute stream
        comm._on_comm_stream(dev, [y], lambda: dist.all_reduce(y))
        z = y + 1.0                                   # consumer on the compute stream after the event wait
        torch.testing.assert_close(z, x * 3.0 + 1.0)


def test_async_reduce_scatter_pending_waits_on_event(nccl_group):
    from alink_amd.parallel import comm
    dist = nccl_group
    dev = torch.device("cuda", 0)
    x = torch.randn(4096, 8, device=dev)
    src = (x * 2.0).contiguous()
    out = torch.empty_like(src)

    def issue():
        w = dist.reduce_scatter_tensor(out, src, async_op=True)
        w.wait()
    _, done = comm._on_comm_stream(dev, [src, out], issue, wait_now=False)
    busy = torch.randn(2048, 2048, device=dev) @ torch.randn(2048, 2048, device=dev)   # overlapping compute
    p = comm.Pending(out, None, lambda v: comm._wait_event(dev, done, v), keep=(src,))
    got = p.wait() + 0.0
    torch.testing.assert_close(got, x * 2.0)
    assert torch.isfinite(busy).all()
