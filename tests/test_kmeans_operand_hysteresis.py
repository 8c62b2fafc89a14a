"""bf16 centroid-operand hysteresis of the general KMeans path (ops/kmeans.py held_operand; the fused update
kernel applies the same rule on the GPU): operands are held inside the one-ulp band of the row's largest
coordinate and re-rounded outside it; ALINK_KMEANS_HYSTERESIS=0 turns it off."""
import torch

from alink_amd.ops import kmeans as K


def test_held_inside_band_rerounded_outside(monkeypatch):
    K._HELD.clear()
    g = torch.Generator().manual_seed(0)
    C = torch.randn(7, 64, dtype=torch.float64, generator=g) * 5
    a = K.held_operand(C)
    assert torch.equal(a, C.to(torch.bfloat16))
    m = C.abs().amax(1, keepdim=True).float()
    ulp = torch.ldexp(torch.ones_like(m), torch.frexp(m)[1] - 8).double()
    b = K.held_operand(C + 0.25 * ulp)                 # |C' - a| <= 0.5 + 0.25 ulp < 1 ulp: held
    assert torch.equal(b, a)
    c = K.held_operand(C + 3.0 * ulp)                  # outside the band: plain rounding
    assert torch.equal(c, (C + 3.0 * ulp).to(torch.bfloat16))
    monkeypatch.setenv("ALINK_KMEANS_HYSTERESIS", "0")
    K._HELD.clear()
    K.held_operand(C)
    d = K.held_operand(C + 0.25 * ulp)
    assert torch.equal(d, (C + 0.25 * ulp).to(torch.bfloat16))
