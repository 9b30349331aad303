"""optim.ReferenceAdam: the reference's torch.optim.Adam(params, lr=…) (model/graph/HCCF.py:33) as
one capturable kernel (hgd_adam_step) — bit for bit torch's own Adam on this device, eagerly and
replayed from a HIP graph, across steps, learning-rate changes (ReduceLROnPlateau) and tensors of
different sizes."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _params(dev, seed=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    shapes = [(3001, 64), (1777, 64), (64, 32), (64, 32), (5,)]
    return [torch.randn(s, device=dev, generator=g) * 0.1 for s in shapes]


def _grads(dev, params, steps, seed=1):
    g = torch.Generator(device=dev).manual_seed(seed)
    return [[torch.randn(p.shape, device=dev, generator=g) * 10.0 ** (-(k % 4)) for p in params]
            for k in range(steps)]


def test_a_kernel_variant_is_bitwise_torch_adam(dev):
    from hypergraph_diffusion_for_recommendation_amd.optim import calibrated_variant
    v = calibrated_variant(dev)
    print(f"hgd_adam_step variant bitwise torch's Adam: {v}")
    assert v is not None


@pytest.mark.parametrize("rows", [512, 8], ids=["table512", "table8"])
@pytest.mark.parametrize("graph", [False, True], ids=["eager", "graph"])
def test_reference_adam_equals_torch_adam(dev, graph, rows, monkeypatch):
    """60 steps, an lr change at step 25 (the table rebuilt), and with an 8-row table its
    rebuilds every 8 steps (the graph keeps reading the same device table and row index)."""
    from hypergraph_diffusion_for_recommendation_amd import optim
    from hypergraph_diffusion_for_recommendation_amd.optim import ReferenceAdam
    monkeypatch.setattr(optim, "_TABLE_ROWS", rows)
    p0 = _params(dev)
    steps = 60
    grads = _grads(dev, p0, steps)
    ref = [p.clone().requires_grad_(True) for p in p0]
    mine = [p.clone().requires_grad_(True) for p in p0]
    topt = torch.optim.Adam(ref, lr=1e-3)
    ropt = ReferenceAdam(mine, lr=1e-3)
    gbuf = [torch.zeros_like(p) for p in p0]
    for p, b in zip(mine, gbuf):
        p.grad = b  # static gradient buffers (what a captured backward writes)
    cap = None
    for k in range(steps):
        if k == 25:  # the scheduler's decay: both read the group's lr at their next step
            for opt in (topt, ropt):
                for group in opt.param_groups:
                    group["lr"] *= 0.7
        for p, gr in zip(ref, grads[k]):
            p.grad = gr.clone()
        topt.step()
        for b, gr in zip(gbuf, grads[k]):
            b.copy_(gr)
        if not graph or k == 0:
            ropt.step()  # the first step allocates the state (as the plugin's eager step)
        else:
            if cap is None:
                torch.cuda.synchronize()
                cap = torch.cuda.CUDAGraph()
                with torch.cuda.graph(cap):
                    ropt.launch()
            ropt.prepare()
            cap.replay()
        for a, b in zip(mine, ref):
            assert torch.equal(a.detach(), b.detach()), k
    for a, b in zip(mine, ref):
        assert torch.equal(ropt.state[a]["exp_avg"], topt.state[b]["exp_avg"])
        assert torch.equal(ropt.state[a]["exp_avg_sq"], topt.state[b]["exp_avg_sq"])
        assert float(ropt.state[a]["step"]) == float(topt.state[b]["step"]) == steps
