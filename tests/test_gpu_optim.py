"""GPU: merlin_clip_adam (csrc/merlin_optim.hip, merlin/optim.py ClipAdam) against the reference's
optimizer step (src/ppo.py:153-156: nn.utils.clip_grad_norm_(params, 0.5) then optim.Adam.step())
run by torch on an identical copy of the parameters: several steps, clipping active and inactive,
the CNNActorCritic parameter shapes and views of one flat buffer (the data-parallel layout).
Tolerance: fp32, the norm summed in another order (rtol 2e-6 on the norm; parameters within a few
ulps of Adam's update size)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _shapes():
    from merlin.actor_critic import CNNActorCritic

    return [tuple(p.shape) for p in CNNActorCritic((56, 56, 3), 3).parameters()]


def _make(shapes, device, flat, seed):
    g = torch.Generator().manual_seed(seed)
    vals = [torch.randn(s, generator=g) * 0.05 for s in shapes]
    if not flat:
        return [v.to(device).requires_grad_() for v in vals]
    buf = torch.cat([v.reshape(-1) for v in vals]).to(device)
    out, off = [], 0
    for v in vals:
        n = v.numel()
        out.append(torch.nn.Parameter(buf[off:off + n].view(v.shape)))
        off += n
    return out


@pytest.mark.parametrize("flat", [False, True])
@pytest.mark.parametrize("gscale", [1e-4, 3.0])
def test_clip_adam_matches_torch(device, flat, gscale):
    from merlin.optim import ClipAdam

    shapes = _shapes()
    mine = _make(shapes, device, flat, 0)
    ref = [torch.nn.Parameter(p.detach().clone()) for p in mine]
    opt_m = torch.optim.Adam(mine, lr=2.5e-4, fused=True)
    opt_r = torch.optim.Adam(ref, lr=2.5e-4, fused=True)
    ca = ClipAdam(opt_m, 0.5)
    gen = torch.Generator().manual_seed(1)
    for step in range(4):
        grads = [(torch.randn(s, generator=gen) * gscale).to(device) for s in shapes]
        for p, q, gr in zip(mine, ref, grads):
            p.grad = gr.clone()
            q.grad = gr.clone()
        n_m = ca.step()
        n_r = torch.nn.utils.clip_grad_norm_(ref, 0.5)
        opt_r.step()
        torch.cuda.synchronize()
        assert torch.allclose(n_m, n_r, rtol=2e-6, atol=0), (step, float(n_m), float(n_r))
        for p, q in zip(mine, ref):
            assert torch.allclose(p.grad, q.grad, rtol=4e-6, atol=1e-12), step
            # per-element Adam update is <= lr; a few ulps of it plus the parameter's own ulp
            torch.testing.assert_close(p.detach(), q.detach(), rtol=2e-6, atol=2.5e-4 * 1e-5)
            sm, sr = opt_m.state[p], opt_r.state[q]
            assert float(sm["step"]) == float(sr["step"]) == step + 1
            torch.testing.assert_close(sm["exp_avg"], sr["exp_avg"], rtol=1e-5, atol=1e-10)
            torch.testing.assert_close(sm["exp_avg_sq"], sr["exp_avg_sq"], rtol=1e-5, atol=1e-14)
    # the torch optimizer can continue from the kernel's state
    assert opt_m.state_dict()["state"].keys() == opt_r.state_dict()["state"].keys()


def test_clip_adam_rejects_mismatched_state(device):
    from merlin import _native as nat

    p = torch.zeros(10, device=device)
    with pytest.raises(ValueError):
        nat.clip_adam([p], [p[:5]], [p], [p], [torch.zeros((), device=device)], 1e-3, 0.9, 0.999, 1e-8, 0.5)


@pytest.mark.parametrize("bad", [float("nan"), float("inf")])
def test_clip_adam_nonfinite_gradient_matches_torch(device, bad):
    """A non-finite gradient element: torch's clip_grad_norm_ keeps the NaN / zero coefficient
    (clamp(max=1) propagates NaN), so the kernel must poison the same elements torch does."""
    from merlin.optim import ClipAdam

    shapes = _shapes()
    mine = _make(shapes, device, True, 3)
    ref = [torch.nn.Parameter(p.detach().clone()) for p in mine]
    opt_m = torch.optim.Adam(mine, lr=2.5e-4, fused=True)
    opt_r = torch.optim.Adam(ref, lr=2.5e-4, fused=True)
    ca = ClipAdam(opt_m, 0.5)
    gen = torch.Generator().manual_seed(2)
    grads = [(torch.randn(s, generator=gen) * 1e-3).to(device) for s in shapes]
    grads[3].view(-1)[7] = bad
    for p, q, gr in zip(mine, ref, grads):
        p.grad = gr.clone()
        q.grad = gr.clone()
    n_m = ca.step()
    n_r = torch.nn.utils.clip_grad_norm_(ref, 0.5)
    opt_r.step()
    torch.cuda.synchronize()
    assert (torch.isnan(n_m) == torch.isnan(n_r)).all() and (torch.isinf(n_m) == torch.isinf(n_r)).all()
    for p, q in zip(mine, ref):
        # same non-finite pattern everywhere; finite values equal up to Adam rounding
        assert torch.equal(torch.isfinite(p.grad), torch.isfinite(q.grad))
        assert torch.equal(torch.isfinite(p.detach()), torch.isfinite(q.detach()))
        fin = torch.isfinite(q.detach())
        torch.testing.assert_close(p.detach()[fin], q.detach()[fin], rtol=2e-6, atol=2.5e-4 * 1e-5)
