"""GPU: PPO._sgd's minibatch step with its launches written out (merlin/fast_step.py: parameter-only work as two
captured HIP graphs, bookkeeping as views of update-wide arrays, gradients written straight into a flat buffer)
against the same kernels driven by the autograd engine (PPO.fast_step = False).  With the weight stage's conv
tables on torch ops (stage_impl "torch") the arithmetic is the autograd path's: the update statistics and every
parameter / Adam moment agree bit for bit over several updates, with the rollouts in between (so later updates
run on weights the earlier ones changed: the captured graphs replay on live parameters).  With the tables on
csrc/merlin_stage.hip (the default) the sums run in another fixed order: float32-level agreement, and the same
bits on every run."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(device, fast, iters=3, stage_impl="hip", first_grads=None):
    from merlin import MerlinVecEnv
    from merlin.ppo import PPO

    env = MerlinVecEnv(256, "mediumhard", seed=5, device=device)
    torch.manual_seed(3)
    agent = PPO(env, lr=1e-3, batch_size=256 * 64, minibatch_size=256 * 16, update_epochs=2, ent_coef=0.05,
                device=device)
    agent.fast_step = fast
    agent.stage_impl = stage_impl
    if first_grads is not None:  # record the first optimizer step's (pre-clip) gradient of every parameter
        ca = agent._clip_adam
        orig = ca.step

        def step():
            if not first_grads:
                first_grads.extend(p.grad.detach().clone() for p in agent.ac.parameters())
            return orig()

        ca.step = step
    stats = []
    for _ in range(iters):
        stats.append(agent.update(agent.collect_rollouts()))
    torch.cuda.synchronize()
    return agent, stats


def test_fast_step_matches_autograd_bitwise(device, monkeypatch):
    from merlin import fast_step

    # the autograd path runs the window GEMMs on hipBLASLt: the same GEMMs here (the h3 form of them is held to
    # fp32-GEMM accuracy by tests/test_gpu_h3.py and to the autograd path by the test below)
    monkeypatch.setattr(fast_step, "WINDOW_H3", False)
    monkeypatch.setattr(fast_step, "WINDOW_BWD_HIP", False)  # its own bounds: tests/test_gpu_window_bwd.py
    # and dz in fp32 as the autograd path has it (the bound-scaled planes: tests/test_gpu_dz_planes.py)
    monkeypatch.setattr(fast_step, "DZ_PLANES", False)
    a0, s0 = _run(device, False)
    a1, s1 = _run(device, True, stage_impl="torch")
    assert a1._wstep is not None and a0._wstep is None
    assert a1.last_num_windows == a0.last_num_windows and a1.last_distinct_frac == a0.last_distinct_frac
    for x, y in zip(s0, s1):
        assert x == y
    for (k, p0), p1 in zip(a0.ac.named_parameters(), a1.ac.parameters()):
        assert torch.equal(p0, p1), k
        st0, st1 = a0.optimizer.state[p0], a1.optimizer.state[p1]
        assert torch.equal(st0["exp_avg"], st1["exp_avg"]) and torch.equal(st0["exp_avg_sq"], st1["exp_avg_sq"]), k
    # the fast step leaves every gradient in its view of one flat buffer
    flat = a1._wstep.flat
    for p in a1.ac.parameters():
        assert p.grad is not None and flat.data_ptr() <= p.grad.data_ptr() < flat.data_ptr() + flat.numel() * 4


def test_fast_step_hip_tables_close_and_reproducible(device):
    g0, g1 = [], []
    a0, s0 = _run(device, False, iters=1, first_grads=g0)
    a1, s1 = _run(device, True, iters=1, first_grads=g1)
    a2, s2 = _run(device, True, iters=1)
    assert s1 == s2
    for p1, p2 in zip(a1.ac.parameters(), a2.ac.parameters()):
        assert torch.equal(p1, p2)
    for k in s0[0]:
        assert abs(s0[0][k] - s1[0][k]) <= 1e-4 * max(1.0, abs(s0[0][k])), k
    # the first optimizer step's gradient of every parameter, HIP tables against the autograd path's torch tables:
    # equal to fp32 level (1e-5 of each tensor's norm; the tables' own gradients: test_stage_tables_match_torch)
    names = [k for k, _ in a0.ac.named_parameters()]
    for k, x, y in zip(names, g0, g1):
        rel = float((x - y).norm() / x.norm().clamp_min(1e-30))
        assert rel <= 1e-5, (k, rel)
    # after the update (8 Adam steps) every parameter within the steps' size (lr each): Adam's per-element
    # normalisation turns an fp32-level difference in a gradient element that cancels to ~0 into a ~lr step of
    # either sign, so the parameters are held to that bound and the gradients above to fp32 level
    for (k, p0), p1 in zip(a0.ac.named_parameters(), a1.ac.parameters()):
        d = (p1 - p0).detach().abs()
        assert float(d.max()) <= 2 * 1e-3 * 8, k


def test_stage_tables_match_torch(device):
    """merlin_stage_tables_fwd / _bwd against CNNActorCritic.conv2_tables_from + autograd on random weights."""
    from merlin import CNNActorCritic
    from merlin import _native as nat

    torch.manual_seed(9)
    ac = CNNActorCritic((56, 56, 3), 3).to(device)
    g = torch.Generator(device=device).manual_seed(1)
    W1 = (torch.randn(2, 32, 3, 8, 8, device=device, generator=g) * 0.2).requires_grad_()
    b1 = (torch.randn(2, 32, device=device, generator=g) * 0.1).requires_grad_()
    W2 = (torch.randn(2, 64, 32, 4, 4, device=device, generator=g) * 0.1).requires_grad_()
    T2 = ac.conv2_tables_from(W1, b1, W2)
    dT2 = torch.randn_like(T2)
    gW1, gb1, gW2 = torch.autograd.grad(T2, (W1, b1, W2), grad_outputs=dT2)
    atlas, idx, koff, kv = ac.stage_consts(device)
    HT, T2h = nat.stage_tables_fwd(W1.detach().contiguous(), b1.detach().contiguous(), W2.detach().contiguous(),
                                   atlas, idx)
    torch.testing.assert_close(T2h, T2.detach(), rtol=1e-5, atol=1e-5)
    hW1, hb1, hW2 = nat.stage_tables_bwd(W2.detach().contiguous(), HT, dT2.contiguous(), atlas, koff, kv)
    for a, b in ((hW1, gW1), (hb1, gb1), (hW2, gW2)):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-4 * float(b.abs().max()))
    again = nat.stage_tables_bwd(W2.detach().contiguous(), HT, dT2.contiguous(), atlas, koff, kv)
    assert all(torch.equal(x, y) for x, y in zip(again, (hW1, hb1, hW2)))


def test_fast_step_recaptures_after_parameter_swap(device):
    """Moving the parameters off the flat buffer invalidates the captured stage graphs."""
    agent, _ = _run(device, True, iters=1)
    st = agent._wstep
    assert st.valid()
    w = agent.ac.actor[0].weight
    w.data = w.data.clone()
    assert not st.valid()


def test_patch_reuse_partial_rows_never_read_directly(device, monkeypatch):
    """with conv3's patch reuse, window_conv3 leaves the non-representative rows of Y3 / the mask words
    unwritten; every consumer reads them through rep_row.  With those rows poisoned (NaN / all-ones words) an update
    gives the same bits as without."""
    from merlin import _native as nat

    a0, s0 = _run(device, True, iters=2)
    monkeypatch.setattr(nat, "POISON_PARTIAL", True)
    a1, s1 = _run(device, True, iters=2)
    assert s0 == s1
    for (k, p0), p1 in zip(a0.ac.named_parameters(), a1.ac.parameters()):
        assert torch.equal(p0, p1), k
