"""GPU: PPO._sgd's minibatch step with its launches written out (merlin/fast_step.py: parameter-only work as two
captured HIP graphs, bookkeeping as views of update-wide arrays, gradients written straight into a flat buffer)
against the same kernels driven by the autograd engine (PPO.fast_step = False).  Same operands, same order: the
update statistics and every parameter / Adam moment agree bit for bit over several updates, with the rollouts
in between (so the second update runs on weights the first one changed: the captured graphs replay on live
parameters)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(device, fast, iters=3):
    from merlin import MerlinVecEnv
    from merlin.ppo import PPO

    env = MerlinVecEnv(256, "mediumhard", seed=5, device=device)
    torch.manual_seed(3)
    agent = PPO(env, lr=1e-3, batch_size=256 * 64, minibatch_size=256 * 16, update_epochs=2, ent_coef=0.05,
                device=device)
    agent.fast_step = fast
    stats = []
    for _ in range(iters):
        stats.append(agent.update(agent.collect_rollouts()))
    torch.cuda.synchronize()
    return agent, stats


def test_fast_step_matches_autograd_bitwise(device):
    a0, s0 = _run(device, False)
    a1, s1 = _run(device, True)
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


def test_fast_step_recaptures_after_parameter_swap(device):
    """Replacing a parameter's storage (e.g. a new module) invalidates the captured stage graphs."""
    agent, _ = _run(device, True, iters=1)
    st = agent._wstep
    assert st.valid()
    w = agent.ac.actor[0].weight
    w.data = w.data.clone()
    assert not st.valid()
