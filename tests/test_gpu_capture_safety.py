"""GPU: HIP-graph captures survive garbage that holds HIP resources, and the fast step survives parameter
changes (round-3 verdict items: the capture-time abort of gpurun_out/t_w.log; ADVICE: WindowStep after a
parameter swap or with a frozen parameter).

* garbage cycles holding a MerlinVecEnv and an old agent with captured graphs exist when a new agent captures
  its rollout, with the collector set to run on every allocation: the capture completes (merlin._native
  capture_guard keeps the collector off inside it) and the replayed rollout equals an eager agent's bit for bit
  (the action draws are counter-based, so the same seeds and weights give the same rollout);
* a native release requested inside an open capture (MerlinVecEnv.close -> merlin_env_destroy) waits for the
  capture to end instead of invalidating it;
* a rebound parameter (p.data = ...) is put back on the flat buffer, the rollout graph is re-captured and the
  next update runs on the fast step; a frozen parameter sends the update down the autograd path and stays
  bit-identical while the others train."""
import gc

import pytest
import torch

pytestmark = pytest.mark.gpu

N, T = 128, 16


def _agent(device, graph=True, seed=777):
    from merlin import MerlinVecEnv
    from merlin.ppo import PPO

    env = MerlinVecEnv(N, "mediumhard", seed=seed, device=device, max_steps=12)
    torch.manual_seed(0)
    return PPO(env, batch_size=N * T, minibatch_size=N * T // 4, update_epochs=1, ent_coef=0.05, device=device,
               rollout_graph=graph)


def _make_garbage(device):
    from merlin import MerlinVecEnv

    old = _agent(device)
    old.update(old.collect_rollouts())  # a captured rollout graph + the fast step's captured stage graphs
    old.collect_rollouts()
    old.cycle = old  # reachable only through a cycle once dropped
    env = MerlinVecEnv(64, "mediumhard", seed=3, device=device)
    env.reset()
    box = {"env": env}
    box["self"] = box


def test_capture_with_cyclic_garbage_holding_hip_resources(device):
    from merlin import _native as nat

    gc.collect()
    eager = _agent(device, graph=False)
    ref = [eager.collect_rollouts().clone() for _ in range(2)]
    ref_codes, ref_act = eager.buf.codes.clone(), eager.buf.actions.clone()
    old_threshold = gc.get_threshold()
    _make_garbage(device)
    gc.set_threshold(1)
    try:
        agent = _agent(device)
        lvs = [agent.collect_rollouts().clone() for _ in range(2)]  # eager + capture, then a replay
    finally:
        gc.set_threshold(*old_threshold)
    assert agent._graph is not None and agent.rollout_graph
    assert gc.isenabled() and not nat._DEFERRED
    torch.cuda.synchronize()
    assert torch.equal(agent.buf.codes, ref_codes) and torch.equal(agent.buf.actions, ref_act)
    for a, b in zip(lvs, ref):
        assert torch.equal(a, b)
    agent.vec.errors()


def test_release_inside_capture_is_deferred(device):
    from merlin import MerlinVecEnv
    from merlin import _native as nat

    victim = MerlinVecEnv(64, "mediumhard", seed=9, device=device)
    victim.reset()
    x = torch.zeros(1024, device=device)
    g = torch.cuda.CUDAGraph()
    with nat.capture_guard(), torch.cuda.graph(g):
        x.add_(1.0)
        victim.close()  # would be a hipFree inside the capture
        assert len(nat._DEFERRED) == 1
    assert not nat._DEFERRED and victim._h is None
    g.replay()
    torch.cuda.synchronize()
    assert float(x[0]) == 1.0


def test_update_after_parameter_rebind(device):
    agent = _agent(device)
    agent.update(agent.collect_rollouts())
    assert agent._wstep is not None and agent._wstep.valid()
    w = agent.ac.actor[0].weight
    w.data = w.data.clone()  # off the flat buffer: the captured graphs hold the old addresses
    assert not agent._params_on_flat()
    with torch.no_grad():
        w.mul_(0.5)  # the next rollout must act with this
    lv = agent.collect_rollouts()
    assert agent._params_on_flat() and agent._graph is not None
    with torch.no_grad():
        _, _, v = agent.ac.act_codes(agent.buf.codes[T])
    torch.testing.assert_close(v, agent.buf.last_value, rtol=1e-5, atol=1e-5)
    before = w.detach().clone()
    stats = agent.update(lv)
    assert all(torch.isfinite(torch.tensor(s)) for s in stats.values())
    assert agent._wstep is not None and agent._wstep.valid()
    assert not torch.equal(before, w.detach())


def test_frozen_parameter_stays_and_others_train(device):
    agent = _agent(device)
    agent.update(agent.collect_rollouts())  # fast step first: every .grad bound to the flat buffer
    frozen = agent.ac.critic[0].bias
    frozen.requires_grad_(False)
    keep = frozen.detach().clone()
    others = [p.detach().clone() for p in agent.ac.parameters() if p.requires_grad]
    for _ in range(2):
        agent.update(agent.collect_rollouts())
    assert torch.equal(frozen.detach(), keep) and frozen.grad is None
    moved = [not torch.equal(a, p.detach()) for a, p in zip(others, [p for p in agent.ac.parameters()
                                                                      if p.requires_grad])]
    assert all(moved)


def test_captured_scale_reduction_replays_correctly(device):
    """merlin_h3_amax inside a captured HIP graph (the fast step's forward graph computes fc1's weight scale this
    way) must give every replay's own max: its zeroing is a kernel, not a hipMemsetAsync -- a memset node captured on
    ROCm 7 replayed with the fill value 0x80808080 (scripts/probe_graph_then.py), an operand scale of 2^120."""
    from merlin import _native as nat

    S = torch.zeros(2, 64, device=device)
    am = torch.zeros(2, dtype=torch.int32, device=device)
    nat.h3_amax(S, out=am)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        nat.h3_amax(S, out=am)
    R = torch.zeros(20, 2, dtype=torch.int32, device=device)
    for k in range(20):
        S.fill_(float(k + 1))
        S[1].mul_(-0.5)
        g.replay()
        R[k].copy_(am)
    torch.cuda.synchronize()
    want = torch.tensor([[k + 1.0, (k + 1.0) / 2] for k in range(20)], device=device)
    assert torch.equal(R.view(torch.float32), want)


def _zero_branch_cases(device):
    """Every library entry point that zero-fills an output without running its main kernel (empty row / frame /
    entry lists, K = 0, or the chunked conv3 backward's scale word), as (name, fn) with fn() -> output tensors."""
    from merlin import _native as nat
    from merlin.windows import SegmentPlan

    f32 = dict(dtype=torch.float32, device=device)
    codes = torch.zeros((4, nat.OBS_WORDS), dtype=torch.int32, device=device)
    T, H, A = 2, 512, 3
    outs = {
        "colsum": torch.empty((T, 64), **f32),
        "relu_bwd_bias": torch.empty((T, 64), **f32),
        "head_b": torch.empty((2, H), **f32), "head_wa": torch.empty((A, H), **f32), "head_wc": torch.empty(H, **f32),
        "x6_tn": torch.empty((T, 16, 24), **f32),
        "seg": torch.empty((T, 10, 64), **f32),
    }
    empty = torch.empty((T, 0, 64), **f32)
    plan = SegmentPlan(torch.empty(0, dtype=torch.int32, device=device), torch.empty(0, dtype=torch.int32,
                                                                                      device=device))
    return outs, [
        ("conv1_lut_bwd", lambda: nat.conv1_lut_bwd(codes, None, torch.empty((T, 0, 13, 13, 32), **f32),
                                                    torch.empty((T, 0, 13, 13, 32), **f32))),
        ("conv2_im2col_bwd", lambda: nat.conv2_im2col_bwd(codes, None, torch.zeros((T, 32, 4, 20), **f32),
                                                          torch.zeros((T, 32), **f32), torch.empty((T, 0, 512), **f32))),
        ("conv3_col2im_bwd_chunked", lambda: nat.conv3_col2im_bwd_chunked(
            torch.empty((T, 0, 576), **f32), torch.empty((T, 0, 64), **f32), torch.zeros((T, 64), **f32))[1:]),
        ("conv2_lut_bwd", lambda: (nat.conv2_lut_bwd(codes, torch.empty((T, 16, 0, 4), **f32),
                                                     torch.zeros(1, dtype=torch.int32, device=device)),)),
        ("relu_bwd", lambda: nat.relu_bwd(empty, empty, out_bias=outs["relu_bwd_bias"])[1:]),
        ("colsum", lambda: (nat.colsum(empty, out=outs["colsum"]),)),
        ("head_bwd", lambda: nat.head_bwd(torch.empty((2, 0, H), **f32), torch.empty((0, A), **f32),
                                          torch.empty(0, **f32), torch.zeros((A, H), **f32), torch.zeros(H, **f32),
                                          out_bias=outs["head_b"], out_w_actor=outs["head_wa"],
                                          out_w_critic=outs["head_wc"])[1:]),
        ("x6_gemm_tn", lambda: (nat.x6_gemm_tn(torch.empty((T, 0, 16), **f32), torch.empty((T, 0, 24), **f32),
                                               out=outs["x6_tn"]),)),
        ("segment_sum", lambda: (nat.segment_sum(empty, plan, 10, out=outs["seg"]),)),
    ]


def test_captured_zero_fills_replay_zero(device):
    """Round-4 verdict item 6: no entry point zero-fills with hipMemsetAsync any more (csrc: merlin::zero_async, a
    kernel), so each zero-fill branch captured into a HIP graph and replayed over poisoned outputs writes zeros, on
    every replay."""
    _, cases = _zero_branch_cases(device)
    for name, fn in cases:
        res = fn()  # eager once (allocations, plans)
        torch.cuda.synchronize()
        for r in res:
            assert torch.count_nonzero(r) == 0, name
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            res = fn()
        for rep in range(3):
            for r in res:
                r.view(torch.int32).fill_(0x7fc00001 + rep)  # NaN payload: nothing but a write of zeros clears it
            g.replay()
            torch.cuda.synchronize()
            for r in res:
                assert torch.count_nonzero(r.view(torch.int32)) == 0, (name, rep)
        del g


def test_release_deferred_by_a_plain_capture_is_drained(device):
    """an env closed inside a user's own torch.cuda.graph capture (no capture_guard) queues its release;
    the queue drains at the next env creation with no capture open, not only at a capture_guard exit."""
    from merlin import MerlinVecEnv
    from merlin import _native as nat

    victim = MerlinVecEnv(64, "mediumhard", seed=9, device=device)
    victim.reset()
    x = torch.zeros(16, device=device)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        x.add_(1.0)
        victim.close()
        assert len(nat._DEFERRED) == 1
    assert len(nat._DEFERRED) == 1  # nothing drained it yet
    other = MerlinVecEnv(64, "mediumhard", seed=10, device=device)
    assert not nat._DEFERRED and victim._h is None
    other.close()
    g.replay()
    torch.cuda.synchronize()
    assert float(x[0]) == 1.0
