"""GPU: the receptive-field window kernels (csrc/merlin_window.hip) and the window-path update.

merlin_tower_window_lut / _window_conv3 against torch gathers of the same tables on a real
rollout's windows; merlin_segment_sum against index_add in float64 (skewed lists, with and
without a minibatch slot map) and bitwise run to run; CNNActorCritic.evaluate_windows against
the reference-structured frame path (F.conv2d towers on the rendered frames): outputs and every
parameter gradient; one PPO update with windows against the per-frame lookup path."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rollout_codes(device, N=256, T=32):
    from merlin import MerlinVecEnv

    env = MerlinVecEnv(N, "mediumhard", seed=777, device=device)
    codes = torch.zeros((T + 1, N, 8), dtype=torch.int32, device=device)
    env.reset(out=codes[0])
    g = torch.Generator(device=device)
    g.manual_seed(5)
    for t in range(T):
        a = torch.randint(0, 3, (N,), device=device, generator=g)
        env.step_into(a, codes[t + 1], torch.empty(N, device=device), None, None, torch.empty(N, device=device))
    env.errors()
    return codes[:T].reshape(-1, 8)


def _plan(device):
    from merlin.dedup import FrameGroups
    from merlin.windows import WindowPlan

    codes = _rollout_codes(device)
    fg = FrameGroups(codes)
    assert fg.ok
    return codes, WindowPlan(codes, fg)


def test_window_lut_and_conv3_match_gathers(device):
    from merlin import _native as nat
    from merlin.windows import P2_OF

    codes, plan = _plan(device)
    torch.manual_seed(0)
    T2 = torch.randn(2, nat.LUT2_ROWS, 64, device=device)
    torch.testing.assert_close(nat.window_lut(plan.rows, T2), T2[:, plan.rows.long()].sum(2), rtol=1e-5, atol=1e-5)
    mb = plan.minibatch(torch.randperm(codes.shape[0], device=device)[:1000])
    nw = plan.num_windows
    Q = torch.randn(2, nw, 576, device=device)
    b3 = torch.randn(2, 64, device=device)
    Y3 = nat.window_conv3(Q, plan.wid, mb.groups, b3)
    w = plan.wid[mb.groups].long()[:, torch.tensor(P2_OF, device=device)]
    ref = torch.relu(Q.view(2, nw, 9, 64)[:, w, torch.arange(9, device=device)].sum(3) + b3[:, None, None])
    torch.testing.assert_close(Y3.view(2, -1, 9, 64), ref, rtol=1e-5, atol=1e-5)
    # the ReLU bit words written beside Y3 (bit co of row r = Y3[t][r][co] > 0), and the masked
    # segment sum reading them == reading the float mask
    Y3b, bits = nat.window_conv3(Q, plan.wid, mb.groups, b3, bits=True)
    assert torch.equal(Y3b, Y3)
    shifts = torch.arange(64, device=device, dtype=torch.int64)
    assert torch.equal((bits.unsqueeze(-1) >> shifts) & 1, (Y3 > 0).long())
    from merlin.windows import SegmentPlan
    n = Y3.shape[1]
    g = torch.Generator(device=device)
    g.manual_seed(3)
    keys = torch.randint(0, 500, (n,), device=device, generator=g)
    o = torch.sort(keys, stable=True).indices
    sp = SegmentPlan(keys[o], o)
    dY = torch.randn_like(Y3)
    a = nat.segment_sum(dY, sp, 500, mask=Y3)
    b = nat.segment_sum(dY, sp, 500, mask=bits)
    assert torch.equal(a, b)


def test_window_conv3_patch_reuse_bitwise(device):
    """merlin_tower_window_conv3_reuse (each distinct patch of a minibatch computed once, the rows sharing it
    copied) == every row computed: Y3, ReLU bit words and the operand scale, bit for bit, on every bulk
    minibatch of two epochs (the last one ragged); copy=2 / 0 write the representative rows (and the masks)
    only.  The bulk builder's maps (merlin_minibatch_patch_maps): rep_row and the live-patch map kmap."""
    from merlin import _native as nat

    codes, plan = _plan(device)
    B = codes.shape[0]
    g = torch.Generator(device=device)
    g.manual_seed(11)
    perms = [torch.randperm(B, device=device, generator=g) for _ in range(2)]
    mbs = plan.update_minibatches(perms, 3000, bulk=True)
    Q = torch.randn(2, plan.num_windows, 576, device=device, generator=g)
    b3 = torch.randn(2, 64, device=device, generator=g)
    shared = 0
    for epoch in mbs:
        for mb in epoch:
            n = int(mb.groups.numel())
            rr = mb.rep_row.long()
            assert rr.numel() == n * 9 and bool((rr >= 0).all()) and bool((rr < n * 9).all())
            assert torch.equal(rr[rr], rr)  # representatives represent themselves
            live = plan.kid[mb.groups].reshape(-1)
            assert torch.equal(live[rr], live)  # and hold the row's patch
            own = torch.arange(n * 9, device=device)
            shared += int((rr != own).sum())
            # the live-patch map of the S pass: kmap[k] = k exactly for the minibatch's patches, else -1
            lv = torch.zeros(plan.num_patches, dtype=torch.bool, device=device)
            lv[live.long()] = True
            assert torch.equal(mb.kmap >= 0, lv)
            assert torch.equal(mb.kmap[lv], torch.nonzero(lv).view(-1).to(torch.int32))
            # one representative per distinct patch
            assert int((rr == own).sum()) == int(lv.sum())
            am0 = torch.zeros(2, dtype=torch.int32, device=device)
            am1 = torch.zeros(2, dtype=torch.int32, device=device)
            Y0, b0 = nat.window_conv3(Q, plan.wid, mb.groups, b3, bits=True, amax=am0)
            Y1, b1 = nat.window_conv3(Q, plan.wid, mb.groups, b3, bits=True, amax=am1, rep_row=mb.rep_row)
            assert torch.equal(Y0, Y1) and torch.equal(b0, b1) and torch.equal(am0, am1)
            for copy in (2, 0):
                am1.zero_()
                Y2, b2 = nat.window_conv3(Q, plan.wid, mb.groups, b3, bits=True, amax=am1, rep_row=mb.rep_row,
                                          copy=copy)
                reps = rr == own
                assert torch.equal(Y2.view(2, -1, 64)[:, reps], Y0.view(2, -1, 64)[:, reps])
                assert torch.equal(b2[:, reps], b0[:, reps]) and torch.equal(am1, am0)
                if copy == 2:
                    assert torch.equal(b2, b0)
                else:  # no copies: the patch sums read every row's mask word through its representative
                    dY = torch.randn(2, n * 9, 64, device=device, generator=g)
                    ref = nat.segment_sum(dY, plan.patch_plan, plan.num_patches, slot=mb.slot, sub=9, mask=b0)
                    got = nat.segment_sum(dY, plan.patch_plan, plan.num_patches, slot=mb.slot, sub=9, mask=b2,
                                          mask_rows=mb.rep_row)
                    assert torch.equal(got, ref)
                    # the same through the two-launch fix-up form (SEG_FUSED off: no head_fix / counters passed)
                    fused0 = nat.SEG_FUSED
                    nat.SEG_FUSED = False
                    try:
                        got2 = nat.segment_sum(dY, plan.patch_plan, plan.num_patches, slot=mb.slot, sub=9, mask=b2,
                                               mask_rows=mb.rep_row)
                    finally:
                        nat.SEG_FUSED = fused0
                    assert torch.equal(got2, ref)
    assert shared > 0  # rows actually copied


@pytest.mark.parametrize("n,nkeys,L,use_slot", [(1, 3, 4, False), (5000, 37, 64, True),
                                                (200000, 3000, 1024, True), (70000, 2, 256, False)])
def test_segment_sum_matches_index_add(device, n, nkeys, L, use_slot):
    from merlin import _native as nat
    from merlin.windows import SegmentPlan

    g = torch.Generator(device=device)
    g.manual_seed(n)
    keys = (torch.rand(n, device=device, generator=g) ** 3 * nkeys).long()  # long and short lists
    F_, S = 5000, 9
    idx = torch.randint(0, F_ * S, (n,), device=device, generator=g)
    o = torch.sort(keys, stable=True).indices
    plan = SegmentPlan(keys[o], idx[o], item_len=L)
    if use_slot:
        slot = torch.full((F_,), -1, dtype=torch.int32, device=device)
        chosen = torch.randperm(F_, device=device, generator=g)[:1500]
        slot[chosen] = torch.arange(1500, dtype=torch.int32, device=device)
        src = torch.randn(2, 1500 * S, 64, device=device, generator=g)
        s = slot[idx // S].long()
        keep = s >= 0
        rows, kk = s[keep] * S + idx[keep] % S, keys[keep]
    else:
        slot = None
        src = torch.randn(2, F_ * S, 64, device=device, generator=g)
        rows, kk = idx, keys
    out = nat.segment_sum(src, plan, nkeys, slot=slot, sub=S)
    ref = torch.zeros(2, nkeys, 64, dtype=torch.float64, device=device)
    mag = torch.zeros_like(ref)
    for t in range(2):
        ref[t].index_add_(0, kk, src[t, rows].double())
        mag[t].index_add_(0, kk, src[t, rows].double().abs())
    err = (out.double() - ref).abs()
    assert (err <= 1e-5 * mag + 1e-6).all(), (err / (mag + 1e-6)).max().item()
    assert torch.equal(out, nat.segment_sum(src, plan, nkeys, slot=slot, sub=S))  # fixed order
    # marks: exactly the keys with a live entry; without fill their rows are the same sums, the others untouched
    mark = torch.full((nkeys,), -1, dtype=torch.int32, device=device)
    got = torch.full_like(out, 7.0)
    nat.segment_sum(src, plan, nkeys, slot=slot, sub=S, out=got, fill=False, mark=mark)
    has = torch.zeros(nkeys, dtype=torch.bool, device=device)
    has[kk] = True
    ar = torch.arange(nkeys, dtype=torch.int32, device=device)
    assert torch.equal(mark, torch.where(has, ar, torch.full_like(ar, -1)))
    assert torch.equal(got[:, has], out[:, has])
    # keys crossing items get their (zero) fix-up row written even when dead; every other dead key is untouched
    crossing = torch.zeros(nkeys, dtype=torch.bool, device=device)
    fx = plan.fix[plan.fix[:, 0] >= 0, 0].long()
    crossing[fx] = True
    assert (got[:, ~has & ~crossing] == 7.0).all()
    # accumulate: a second list added onto the first's sums, exactly the fp32 sum of the two
    keys2 = torch.randint(0, nkeys, (n,), device=device, generator=g)
    o2 = torch.sort(keys2, stable=True).indices
    plan2 = SegmentPlan(keys2[o2], idx[o2], item_len=L)
    out2 = nat.segment_sum(src, plan2, nkeys, slot=slot, sub=S)
    both = nat.segment_sum(src, plan2, nkeys, slot=slot, sub=S, out=out.clone(), accumulate=True)
    assert torch.equal(both, out + out2)


@pytest.mark.parametrize("n,nkeys,L", [(300000, 50, 64), (200000, 3000, 16), (5000, 4000, 1024)])
def test_segment_sum_in_launch_fixups_equal_fix_pass(device, n, nkeys, L, monkeypatch):
    """merlin_segment_sum_fused: destinations spanning items (some over thousands of them) are finished inside the
    launch by the item that completes their count -- the same bits as the separate k_seg_fix pass, on every call
    (the counters come back to zero), with accumulate and a slot map too."""
    from merlin import _native as nat
    from merlin.windows import SegmentPlan

    g = torch.Generator(device=device)
    g.manual_seed(n + L)
    keys = (torch.rand(n, device=device, generator=g) ** 4 * nkeys).long()
    F_, S = 3000, 9
    idx = torch.randint(0, F_ * S, (n,), device=device, generator=g)
    o = torch.sort(keys, stable=True).indices
    plan = SegmentPlan(keys[o], idx[o], item_len=L)
    assert int((plan.fix[:, 2] - plan.fix[:, 1]).max()) >= 1  # rows spanning items
    slot = torch.full((F_,), -1, dtype=torch.int32, device=device)
    slot[torch.randperm(F_, device=device, generator=g)[:2000]] = torch.arange(2000, dtype=torch.int32, device=device)
    src = torch.randn(2, 2000 * S, 64, device=device, generator=g)
    base = torch.randn(2, nkeys, 64, device=device, generator=g)
    monkeypatch.setattr(nat, "SEG_FUSED", False)
    want = nat.segment_sum(src, plan, nkeys, slot=slot, sub=S)
    want_acc = nat.segment_sum(src, plan, nkeys, slot=slot, sub=S, out=base.clone(), accumulate=True)
    monkeypatch.setattr(nat, "SEG_FUSED", True)
    for _ in range(3):
        assert torch.equal(nat.segment_sum(src, plan, nkeys, slot=slot, sub=S), want)
        assert torch.equal(nat.segment_sum(src, plan, nkeys, slot=slot, sub=S, out=base.clone(), accumulate=True),
                           want_acc)
        assert int(plan.counters.abs().sum()) == 0


@pytest.mark.parametrize("L", [16, 1024])
def test_segment_sum_masked_no_fill(device, L):
    """merlin_segment_sum_masked: the ReLU mask of a second tensor fused into the gathers, and
    NO_FILL leaving the rows of keys without a live entry untouched (here a NaN sentinel)."""
    from merlin import _native as nat
    from merlin.windows import SegmentPlan

    g = torch.Generator(device=device)
    g.manual_seed(L)
    n, nkeys, F_, S = 60000, 9000, 4000, 9
    keys = (torch.rand(n, device=device, generator=g) ** 2 * nkeys).long()
    idx = torch.randint(0, F_ * S, (n,), device=device, generator=g)
    o = torch.sort(keys, stable=True).indices
    plan = SegmentPlan(keys[o], idx[o], item_len=L)
    slot = torch.full((F_,), -1, dtype=torch.int32, device=device)
    chosen = torch.randperm(F_, device=device, generator=g)[:700]
    slot[chosen] = torch.arange(700, dtype=torch.int32, device=device)
    src = torch.randn(2, 700 * S, 64, device=device, generator=g)
    mask = torch.randn(2, 700 * S, 64, device=device, generator=g)
    out = torch.full((2, nkeys, 64), float("nan"), device=device)
    nat.segment_sum(src, plan, nkeys, slot=slot, sub=S, mask=mask, fill=False, out=out)
    s = slot[idx // S].long()
    keep = s >= 0
    rows, kk = s[keep] * S + idx[keep] % S, keys[keep]
    dz = torch.where(mask > 0, src, torch.zeros((), device=device)).double()
    ref = torch.zeros(2, nkeys, 64, dtype=torch.float64, device=device)
    mag = torch.zeros_like(ref)
    for t in range(2):
        ref[t].index_add_(0, kk, dz[t, rows])
        mag[t].index_add_(0, kk, dz[t, rows].abs())
    live = torch.zeros(nkeys, dtype=torch.bool, device=device)
    live[kk] = True
    # keys whose entries all fall outside the slot map: untouched, unless they span items (the
    # fix-up writes their zero carry)
    spans = torch.zeros(nkeys, dtype=torch.bool, device=device)
    f = plan.fix[:, 0].long()
    spans[f[f >= 0]] = True
    assert torch.isnan(out[:, ~live & ~spans]).all()
    assert (out[:, ~live & spans] == 0).all()
    err = (out[:, live].double() - ref[:, live]).abs()
    assert (err <= 1e-5 * mag[:, live] + 1e-6).all()


def _loss(lp, ent, v):
    return -(lp.exp() * 0.7).mean() + 0.5 * (v ** 2).mean() - 0.05 * ent.mean()


def test_evaluate_windows_matches_frames(device):
    """evaluate_windows (conv2/conv3 once per distinct window) against the reference-structured frame
    path (rendered frames through the F.conv2d towers) computed in float64: outputs and every
    parameter's gradient.  (float64 is the yardstick: the fp32 MIOpen path itself drifts by 1e-3 on the
    conv-1 weight gradient with the FAST find mode the suite runs under, tests/conftest.py.)"""
    from merlin import _native as nat
    from merlin.actor_critic import CNNActorCritic

    codes, plan = _plan(device)
    mb_idx = torch.randperm(codes.shape[0], device=device)[:2048]
    acts = torch.randint(0, 3, (2048,), device=device)
    torch.manual_seed(12)
    ac = CNNActorCritic((56, 56, 3), 3).to(device)
    lp1, e1, v1 = ac.evaluate_windows(plan, plan.minibatch(mb_idx), acts)
    _loss(lp1, e1, v1).backward()
    g1 = [p.grad.clone() for p in ac.parameters()]
    ac64 = CNNActorCritic((56, 56, 3), 3).to(device)
    ac64.load_state_dict(ac.state_dict())
    ac64.double()
    frames = nat.expand_obs(codes, index=mb_idx, scale=1.0 / 255.0).double()
    logits = ac64.actor(ac64.actor_extractor(frames, prescaled=True))
    v2 = ac64.critic(ac64.critic_extractor(frames, prescaled=True)).squeeze(-1)
    logp = logits.log_softmax(-1)
    lp2 = logp.gather(-1, acts[:, None]).squeeze(-1)
    e2 = -(logp.exp() * logp).sum(-1)
    _loss(lp2, e2, v2).backward()
    g2 = [p.grad for p in ac64.parameters()]
    torch.testing.assert_close(lp1.double(), lp2, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(e1.double(), e2, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(v1.double(), v2, rtol=1e-5, atol=1e-5)
    for (name, _), a, b in zip(ac.named_parameters(), g1, g2):
        rel = ((a.double() - b).norm() / b.norm().clamp_min(1e-30)).item()
        assert rel < 1e-4, (name, rel)


def test_window_update_matches_lookup_path(device):
    """PPO.update through the windows == through per-frame table lookups, same rollout."""
    from merlin import MerlinVecEnv
    from merlin.ppo import PPO

    N, T = 256, 32
    res = []
    for windows in (True, False):
        env = MerlinVecEnv(N, "mediumhard", seed=777, device=device)
        torch.manual_seed(3)
        g = torch.Generator(device=device)
        g.manual_seed(11)
        agent = PPO(env, batch_size=N * T, minibatch_size=N * T // 4, update_epochs=2, ent_coef=0.05,
                    device=device, windows=windows,
                    perm_fn=lambda n, e: torch.randperm(n, device=device, generator=g))
        torch.manual_seed(4)
        stats = agent.update(agent.collect_rollouts())
        res.append((stats, [p.detach().clone() for p in agent.ac.parameters()], agent.last_num_windows))
    (s1, p1, nw), (s2, p2, none) = res
    assert none is None and 0 < nw < 25 * N * T, nw
    for k in s1:
        tol = 4.0 / (N * T // 4) if k == "clipfrac" else 1e-4 * max(1.0, abs(s2[k]))
        assert abs(s1[k] - s2[k]) <= tol, (k, s1[k], s2[k])
    # Adam moves an element by at most ~lr per step, so fp32 summation-order noise in a
    # near-zero gradient can flip an element's step sign: bound every element by 2 lr x steps,
    # and count noticeable differences over all parameters at once (a per-tensor fraction on a
    # 32-element bias is 1/32-granular; the lookup path's atomic conv2-table histogram makes it
    # vary in the last bits from run to run)
    ds = [(a - b).abs().flatten() for a, b in zip(p1, p2)]
    for d in ds:
        assert d.max().item() <= 2 * 3e-4 * 8
    assert (torch.cat(ds) > 5e-5).float().mean().item() < 0.05


def test_evaluate_windows_autograd_grad_fc1(device):
    """torch.autograd.grad through evaluate_windows for the fc1 weights: the x6 path hands fc1's weight
    gradient back through autograd (the deferred .grad delivery is only for PPO._sgd, which opts in
    with deferred_fc1_wgrad), leaves .grad untouched, and equals what loss.backward() accumulates,
    with and without the opt-in."""
    from merlin.actor_critic import CNNActorCritic
    from merlin.windows import deferred_fc1_wgrad

    codes, plan = _plan(device)
    mb = plan.minibatch(torch.randperm(codes.shape[0], device=device)[:2048])
    acts = torch.randint(0, 3, (2048,), device=device)
    torch.manual_seed(12)
    ac = CNNActorCritic((56, 56, 3), 3).to(device)
    w = [ac.actor[0].weight, ac.critic[0].weight]
    ga = torch.autograd.grad(_loss(*ac.evaluate_windows(plan, mb, acts)), w)
    torch.cuda.synchronize()
    assert all(p.grad is None for p in ac.parameters())
    _loss(*ac.evaluate_windows(plan, mb, acts)).backward()
    gb = [p.grad.clone() for p in w]
    ac.zero_grad(set_to_none=True)
    with deferred_fc1_wgrad():
        _loss(*ac.evaluate_windows(plan, mb, acts)).backward()
    torch.cuda.synchronize()
    gc = [p.grad.clone() for p in w]
    # (evaluate_windows' index_select backward is an atomic index_add over the samples of a frame, so
    # the three runs agree to fp32 summation order, not bit for bit)
    for a, b, c in zip(ga, gb, gc):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-9)
        torch.testing.assert_close(c, b, rtol=1e-4, atol=1e-9)
    # requires_grad=False on fc1: no gradient anywhere near it, other parameters still get theirs
    ac.zero_grad(set_to_none=True)
    for p in w:
        p.requires_grad_(False)
    with deferred_fc1_wgrad():
        _loss(*ac.evaluate_windows(plan, mb, acts)).backward()
    torch.cuda.synchronize()
    assert all(p.grad is None for p in w)
    assert ac.actor_extractor.network[0].weight.grad is not None
