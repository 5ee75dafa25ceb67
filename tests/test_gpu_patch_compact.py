"""GPU: the minibatch's compact patch list (merlin_patch_compact, round 6) against a torch restatement of its
definition -- the live entries of a destination-sorted plan in plan order, their source rows, each source row's
compact index and the item fix-up rows merlin.windows.SegmentPlan makes for the compact list -- on plans with runs
longer than an item, empty and full slot maps; the R-pass sum over it against the update-wide plan's; the sum over
rows scattered into compact order (the input-gradient GEMM's row-map epilogue) bit for bit against the gathered
form; and merlin_h3_gemm_nt_planes_rowmap bit for bit against the plain GEMM's rows moved by the map."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _plan(device, nnz, F, sub, long_runs, seed):
    from merlin.windows import SegmentPlan

    g = torch.Generator().manual_seed(seed)
    # destinations with geometric run lengths plus a few runs far longer than an item
    runs = torch.distributions.Geometric(torch.tensor(0.3)).sample((nnz,)).long() + 1
    if long_runs:
        runs[torch.randint(0, nnz, (8,), generator=g)] = 700
    key = torch.repeat_interleave(torch.arange(runs.numel()), runs)[:nnz]
    idx = torch.randperm(F * sub, generator=g)[:nnz]
    return SegmentPlan(key.to(torch.int32).to(device), idx.to(torch.int32).to(device), 64)


def _slot(device, F, frac, seed):
    g = torch.Generator().manual_seed(seed)
    live = torch.rand(F, generator=g) < frac
    slot = torch.full((F,), -1, dtype=torch.int32)
    slot[live] = torch.randperm(int(live.sum()), generator=g).to(torch.int32)
    return slot.to(device), int(live.sum())


def _reference(plan, slot, sub, mrow, L, src_rows):
    from merlin.windows import SegmentPlan

    idx = plan.idx.long()
    e = (slot[idx // sub] >= 0).nonzero().squeeze(1)
    ckey = plan.key[e]
    crow = slot[idx[e] // sub].long() * sub + idx[e] % sub
    assert int(crow.max()) < src_rows if crow.numel() else True
    pos = torch.full((src_rows,), -1, dtype=torch.int64, device=crow.device)
    pos[crow] = torch.arange(crow.numel(), device=crow.device)
    cmrow = crow if mrow is None else mrow.long()[crow]
    sp = SegmentPlan(ckey, crow, L) if crow.numel() else None
    return ckey, crow, pos, cmrow, sp


@pytest.mark.parametrize("frac,long_runs", [(0.125, True), (1.0, False), (0.0, False), (0.4, True)])
def test_patch_compact_matches_definition(device, frac, long_runs):
    from merlin import _native as nat

    F, sub = 9000, 9
    plan = _plan(device, 60000, F, sub, long_runs, seed=3)
    slot, nlive_frames = _slot(device, F, frac, seed=4)
    # n_live = the live entries (every row of a live frame need not be in the plan: count them)
    n_live = int((slot[plan.idx.long() // sub] >= 0).sum())
    mrow = torch.randint(0, max(nlive_frames * sub, 1), (max(nlive_frames * sub, 1),), dtype=torch.int32,
                         device=device)[:nlive_frames * sub]
    L = 32
    for use_mrow in (False, True):
        cp = nat.patch_compact(plan, slot, sub, n_live, mask_rows=mrow if use_mrow else None, layout="gather",
                               item_len=L, src_rows=nlive_frames * sub)
        torch.cuda.synchronize()
        ckey, crow, pos, cmrow, sp = _reference(plan, slot, sub, mrow if use_mrow else None, L, nlive_frames * sub)
        assert cp.nnz == n_live == int(ckey.numel())
        assert torch.equal(cp.key.long(), ckey.long())
        assert torch.equal(cp.crow.long(), crow)
        assert torch.equal(cp.cmrow.long(), cmrow.long())
        if n_live:
            assert torch.equal(cp.pos.long()[crow], torch.arange(n_live, device=device))
            assert torch.equal(cp.fix, sp.fix) and torch.equal(cp.head_fix, sp.head_fix)


def _bits(T, rows, device, seed):
    g = torch.Generator(device=device).manual_seed(seed)
    return torch.randint(-2 ** 62, 2 ** 62, (T, rows), dtype=torch.int64, device=device, generator=g)


@pytest.mark.parametrize("L", [32, 128])
def test_compact_sum_matches_full_plan_and_scatter_is_gather(device, L):
    from merlin import _native as nat

    F, sub, T = 6000, 9, 2
    plan = _plan(device, F * sub, F, sub, True, seed=5)  # every (frame, position) once, as a patch plan has them
    slot, nf = _slot(device, F, 0.125, seed=6)
    n = nf * sub
    g = torch.Generator(device=device).manual_seed(7)
    src = torch.randn(T, n, 64, device=device, generator=g)
    bits = _bits(T, n, device, 8)
    K = int(plan.key.max()) + 1
    full = nat.segment_sum(src, plan, K, slot=slot, sub=sub, mask=bits, fill=False)
    cg = nat.patch_compact(plan, slot, sub, n, layout="gather", item_len=L)
    comp = nat.segment_sum(src, cg, K, mask=bits, fill=False)
    live = torch.zeros(K, dtype=torch.bool, device=device)
    live[cg.key.long()] = True
    torch.testing.assert_close(comp[:, live], full[:, live], rtol=1e-5, atol=1e-5)
    # the rows moved into compact order, the mask words through cmrow: the same bits as the gathered sum
    cs = nat.patch_compact(plan, slot, sub, n, layout="scatter", item_len=L)
    src_c = torch.empty_like(src)
    src_c[:, cs.pos.long()] = src
    scat = nat.segment_sum(src_c, cs, K, mask=bits, fill=False, mask_rows=cs.cmrow)
    assert torch.equal(scat[:, live], comp[:, live])
    # and with a row map for the mask words (conv3's patch representatives) on both sides
    mrow = torch.randint(0, n, (n,), dtype=torch.int32, device=device)
    cg2 = nat.patch_compact(plan, slot, sub, n, mask_rows=mrow, layout="gather", item_len=L)
    cs2 = nat.patch_compact(plan, slot, sub, n, mask_rows=mrow, layout="scatter", item_len=L)
    a = nat.segment_sum(src, cg2, K, mask=bits, fill=False, mask_rows=mrow)
    b = nat.segment_sum(src_c, cs2, K, mask=bits, fill=False, mask_rows=cs2.cmrow)
    assert torch.equal(a[:, live], b[:, live])


@pytest.mark.parametrize("M", [1000, 4096 + 77])
def test_h3_rowmap_gemm_is_the_plain_gemm_moved(device, M):
    from merlin import _native as nat

    g = torch.Generator(device=device).manual_seed(11)
    T, K, N = 2, 512, 576
    dz = torch.randn(T, M, K, device=device, generator=g) * 1e-3
    W = torch.randn(T, K, N, device=device, generator=g) / 24
    Wt = W.transpose(1, 2).contiguous()
    amW, amz = nat.h3_amax(Wt), nat.h3_amax(dz)
    PW, pdz = nat.h3_split(Wt, amW), nat.h3_split(dz, amz)
    plain = nat.h3_gemm_nt_planes(pdz, amz, PW, amW, cfg=62)
    rmap = torch.randperm(M * N // 64, device=device, generator=g).to(torch.int32)
    moved = nat.h3_gemm_nt_planes(pdz, amz, PW, amW, cfg=62, row_map=rmap)
    torch.cuda.synchronize()
    assert torch.equal(moved.view(T, -1, 64)[:, rmap.long()], plain.view(T, -1, 64))
