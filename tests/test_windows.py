"""CPU: the receptive-field window plan of merlin/windows.py (what the kernels of
csrc/merlin_window.hip consume), in float64 with torch gathers standing in for the kernels:
  * window keys / table rows == the per-position conv2 table rows (lut2_rows, itself checked
    against F.conv2d in test_conv2_tables.py);
  * the segment plans (fixed-length items + fix-ups), restated step by step as k_seg_sum /
    k_seg_fix run them, == index_add, with and without a minibatch slot map;
  * conv2 -> conv3 through the windows == the reference towers' convolutions of the rendered
    frames, and the plan's backward lists (the two dQ passes through the 5x5 patches with the
    ReLU mask fused, dT2) == autograd of the gathers."""
import numpy as np
import pytest
import torch

from test_conv2_tables import _model, lut2_rows


def pack(codes_u8: np.ndarray) -> np.ndarray:
    n = codes_u8.shape[0]
    nib = np.zeros((n, 64), dtype=np.uint32)
    nib[:, :49] = codes_u8
    w = (nib.reshape(n, 8, 8) << (4 * np.arange(8, dtype=np.uint32))).sum(-1).astype(np.uint32)
    return w.view(np.int32)


def test_window_rows_match_position_rows():
    from merlin.windows import unpack_classes, window_keys, window_rows

    rs = np.random.RandomState(0)
    c = rs.randint(0, 5, size=(300, 49)).astype(np.uint8)
    cls = unpack_classes(torch.from_numpy(pack(c)))
    assert (cls.reshape(300, 49).numpy() == c).all()
    rows = window_rows(window_keys(cls).reshape(-1)).reshape(300, 25, 16)
    assert (rows.numpy() == lut2_rows(c)).all()


def emulate_segment_sum(plan, src, out_rows, slot=None, sub=1, mask=None, fill=True):
    """Step-by-step restatement of k_seg_sum + k_seg_fix (csrc/merlin_window.hip); mask: rows of
    src where mask > 0 (the MASK variant); fill=False: unwritten rows come back NaN."""
    T, C = src.shape[0], src.shape[2]
    if mask is not None:
        src = torch.where(mask > 0, src, torch.zeros((), dtype=src.dtype))
    out = torch.zeros(T, out_rows, C, dtype=src.dtype) if fill else torch.full((T, out_rows, C), float("nan"),
                                                                                 dtype=src.dtype)
    carry = torch.zeros(T, max(plan.nitems, 1), 2, C, dtype=src.dtype)
    key, idx, L, n = plan.key.tolist(), plan.idx.tolist(), plan.item_len, plan.nnz
    for it in range(plan.nitems):
        e0, e1 = it * L, min(n, it * L + L)
        kf, kl = key[e0], key[e1 - 1]
        xf = e0 > 0 and key[e0 - 1] == kf
        xl = e1 < n and key[e1] == kl
        sums = {}
        for e in range(e0, e1):
            v = idx[e]
            if slot is not None:
                s = int(slot[v // sub])
                if s < 0:
                    continue
                v = s * sub + v % sub
            sums[key[e]] = sums[key[e]] + src[:, v] if key[e] in sums else src[:, v].clone()
        for k, a in sums.items():
            if k == kf and (xf or (kf == kl and xl)):
                carry[:, it, 0] = a
            elif k == kl and xl:
                carry[:, it, 1] = a
            else:
                out[:, k] = a
    for d, j0, j1, s0 in plan.fix.tolist():
        if d < 0:
            continue
        a = carry[:, j0, s0].clone()
        part = [torch.zeros_like(a) for _ in range(4)]  # k_seg_fix: item j0+1+i goes to partial i % 4
        for i, j in enumerate(range(j0 + 1, j1 + 1)):
            part[i % 4] += carry[:, j, 0]
        out[:, d] = a + ((part[0] + part[1]) + (part[2] + part[3]))
    return out


@pytest.mark.parametrize("n,nkeys,L,skew", [(1, 3, 4, False), (50, 5, 7, False), (500, 20, 16, True),
                                            (300, 1, 8, False), (257, 300, 4, False), (0, 4, 8, False),
                                            (3000, 3, 4, True)])
def test_segment_plan_sums_every_destination(n, nkeys, L, skew):
    from merlin.windows import SegmentPlan

    g = torch.Generator().manual_seed(n + nkeys)
    keys = (torch.rand(n, generator=g) ** 4 * nkeys).long() if skew else torch.randint(0, nkeys, (n,), generator=g)
    idx = torch.randint(0, 40, (n,), generator=g)
    o = torch.sort(keys, stable=True).indices
    plan = SegmentPlan(keys[o], idx[o], item_len=L)
    src = torch.randn(2, 40, 64, dtype=torch.float64, generator=g)
    ref = torch.zeros(2, nkeys, 64, dtype=torch.float64)
    for t in range(2):
        ref[t].index_add_(0, keys, src[t, idx])
    torch.testing.assert_close(emulate_segment_sum(plan, src, nkeys), ref)
    # through a slot map: entry v = frame * 4 + k reads row slot[frame] * 4 + k; frames outside skipped
    slot = torch.full((10,), -1, dtype=torch.int32)
    slot[torch.tensor([1, 3, 4, 8])] = torch.arange(4, dtype=torch.int32)
    src_mb = torch.randn(2, 16, 64, dtype=torch.float64, generator=g)
    ref = torch.zeros(2, nkeys, 64, dtype=torch.float64)
    for e in range(n):
        s = int(slot[idx[e] // 4])
        if s >= 0:
            ref[:, keys[e]] += src_mb[:, s * 4 + idx[e] % 4]
    torch.testing.assert_close(emulate_segment_sum(plan, src_mb, nkeys, slot=slot, sub=4), ref)


def test_window_towers_match_frame_convs(golden):
    """Y3 through windows == relu(conv3(relu(conv2(relu(conv1(frame)))))) of the reference
    modules; dQ and dT2 from the plan's lists == autograd of the torch gathers."""
    import oracle as O

    from merlin.dedup import FrameGroups
    from merlin.windows import P2_OF, WindowPlan

    ac, atlas = _model(41, golden, torch.float64)
    rs = np.random.RandomState(42)
    c = rs.randint(0, 5, size=(12, 49)).astype(np.uint8)
    c[:, 45] = 4
    c = np.concatenate([c, c[:5]])  # repeated observations share a frame id
    codes = torch.from_numpy(pack(c))
    plan = WindowPlan(codes, FrameGroups(codes), item_len=16, hist_item_len=8)
    assert plan.num_frames == 12
    mb_idx = torch.tensor([0, 3, 12, 5, 7, 14, 9, 3])
    mb = plan.minibatch(mb_idx)
    ea, ec = ac.actor_extractor.network, ac.critic_extractor.network
    T2 = ac.conv2_tables().detach().requires_grad_(True)
    Z2w = T2[:, plan.rows.long()].sum(2)  # k_window_lut
    a2w = torch.relu(Z2w + torch.stack([ea[2].bias, ec[2].bias]).unsqueeze(1))
    W3 = torch.stack([ea[4].weight, ec[4].weight])
    Q = torch.bmm(a2w, W3.permute(0, 2, 3, 4, 1).reshape(2, 64, 576)).detach().requires_grad_(True)
    w = plan.wid[mb.groups].long()[:, torch.tensor(P2_OF)]  # [U, 9 p3, 9 tap]
    b3 = torch.stack([ea[4].bias, ec[4].bias]).detach()
    Y3 = torch.relu(Q.view(2, -1, 9, 64)[:, w, torch.arange(9)].sum(3) + b3[:, None, None])  # k_window_conv3
    x = torch.from_numpy(O.render(c[mb_idx.numpy()], atlas).astype(np.float64)).permute(0, 3, 1, 2) / 255.0
    with torch.no_grad():
        for t, net in enumerate((ea, ec)):
            ref = net[:6](x).permute(0, 2, 3, 1).reshape(-1, 9, 64)
            torch.testing.assert_close(Y3[t][mb.inv], ref, rtol=1e-10, atol=1e-10)
    g = torch.randn(2, mb.groups.numel(), 9, 64, dtype=torch.float64)
    (Y3 * g).sum().backward()
    # the three passes of _WindowConv3.backward: per-patch sums of the masked rows (patches of
    # frames outside the minibatch left unwritten = NaN here), band sums over the live patches,
    # then dQ from the bands
    assert plan.num_patches <= 12 * 9 and plan.patch_plan.nnz == 12 * 9
    assert plan.band_plan.nnz == plan.num_patches * 3 and plan.dq_plan.nnz == plan.num_bands * 3
    R = emulate_segment_sum(plan.patch_plan, g.reshape(2, -1, 64), plan.num_patches, slot=mb.slot, sub=9,
                            mask=Y3.detach().reshape(2, -1, 64), fill=False)
    live = plan.kid[mb.groups].reshape(-1).long()
    kmap = torch.full((plan.num_patches,), -1, dtype=torch.int32)
    kmap[live] = live.to(torch.int32)
    assert torch.isnan(R[:, kmap < 0]).all() and not torch.isnan(R[:, live]).any()
    S = emulate_segment_sum(plan.band_plan, R, plan.num_bands, slot=kmap, sub=1)
    dQ = emulate_segment_sum(plan.dq_plan, S, plan.num_windows * 9)
    torch.testing.assert_close(dQ.view_as(Q), Q.grad)
    dZ3 = torch.where(Y3 > 0, g, torch.zeros((), dtype=g.dtype))
    torch.testing.assert_close(dQ.view(2, plan.num_windows, 9, 64)[:, :, 0].sum(1), dZ3.sum((1, 2)))  # db3
    dZ2w = torch.randn(2, plan.num_windows, 64, dtype=torch.float64)
    (T2[:, plan.rows.long()].sum(2) * dZ2w).sum().backward()
    torch.testing.assert_close(emulate_segment_sum(plan.hist, dZ2w, 2720), T2.grad)


def test_epoch_minibatches_match_per_minibatch_grouping():
    """WindowPlan.epoch_minibatches (one sort per epoch) == minibatch() on every chunk."""
    from merlin.dedup import FrameGroups
    from merlin.windows import WindowPlan

    rs = np.random.RandomState(7)
    base = rs.randint(0, 5, size=(40, 49)).astype(np.uint8)
    codes = torch.from_numpy(pack(base[rs.randint(0, 40, size=1000)]))
    plan = WindowPlan(codes, FrameGroups(codes))
    idxs = torch.randperm(1000, generator=torch.Generator().manual_seed(1))
    for mbs in (128, 300, 1000):
        got = plan.epoch_minibatches(idxs, mbs)
        assert len(got) == (1000 + mbs - 1) // mbs
        for k, m in enumerate(got):
            ref = plan.minibatch(idxs[k * mbs:(k + 1) * mbs])
            assert torch.equal(m.groups, ref.groups) and torch.equal(m.inv, ref.inv)
            assert m.groups.dtype == torch.int64 and m.inv.dtype == torch.int64 and m.slot.dtype == torch.int32
            assert torch.equal(m.slot, ref.slot)
            assert torch.equal(m.order, ref.order) and torch.equal(m.offs, ref.offs)
            # CSR: frame u's samples are order[offs[u]:offs[u+1]], ascending, all with inv == u
            o, f = m.order.long(), m.offs.long()
            assert f[0] == 0 and f[-1] == o.numel() and bool((f[1:] > f[:-1]).all())
            frame_of = torch.repeat_interleave(torch.arange(f.numel() - 1), f[1:] - f[:-1])
            assert torch.equal(m.inv[o], frame_of)
            assert bool((o[1:] > o[:-1])[frame_of[1:] == frame_of[:-1]].all())
    # every epoch at once (one host read per update) == epoch by epoch
    perms = [torch.randperm(1000, generator=torch.Generator().manual_seed(s)) for s in (2, 3, 4)]
    for mbs in (128, 300):
        allm = plan.update_minibatches(perms, mbs)
        for e, p in enumerate(perms):
            ref = plan.epoch_minibatches(p, mbs)
            assert len(allm[e]) == len(ref)
            for m, r in zip(allm[e], ref):
                for a in ("groups", "inv", "slot", "order", "offs"):
                    assert torch.equal(getattr(m, a), getattr(r, a)), a


def test_window_and_patch_keys_match_digit_loops():
    """window_keys / patch_keys (built from per-row keys) == the tile-by-tile base-5 accumulation, tile (0, 0) most
    significant, on random class grids including the all-4 corner case."""
    from merlin.windows import patch_keys, window_keys

    cls = torch.randint(0, 5, (300, 7, 7), generator=torch.Generator().manual_seed(2), dtype=torch.int64)
    cls[0] = 4
    wk = torch.zeros((300, 5, 5), dtype=torch.int64)
    for a in range(3):
        for b in range(3):
            wk = wk * 5 + cls[:, a:a + 5, b:b + 5]
    pk = torch.zeros((300, 3, 3), dtype=torch.int64)
    for a in range(5):
        for b in range(5):
            pk = pk * 5 + cls[:, a:a + 3, b:b + 3]
    assert torch.equal(window_keys(cls), wk.reshape(-1, 25)) and torch.equal(patch_keys(cls), pk.reshape(-1, 9))
    assert int(pk.max()) == 5 ** 25 - 1


def test_compact_window_keys_cover_observable_windows():
    """The acting table's compact keys (csrc/merlin_window.hip k_codes_conv3, round 5): every window an observation
    can hold has exactly one key, and the key the kernel computes for a window (restated here) names a table row
    built for that same window (merlin/windows.py compact_window_keys -> window_rows)."""
    import torch

    from merlin.windows import compact_window_keys

    keys = compact_window_keys("cpu")
    assert keys.numel() == 4 ** 9 + 3 * 4 ** 8 and torch.unique(keys).numel() == keys.numel()
    digits = torch.stack([(keys // 5 ** (8 - i)) % 5 for i in range(9)], 1)
    agent = digits == 4
    assert int(agent[: 4 ** 9].sum()) == 0 and bool((agent[4 ** 9:].sum(1) == 1).all())

    def kernel_key(view, wy, wx):  # k_codes_conv3's key of the window at conv2 position (wy, wx)
        skip = 9 - wx if (wy == 4 and 1 <= wx <= 3) else -1
        k = 0
        for a in range(3):
            for b in range(3):
                if 3 * a + b != skip:
                    k = k * 4 + min(int(view[wy + a][wx + b]), 3)
        return k + (262144 + (wx - 1) * 65536 if skip >= 0 else 0)

    g = torch.Generator().manual_seed(0)
    for _ in range(200):
        view = torch.randint(0, 4, (7, 7), generator=g)
        view[6][3] = 4  # the agent's tile, always at view cell (3, 6)
        for wy in range(5):
            for wx in range(5):
                base5 = sum(int(view[wy + a][wx + b]) * 5 ** (8 - 3 * a - b) for a in range(3) for b in range(3))
                assert int(keys[kernel_key(view, wy, wx)]) == base5
