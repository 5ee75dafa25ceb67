"""Receptive-field windows: conv2 and conv3 of both towers evaluated once per distinct window.

Every observation is a 7x7 blit of 5 atlas tiles and the towers' convolutions
(src/actor_critic.py:9-14) are translation invariant, so conv2's output at position (py, px)
of a frame is a function of the frame's 3x3 tile-class window at (py, px) alone (conv1 k8/s4
then conv2 k4/s2 see 20 px: tiles py..py+2, the third by its first half).  A bench rollout
of 1,048,576 frames holds 5,411 distinct windows (scripts/probe_windows.py), so each update
numbers them once (WindowPlan) and every minibatch evaluates

  Z2w[t][w]     = conv2(relu(conv1)) of window w: its 16 conv2-table rows summed
                  (merlin_tower_window_lut; tables from CNNActorCritic.conv2_tables)
  Q[t][w][tap]  = relu(Z2w[t][w] + b2[t]) . W3[t][:, :, tap]    one [windows, 64] x [64, 576] GEMM
  Y3[t][u, p3]  = relu(b3[t] + sum over the 9 taps of Q[t][wid[u][p3 + tap]][tap])
                  (merlin_tower_window_conv3) = relu(conv3) of distinct frame u at p3

instead of conv3's im2col rows and GEMMs over every (frame, position).  Backward, autograd
runs through the tables and the GEMM, and the adjoints of the two gathers are segmented sums
over lists sorted once per update (merlin_segment_sum: fixed order, no atomics):

  dQ[t][w][tap] = sum of dZ3[t][u, p3] over the minibatch's (u, p3) whose window at p3 + tap
                  is w, dZ3 = [Y3 > 0] * dY3 (conv3's ReLU backward), in three passes over the
                  5x5-tile patch under each conv3 output (its 9 windows are the patch's 3x3
                  sub-windows at tap = (ky, kx), so (u, p3) with equal patches feed the same 9
                  destinations) and the patch's three 3x5-tile row bands (rows ky..ky+2):
     R[t][k]        = sum of dZ3[t][u, p3] over the (u, p3) whose patch is k   (ReLU mask fused:
                      dY3 rows gathered once each with the 8-B ReLU bit mask that
                      merlin_tower_window_conv3_bits wrote beside Y3; dZ3 never materialised)
     S[t][ky][b]    = sum of R[t][k] over the live patches k whose band ky is b
     dQ[t][w][tap]  = sum of S[t][ky][b] over the bands b of row ky whose window at column kx
                      is w
                  A bench rollout has ~0.5-1M distinct patches but only ~40-70k distinct bands
                  per ky (and ~6k windows): each source row is read once, each R row 3 times
                  and the small S table 3 times (instead of 81 scattered 256-B row gathers per
                  frame from dZ3: 5.6 GB per minibatch)
  db3[t]        = sum over w of dQ[t][w][tap 0]  (every (u, p3) has one window at p3 + 0)
  dT2[t][row]   = sum of dZ2w[t][w] over the (w, tap) that read table row `row`

Same function and gradients as the reference towers, fp32 sums regrouped.  The minibatch's
frames are its distinct observations (merlin/dedup.py); fc1 and the heads run on them.
"""
from __future__ import annotations

import contextlib
import threading

import torch

from . import _native as nat

# conv3 output p3 = (oy, ox) and tap = (ky, kx) -> conv2 position (oy + ky) * 5 + (ox + kx)
P2_OF = [[(p // 3 + k // 3) * 5 + p % 3 + k % 3 for k in range(9)] for p in range(9)]
# (The single-pass form -- dQ straight from dZ3, 81 entries per frame each gathering a 256-B row,
# every row 9 times -- read 5.6 GB per minibatch at the bench size, 0.93 ms, plus a 0.27 ms ReLU
# backward pass writing dZ3: profiles/r02_kernel_stats.md / r02_pmc.json.)


def auto_item_len(nnz: int) -> int:
    """Entries per wave: enough items (~16k, 16 waves per CU) to fill the chip -- a wave walks its
    item's entries in dependent rounds, so a list of few long items is latency-bound (measured on
    the bench's band / dQ lists: 1024-entry items 211 / 187 us, 64 / 32-entry items 87 / 50 us,
    scripts/probe_dq.py) -- between 32 and 1024, a power of two."""
    L = 32
    while L < 1024 and L * 2 * 16384 <= nnz:
        L *= 2
    return L


def unpack_classes(codes: torch.Tensor) -> torch.Tensor:
    """int32 [n, 8] observation codes -> int64 [n, 7, 7] tile classes (cell r*7 + c is nibble
    cell % 8 of word cell // 8, include/merlin_hip.h; clamped to 4 like the kernels)."""
    shifts = torch.arange(0, 32, 4, dtype=torch.int32, device=codes.device)
    nib = (codes.unsqueeze(-1) >> shifts) & 0xF
    return nib.reshape(codes.shape[0], 64)[:, :49].to(torch.int64).clamp_(max=4).view(-1, 7, 7)


def window_keys(cls: torch.Tensor) -> torch.Tensor:
    """[n, 7, 7] classes -> int64 [n, 25]: the 3x3 window at each conv2 position as 9 base-5
    digits, window tile (0, 0) most significant."""
    r = cls[:, :, 0:5] * 25 + cls[:, :, 1:6] * 5 + cls[:, :, 2:7]  # [n, 7, 5]: 3-tile row keys
    return (r[:, 0:5] * 15625 + r[:, 1:6] * 125 + r[:, 2:7]).reshape(-1, 25)


def patch_keys(cls: torch.Tensor) -> torch.Tensor:
    """[n, 7, 7] classes -> int64 [n, 9]: the 5x5-tile patch under each conv3 output p3 =
    (oy, ox) (conv2 positions oy..oy+2 x ox..ox+2, i.e. tiles oy..oy+4 x ox..ox+4) as 25 base-5
    digits, patch tile (0, 0) most significant."""
    r = cls[:, :, 0:3]
    for b in range(1, 5):
        r = r * 5 + cls[:, :, b:b + 3]  # [n, 7, 3]: 5-tile row keys
    k = r[:, 0:3]
    for a in range(1, 5):
        k = k * 3125 + r[:, a:a + 3]
    return k.reshape(-1, 9)


def base5(digits: torch.Tensor) -> torch.Tensor:
    """int64 [n, m] base-5 digits (most significant first) -> int64 [n] keys."""
    k = torch.zeros(digits.shape[0], dtype=torch.int64, device=digits.device)
    for i in range(digits.shape[1]):
        k = k * 5 + digits[:, i]
    return k


def digits5(keys: torch.Tensor, m: int) -> torch.Tensor:
    """int64 [n] keys -> int64 [n, m] base-5 digits, most significant first (inverse of base5)."""
    return torch.stack([(keys // 5 ** (m - 1 - i)) % 5 for i in range(m)], 1)


def window_rows(keys: torch.Tensor) -> torch.Tensor:
    """int64 [m] window keys -> int32 [m, 16]: the conv2 table row each tap 4*ky + kx reads
    (row layout of csrc/merlin_conv2lut.hip, tap_rows)."""
    d = [(keys // 5 ** (8 - i)) % 5 for i in range(9)]  # d[3a + b] = class of window tile (a, b)
    rows = []
    for ky in range(4):
        for kx in range(4):
            i, j = 3 * (ky >> 1) + (kx >> 1), 2 * (ky >> 1) + (kx >> 1)
            if not ky & 1 and not kx & 1:
                r = 4 * d[i] + j
            elif not ky & 1:
                r = 20 + 4 * (5 * d[i] + d[i + 1]) + j
            elif not kx & 1:
                r = 120 + 4 * (5 * d[i] + d[i + 3]) + j
            else:
                r = 220 + 4 * (125 * d[i] + 25 * d[i + 1] + 5 * d[i + 3] + d[i + 4]) + j
            rows.append(r)
    return torch.stack(rows, 1).to(torch.int32)


def compact_window_keys(device) -> torch.Tensor:
    """int64 [4^9 + 3 * 4^8]: the base-5 window key (window_rows' input) of every compact key of the acting path's
    table (csrc/merlin_window.hip k_codes_conv3): keys 0 .. 4^9 - 1 = 9 tile classes 0..3 in base 4 (windows away
    from the agent's view cell); 4^9 + (wx - 1) 4^8 + m = the window at conv2 position (4, wx) with the agent's tile
    (class 4) at local (2, 3 - wx) and its other 8 classes m in base 4."""
    d9 = torch.arange(4 ** 9, dtype=torch.int64, device=device)
    digits = [(d9 // 4 ** (8 - i)) % 4 for i in range(9)]  # digits[3a + b] = class of tile (a, b)
    out = [sum(digits[i] * 5 ** (8 - i) for i in range(9))]
    m = torch.arange(4 ** 8, dtype=torch.int64, device=device)
    d8 = [(m // 4 ** (7 - i)) % 4 for i in range(8)]
    for wx in (1, 2, 3):
        skip = 9 - wx  # local slot 3 * 2 + (3 - wx)
        cls, j = [], 0
        for i in range(9):
            if i == skip:
                cls.append(torch.full_like(m, 4))
            else:
                cls.append(d8[j])
                j += 1
        out.append(sum(cls[i] * 5 ** (8 - i) for i in range(9)))
    return torch.cat(out)


class SegmentPlan:
    """A destination-sorted entry list for merlin_segment_sum: out[key[e]] = sum of src[row(e)]
    over the entries e of that key, in list order.  The list is cut into items of item_len
    entries (one wave each); `fix` holds one row per item, (dst, first item, last item, carry slot
    of the first item) for the destination that starts in that item and continues past it, or
    dst = -1: its partial sums are added in item order.  Built without a host read (a stream
    drain each): every size here is known from the list length."""

    def __init__(self, key_sorted: torch.Tensor, idx_sorted: torch.Tensor, item_len: int | None = None):
        dev = key_sorted.device
        n = int(key_sorted.numel())
        L = auto_item_len(n) if item_len is None else int(item_len)
        self.nnz, self.item_len = n, L
        self.nitems = (n + L - 1) // L
        self.key = key_sorted.to(torch.int32).contiguous()
        self.idx = idx_sorted.to(torch.int32).contiguous()
        if n == 0:
            self.fix = torch.zeros((0, 4), dtype=torch.int32, device=dev)
            self.head_fix = torch.zeros(0, dtype=torch.int32, device=dev)
            self.counters = torch.zeros(0, dtype=torch.int32, device=dev)
            return
        j = torch.arange(self.nitems, dtype=torch.int64, device=dev)
        p = torch.clamp((j + 1) * L, max=n) - 1  # each item's last entry
        # [s, e) = the run of p's key in the sorted list: two binary searches per item (a cummax /
        # cummin scan over all n entries took ~1.3 ms each at the bench size)
        kp = self.key[p].contiguous()
        s = torch.searchsorted(self.key, kp, side="left")
        e = torch.searchsorted(self.key, kp, side="right")
        live = (e > (j + 1) * L) & (s >= j * L)  # starts in this item, continues past it
        dst = torch.where(live, self.key[p].long(), torch.full_like(j, -1))
        self.fix = torch.stack([dst, j, (e - 1) // L, (s != j * L).long()], 1).to(torch.int32).contiguous()
        # for the in-launch fix-ups (merlin_segment_sum_fused): the fix row (= item) at which each item's first
        # destination started, when it continues into the item, else -1; and the rows' arrival counters (each
        # launch leaves them zero)
        kf = self.key[j * L].contiguous()
        sf = torch.searchsorted(self.key, kf, side="left")
        self.head_fix = torch.where(sf < j * L, sf // L, torch.full_like(j, -1)).to(torch.int32).contiguous()
        self.counters = torch.zeros(self.nitems, dtype=torch.int32, device=dev)


class MinibatchWindows:
    """One minibatch's distinct frames: groups int64 [U] (frame ids of the plan, ascending),
    inv int64 [n] (sample -> position in groups), slot int32 [F] (frame id -> position or -1),
    and the samples of each frame as CSR: order int32 [n] (sample positions grouped by frame,
    ascending within a frame), offs int32 [U+1] (merlin_ppo_loss sums per frame in that order)."""

    def __init__(self, groups: torch.Tensor, inv: torch.Tensor, slot, order=None, offs=None, lazy=None):
        self.groups = groups
        self._inv, self._slot, self._order, self._offs = inv, slot, order, offs
        # lazy = (F, inv_sorted, perm, starts, lo, hi, off): the tensors are derived on first use,
        # when the minibatch's step runs (update_minibatches makes all 80 of an update right after
        # its host read: derived there, their ~400 small launches would be host work with an idle GPU)
        self._lazy = lazy

    def _derive(self):
        F, inv, perm, starts, lo, hi, off = self._lazy
        g, dev = self.groups, self.groups.device
        c = g.numel()
        s = torch.full((F,), -1, dtype=torch.int32, device=dev)
        s[g] = torch.arange(c, dtype=torch.int32, device=dev)
        self._slot = s
        self._inv = inv[lo:hi] - off
        # sorted positions lo..hi hold exactly this minibatch's samples (mb_of is the major key)
        self._order = (perm[lo:hi] - lo).to(torch.int32)
        self._offs = _frame_csr(starts[off:off + c] - lo, hi - lo)
        self._lazy = None

    @property
    def slot(self) -> torch.Tensor:
        if self._lazy is not None:
            self._derive()
        return self._slot

    @property
    def inv(self) -> torch.Tensor:
        if self._lazy is not None:
            self._derive()
        return self._inv

    @property
    def order(self):
        if self._lazy is not None:
            self._derive()
        return self._order

    @property
    def offs(self):
        if self._lazy is not None:
            self._derive()
        return self._offs


def _frame_csr(starts: torch.Tensor, n: int) -> torch.Tensor:
    out = torch.empty(starts.numel() + 1, dtype=torch.int32, device=starts.device)
    out[:-1] = starts
    out[-1:].fill_(n)  # a fill kernel (indexed assignment of a Python int copies it host->device: a sync)
    return out


class WindowPlan:
    """Per-update numbering of the receptive-field windows of a rollout's distinct frames
    (frame id = merlin.dedup.FrameGroups group id) and the two backward entry lists."""

    def __init__(self, codes: torch.Tensor, frame_groups, item_len: int | None = None,
                 hist_item_len: int | None = None):
        dev = codes.device
        self.frame_groups = frame_groups
        rep = codes.index_select(0, frame_groups.rep)  # one code row per distinct frame
        F = int(rep.shape[0])
        cls = unpack_classes(rep)
        # (keys < 5**9, kid / band / window ids < 2**31: the sorts below run on int32 keys, half the
        # radix passes of int64)
        uniq, inv = torch.unique(window_keys(cls).reshape(-1).to(torch.int32), return_inverse=True)
        nw = int(uniq.numel())
        self.num_frames, self.num_windows = F, nw
        self.wid = inv.view(F, 25).to(torch.int32).contiguous()
        self.rows = window_rows(uniq).contiguous()
        assert int(self.rows.max()) < nat.LUT2_ROWS
        # dT2 lists: entry (w, tap) -> table row rows[w][tap]; source row w of dZ2w
        hk, ho = torch.sort(self.rows.reshape(-1), stable=True)
        self.hist = SegmentPlan(hk, ho // 16, hist_item_len)
        # patch lists: entry g*9 + p3 (frame g, conv3 output p3) -> its 5x5-tile patch k
        # (patch_keys: 25 base-5 digits < 5**25 < 2**63), sorted by k; source dY3 row / mask word
        # slot[g]*9 + p3 of the minibatch
        pk, kid = torch.unique(patch_keys(cls).reshape(-1), return_inverse=True)
        self.num_patches = int(pk.numel())
        self.kid = kid.view(F, 9).to(torch.int32).contiguous()
        ks, ko = torch.sort(kid.to(torch.int32), stable=True)
        self.patch_plan = SegmentPlan(ks, ko, item_len)
        # band lists: entry (patch k, ky) -> S row (k's band ky), bands numbered by (ky, band key); source R row k.
        # Band ky of a patch is its tile rows ky..ky+2, digits 5 ky .. 5 ky + 14 of the patch key: one division and
        # one remainder; the three rows' bands are numbered by one unique over (ky, band key) (one host read)
        K = self.num_patches
        B15 = 5 ** 15
        ky3 = torch.arange(3, dtype=torch.int64, device=dev)
        bkeys = ky3.unsqueeze(1) * B15 + (pk.unsqueeze(0) // (5 ** (10 - 5 * ky3)).unsqueeze(1)) % B15  # [3, K]
        ub, bid = torch.unique(bkeys.reshape(-1), return_inverse=True)
        self.num_bands = int(ub.numel())
        bk, bo = torch.sort(bid.to(torch.int32), stable=True)
        self.band_plan = SegmentPlan(bk, (bo % K), item_len)
        # dQ entries of the bands: (band j, kx) -> Q row w*9 + ky*3 + kx, w = the band's window at column kx: rows
        # r < 3 of the band (5 digits each), their columns kx..kx+2 (3 digits), numbered by searching the sorted
        # window keys
        bky, bkey = ub // B15, ub % B15
        brow = (bkey.unsqueeze(1) // (3125 ** (2 - ky3)).unsqueeze(0)) % 3125  # [nb, 3]
        jb = torch.arange(self.num_bands, dtype=torch.int64, device=dev)
        ddst, dsrc = [], []
        for kx in range(3):
            c = (brow // 5 ** (2 - kx)) % 125
            w = torch.searchsorted(uniq, ((c[:, 0] * 125 + c[:, 1]) * 125 + c[:, 2]).to(torch.int32))
            ddst.append(w * 9 + bky * 3 + kx)
            dsrc.append(jb)
        dk, do = torch.sort(torch.cat(ddst).to(torch.int32), stable=True)
        self.dq_plan = SegmentPlan(dk, torch.cat(dsrc)[do], item_len)

    def update_minibatches(self, perms: list, minibatch_size: int, bulk: bool = False) -> list:
        """epoch_minibatches for every epoch's permutation at once: one stable sort and one host
        read for the whole update (each host read drains the stream; per epoch that was ten
        pipeline drains per update).  Returns one list of MinibatchWindows per epoch."""
        B = int(perms[0].numel())
        flat = self.epoch_minibatches(torch.cat(perms), minibatch_size, period=B, bulk=bulk)
        nmb = (B + minibatch_size - 1) // minibatch_size
        return [flat[e * nmb:(e + 1) * nmb] for e in range(len(perms))]

    def _bulk_minibatches(self, uniq, inv, perm, starts, mb_of, counts, P, per, minibatch_size) -> list:
        """Every minibatch's MinibatchWindows tensors for the whole update in a few launches (merlin/fast_step.py:
        the minibatch step then issues none of its own): each minibatch's slot / inv / order / offs and its live
        patch map kmap are views of update-wide arrays (slot [nmb, F] and kmap [nmb, K] int32)."""
        dev, F, K = uniq.device, self.num_frames, self.num_patches
        nmb, G = len(counts), int(uniq.numel())
        goff_h = [0]
        for c in counts:
            goff_h.append(goff_h[-1] + c)
        lo_h = [(m // per) * P + (m % per) * minibatch_size for m in range(nmb)]
        hi_h = [(m // per) * P + min(P, (m % per + 1) * minibatch_size) for m in range(nmb)]
        goff = torch.tensor(goff_h, dtype=torch.int64).to(dev, non_blocking=True)
        lo = torch.tensor(lo_h, dtype=torch.int64).to(dev, non_blocking=True)
        span = torch.tensor([h - l for h, l in zip(hi_h, lo_h)], dtype=torch.int32).to(dev, non_blocking=True)
        mbg = uniq // F  # minibatch of each (minibatch, frame) group
        gall = uniq - mbg * F
        j = torch.arange(G, device=dev) - goff[mbg]  # position of the group in its minibatch
        slot = torch.full((nmb, F), -1, dtype=torch.int32, device=dev)
        slot.view(-1)[mbg * F + gall] = j.to(torch.int32)
        inv_local = inv - goff[mb_of]
        # sorted positions lo..hi hold exactly minibatch m's samples: order = position - lo of its minibatch
        order = ((perm % P) % minibatch_size).to(torch.int32)
        offs = torch.empty(G + nmb, dtype=torch.int32, device=dev)
        offs[torch.arange(G, device=dev) + mbg] = (starts - lo[mbg]).to(torch.int32)
        offs[goff[1:] + torch.arange(nmb, device=dev)] = span
        # the live-patch maps kmap [nmb, K] (the S pass's slot maps) and conv3's patch reuse rows rep_row [G * 9]
        # (merlin_tower_window_conv3_reuse: per row j*9 + p3 of its minibatch, one row of the minibatch holding the
        # same patch -- which one wins does not matter, they compute the same bits): two launches over the G * 9
        # (group, position)s (merlin_minibatch_patch_maps; the torch scatter / gather chain took ~3.6 ms per update)
        kmap, rep_row = nat.minibatch_patch_maps(self.kid, uniq, F, goff, nmb, K)
        # bench timing only: representative rows per minibatch = its distinct patches (the k_window_conv3 span's
        # algorithmic bytes; one reduction per update, read back after the timed region)
        n_reps = (kmap >= 0).sum(dim=1) if nat.KernelTimer.active() else None
        out = []
        for m, c in enumerate(counts):
            g0 = goff_h[m]
            mw = MinibatchWindows(gall[g0:g0 + c], inv_local[lo_h[m]:hi_h[m]], slot[m], order[lo_h[m]:hi_h[m]],
                                  offs[g0 + m:g0 + m + c + 1])
            mw.kmap = kmap[m]
            mw.rep_row = rep_row[g0 * 9:(g0 + c) * 9]
            mw.n_reps = n_reps[m] if n_reps is not None else None
            out.append(mw)
        return out

    def epoch_minibatches(self, idxs: torch.Tensor, minibatch_size: int, period: int | None = None,
                          bulk: bool = False) -> list:
        """MinibatchWindows of every minibatch idxs[k*mb:(k+1)*mb] of one epoch's permutation,
        grouped by one stable sort and one host read for the whole epoch (a torch.unique per
        minibatch would stall the host at every optimizer step).  Same groups as minibatch().
        period: idxs holds several epochs' permutations of that length back to back, each cut
        into minibatches on its own (update_minibatches)."""
        dev, B, F = idxs.device, int(idxs.numel()), self.num_frames
        P = B if period is None else int(period)
        per = (P + minibatch_size - 1) // minibatch_size
        nmb = (B // P) * per
        pos = torch.arange(B, device=dev)
        mb_of = (pos // P) * per + (pos % P) // minibatch_size
        key = mb_of * F + self.frame_groups.uid[idxs]
        if nmb * F < 2 ** 31:  # int32 radix sort: half the passes
            key = key.to(torch.int32)
        sk, perm = torch.sort(key, stable=True)
        new = torch.ones(B, dtype=torch.bool, device=dev)
        new[1:] = sk[1:] != sk[:-1]
        inv = torch.empty(B, dtype=torch.int64, device=dev)
        inv[perm] = torch.cumsum(new, 0) - 1
        starts = torch.nonzero(new).squeeze(1)  # first sorted position of each (minibatch, frame)
        uniq = sk[starts].long()
        counts = torch.bincount(uniq // F, minlength=nmb).tolist()
        if bulk:
            return self._bulk_minibatches(uniq, inv, perm, starts, mb_of, counts, P, per, minibatch_size)
        out, off = [], 0
        gall = uniq % F  # frame ids; each minibatch's groups are a view of it
        for m, c in enumerate(counts):
            e, k = divmod(m, per)
            lo, hi = e * P + k * minibatch_size, e * P + min(P, (k + 1) * minibatch_size)
            out.append(MinibatchWindows(gall[off:off + c], None, None, lazy=(F, inv, perm, starts, lo, hi, off)))
            off += c
        return out

    def minibatch(self, mb_idx: torch.Tensor) -> MinibatchWindows:
        n = int(mb_idx.numel())
        sk, perm = torch.sort(self.frame_groups.uid[mb_idx], stable=True)
        new = torch.ones(n, dtype=torch.bool, device=mb_idx.device)
        new[1:] = sk[1:] != sk[:-1]
        starts = torch.nonzero(new).squeeze(1)
        g = sk[starts]
        inv = torch.empty(n, dtype=torch.int64, device=mb_idx.device)
        inv[perm] = torch.cumsum(new, 0) - 1
        slot = torch.full((self.num_frames,), -1, dtype=torch.int32, device=g.device)
        slot[g] = torch.arange(g.numel(), dtype=torch.int32, device=g.device)
        return MinibatchWindows(g, inv, slot, perm.to(torch.int32), _frame_csr(starts, n))


class _WindowConv2(torch.autograd.Function):
    """Z2w [2, windows, 64] = conv2(relu(conv1)) of every window (no conv2 bias) from the tables
    ([2, nw_pad, 64] with zero rows past the windows when the window GEMMs are padded to a tuned
    shape, merlin/gemm_tuning.py)."""

    @staticmethod
    def forward(ctx, T2, plan, nw_pad):
        ctx.plan = plan
        Z = nat.window_lut(plan.rows, T2.detach().contiguous())
        if nw_pad > Z.shape[1]:
            Zp = Z.new_zeros((Z.shape[0], nw_pad, 64))
            Zp[:, :Z.shape[1]] = Z
            Z = Zp
        return Z

    @staticmethod
    def backward(ctx, dZ2w):
        dT2 = nat.segment_sum(dZ2w.contiguous(), ctx.plan.hist, nat.LUT2_ROWS, name="k_seg_sum_dT2")
        return dT2, None, None


def _colsum(x):
    """x [T, n, C] (rows may be strided) -> [T, C] column sums (merlin_tower_colsum: one pass, fixed
    order; torch's dim-1 reduce over these [2, ~6.5k, 64] shapes took ~50 us, a ones-row GEMM ~32)."""
    return nat.colsum(x)


class _BiasRelu(torch.autograd.Function):
    """relu(Z + b[:, None]) for Z [T, n, C], b [T, C]; backward: the ReLU mask and the bias gradient in
    one HIP pass (merlin_tower_relu_bwd)."""

    @staticmethod
    def forward(ctx, Z, b):
        A = torch.relu(Z + b.unsqueeze(1))
        ctx.save_for_backward(A)
        return A

    @staticmethod
    def backward(ctx, dA):
        (A,) = ctx.saved_tensors
        return nat.relu_bwd(A, dA.contiguous())


class _TunedBmm(torch.autograd.Function):
    """A @ B (batched) with the forward and both backward GEMMs on the pre-tuned solutions
    (merlin/gemm_tuning.py; autograd's own bmm backward would run outside tuned())."""

    @staticmethod
    def forward(ctx, A, B):
        from .gemm_tuning import tuned

        ctx.save_for_backward(A, B)
        with tuned("window"):
            return torch.bmm(A, B)

    @staticmethod
    def backward(ctx, dC):
        from .gemm_tuning import tuned

        A, B = ctx.saved_tensors
        dC = dC.contiguous()
        with tuned("window"):
            dA = torch.bmm(dC, B.transpose(1, 2)) if ctx.needs_input_grad[0] else None
            dB = torch.bmm(A.transpose(1, 2), dC) if ctx.needs_input_grad[1] else None
        return dA, dB


class _WindowGemm(torch.autograd.Function):
    """Q = a2w @ W3r over both towers (a2w [T, windows, 64], W3r [T, 64, 576]); backward da2w = dQ W3r^T
    and dW3r = a2w^T dQ, the latter split over 256-window chunks: its output is only 64 x 576 per tower,
    so hipBLASLt's plain form runs ~36 workgroups over the ~6.6k-deep reduction (280 us per minibatch in
    profiles/r03a_step_sequence.md, on the critical path); the split form fills the chip."""

    @staticmethod
    def forward(ctx, a2w, W3r):
        ctx.save_for_backward(a2w, W3r)
        return torch.bmm(a2w, W3r)

    @staticmethod
    def backward(ctx, dQ):
        from .actor_critic import _splitk_bmm_tn

        a2w, W3r = ctx.saved_tensors
        dQ = dQ.contiguous()
        da2w = torch.bmm(dQ, W3r.transpose(1, 2)) if ctx.needs_input_grad[0] else None
        chunks = max(1, a2w.shape[1] // 256)
        dW3r = _splitk_bmm_tn(a2w, dQ, chunks, min_chunk=128, name="gemm_window_wgrad") if ctx.needs_input_grad[1] \
            else None
        return da2w, dW3r


class _WindowConv3(torch.autograd.Function):
    """Y3 [2, U*9, 64] = relu(conv3) rows (u, p3) of the minibatch's distinct frames, from Q."""

    @staticmethod
    def forward(ctx, Q, b3, plan, mb, rows):
        Y3, bits = nat.window_conv3(Q.detach().contiguous(), plan.wid, mb.groups, b3.detach().contiguous(), bits=True,
                                    rows=rows)
        ctx.save_for_backward(bits)
        ctx.nw_q = Q.shape[1]
        ctx.plan, ctx.mb = plan, mb
        return Y3

    @staticmethod
    def backward(ctx, dY3):
        (bits,) = ctx.saved_tensors
        dQ, db3 = _conv3_backward(ctx.plan, ctx.mb, bits, dY3, ctx.nw_q)
        return dQ, db3, None, None, None


def _conv3_backward(plan, mb, bits, dY3, nw):
    """(dQ [T, nw, 576], db3 [T, 64]) from dY3 [T, U*9, 64] (conv3's output gradient) and the ReLU bit
    words of the forward: the patch -> band -> window segmented sums of the module docstring."""
    T = bits.shape[0]
    # pass 1: per-patch sums of the ReLU-masked dY3 rows of this minibatch's frames (rows of
    # patches absent from the minibatch are left unwritten and skipped below)
    R = nat.segment_sum(dY3.contiguous(), plan.patch_plan, plan.num_patches, slot=mb.slot, sub=9,
                        name="k_seg_sum_R", mask=bits, fill=False)
    live = plan.kid.index_select(0, mb.groups).reshape(-1)
    kmap = torch.full((plan.num_patches,), -1, dtype=torch.int32, device=bits.device)
    kmap[live] = live
    # pass 2: band sums over the live patches, marking the bands that got one; pass 3: dQ[w][tap] from the
    # marked bands (the others hold no sum and are neither zeroed nor read)
    bslot = torch.full((plan.num_bands,), -1, dtype=torch.int32, device=bits.device)
    S = nat.segment_sum(R, plan.band_plan, plan.num_bands, slot=kmap, sub=1, name="k_seg_sum_S", fill=False,
                        mark=bslot)
    dQ = nat.segment_sum(S, plan.dq_plan, nw * 9, slot=bslot, sub=1, name="k_seg_sum_dQ")
    dQ = dQ.view(T, nw, 9, 64)
    db3 = _colsum(dQ[:, :, 0])
    return dQ.view(T, nw, 576), db3


# fc1's weight gradient on a side stream, overlapped with conv3's backward segmented sums: True =
# joined before the window Function returns; "deferred" = delivered to the fc1 weights only at the
# end of the backward pass (autograd-engine callback), so it also overlaps the window GEMMs and the
# conv tables.  scripts/ab_update.py, one update replayed per setting: 300.6 (off) / 297.0 (True) /
# 293.4 (deferred) ms per update.
OVERLAP_WGRAD = "deferred"
_SIDE = {}
# The deferred delivery writes .grad of the fc1 weights itself, around autograd: it is only right for a
# caller that runs loss.backward() and reads p.grad (PPO._sgd).  Everyone else (torch.autograd.grad,
# backward(inputs=...), grad hooks) gets the joined side-stream mode, which returns dW4p through
# autograd.  PPO._sgd opts in with `with deferred_fc1_wgrad():` around its forward.
_DEFER = threading.local()


@contextlib.contextmanager
def deferred_fc1_wgrad(enabled: bool = True):
    prev = getattr(_DEFER, "on", False)
    _DEFER.on = bool(enabled)
    try:
        yield
    finally:
        _DEFER.on = prev


def _defer_active() -> bool:
    return OVERLAP_WGRAD == "deferred" and getattr(_DEFER, "on", False)


def _side_stream(device):
    if torch.cuda.is_current_stream_capturing():
        return None
    st = _SIDE.get(device)
    if st is None:
        st = _SIDE[device] = torch.cuda.Stream(device=device)
    return st


class _Fc1:
    """fc1's three GEMMs on the matrix cores: impl "h3" (two f16 planes per value, per-tower scales from max |x|,
    csrc/merlin_h3.hip) or "x6" (three bf16 planes, csrc/merlin_gemm.hip / merlin_gemm2.hip)."""

    def __init__(self, impl, W4p):
        self.impl = impl
        W = W4p.detach().contiguous()
        Wt = W.transpose(1, 2).contiguous()
        if impl == "h3":
            self.amW = nat.h3_amax(W)  # W4p^T holds the same values: one scale for both
            self.P, self.Pt = nat.h3_split(W, self.amW), nat.h3_split(Wt, self.amW)
        else:
            self.P, self.Pt = nat.x6_split(W), nat.x6_split(Wt)

    def fwd(self, a3, b4, am3=None):
        if self.impl == "h3":
            return nat.h3_gemm_nt(a3, am3, self.P, self.amW, bias=b4, cfg=nat.H3_NT_CFG["fwd"], name="gemm_fc1_fwd")
        return nat.x6_gemm_nt(a3, self.P, bias=b4, cfg=nat.X6_NT_CFG["fwd"], name="gemm_fc1_fwd")

    def dgrad(self, dz, amz=None):
        if self.impl == "h3":
            return nat.h3_gemm_nt(dz, amz, self.Pt, self.amW, cfg=nat.H3_NT_CFG["dgrad"], name="gemm_fc1_dgrad")
        return nat.x6_gemm_nt(dz, self.Pt, cfg=nat.X6_NT_CFG["dgrad"], name="gemm_fc1_dgrad")

    def wgrad(self, dz, a3, amz=None, am3=None, out=None):
        if self.impl == "h3":
            return nat.h3_gemm_tn(dz, amz, a3, am3, name="gemm_wgrad", out=out)
        return nat.x6_gemm_tn(dz, a3, name="gemm_wgrad", out=out)


class _WindowTowerHeadX6(torch.autograd.Function):
    """conv3 -> fc1 -> ReLU -> heads of both towers for the minibatch's distinct frames, with fc1's
    three GEMMs on the matrix cores (_Fc1: f16 two-plane form by default, csrc/merlin_h3.hip, or the exact
    bf16 three-plane form, csrc/merlin_gemm.hip):
      forward   a3 = relu(conv3) from Q (k_window_conv3, with the ReLU bit words), h = relu(a3 W4p^T +
                b4) (merlin_x6_gemm_nt, bias + ReLU epilogue), logits = h0 Wa^T (+ ba), value = h1 wc
                (+ bc)   (src/actor_critic.py:13-14, 31-41)
      backward  the heads' backward through fc1's ReLU (k_head_bwd), da3 = dz W4p (x6 NT against the
                planes of W4p^T), dW4p = dz^T a3 (x6 TN, split-K), then conv3's backward through the
                patch / band / window sums (_conv3_backward).
    fp32 products throughout (the activations are split into planes inside the GEMMs)."""

    @staticmethod
    def forward(ctx, Q, b3, W4p, b4, Wa, ba, Wc, bc, plan, mb, fc1_weights=None, impl="x6"):
        am = torch.zeros(4, dtype=torch.int32, device=Q.device) if impl == "h3" else None  # max |a3|, max |dz|
        Y3, bits = nat.window_conv3(Q.detach().contiguous(), plan.wid, mb.groups, b3.detach().contiguous(), bits=True,
                                    amax=am[0:2] if am is not None else None)
        n = int(mb.groups.numel())
        a3 = Y3.view(2, n, 576)
        fc1 = _Fc1(impl, W4p)
        if impl == "h3" and nat.H3_HEADS_EPILOGUE and nat.lib().merlin_h3_heads_parts(W4p.shape[1],
                                                                                        nat.H3_NT_CFG["fwd"]) > 0:
            # both heads in the forward GEMM's epilogue (merlin_h3_gemm_nt_heads), biases added after the sums
            h, logits, value = nat.h3_gemm_nt_heads(a3, am[0:2], fc1.P, fc1.amW, b4.detach().contiguous(),
                                                    Wa.detach().contiguous(), Wc.detach().contiguous(),
                                                    cfg=nat.H3_NT_CFG["fwd"], name="gemm_fc1_fwd")
            if ba is not None:
                logits = logits + ba.detach()
            if bc is not None:
                value = value + bc.detach()
        else:
            h = fc1.fwd(a3, b4.detach(), am[0:2] if am is not None else None)
            logits, value = nat.heads_fwd(h, Wa, Wc, ba, bc)  # both heads in one pass over h
        ctx.save_for_backward(a3, bits, W4p, h, Wa, Wc)
        ctx.fc1, ctx.am = fc1, am
        ctx.head_bias = (ba is not None, bc is not None)
        ctx.plan, ctx.mb, ctx.nw_q = plan, mb, Q.shape[1]
        ctx.fc1_weights = fc1_weights  # (actor, critic) fc1 weights W4p was stacked from (deferred mode)
        return logits, value

    @staticmethod
    def backward(ctx, dlogits, dvalue):
        a3, bits, W4p, h, Wa, Wc = ctx.saved_tensors
        n = h.shape[1]
        dlogits = h.new_zeros(n, Wa.shape[0]) if dlogits is None else dlogits.contiguous()
        dvalue = h.new_zeros(n) if dvalue is None else dvalue.contiguous()
        fc1, am = ctx.fc1, ctx.am
        amz, am3 = (am[2:4], am[0:2]) if am is not None else (None, None)
        dz, db4, dWa, dWc = nat.head_bwd(h, dlogits, dvalue, Wa.detach().contiguous(), Wc.detach().contiguous(),
                                         amax=amz)
        da3 = fc1.dgrad(dz, amz)
        side = _side_stream(dz.device) if OVERLAP_WGRAD else None
        if side is None:
            dW4p = fc1.wgrad(dz, a3, amz, am3)
        else:
            # the weight gradient (matrix-core bound, one 120-KB-LDS block per CU) on a second stream,
            # beside conv3's memory-bound patch / band / window sums on this one (no LDS: their waves
            # fit next to the GEMM's on each CU); joined before the gradients are handed back
            main = torch.cuda.current_stream(dz.device)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                dW4p = fc1.wgrad(dz, a3, amz, am3)
            dz.record_stream(side)
            a3.record_stream(side)
            if am is not None:
                am.record_stream(side)
            dW4p.record_stream(main)
        dQ, db3 = _conv3_backward(ctx.plan, ctx.mb, bits, da3.view(2, n * 9, 64), ctx.nw_q)
        dba = dlogits.sum(0) if ctx.head_bias[0] else None
        dbc = dvalue.sum(0, keepdim=True) if ctx.head_bias[1] else None
        if side is not None and OVERLAP_WGRAD == "deferred" and ctx.fc1_weights is not None:
            # deliver fc1's weight gradient only at the end of the backward pass (autograd-engine
            # callback), so the side stream also runs beside the window GEMMs and the conv tables
            weights, H = ctx.fc1_weights, dW4p.shape[1]
            g = dW4p

            def finish():
                torch.cuda.current_stream(g.device).wait_stream(side)
                dW4 = g.view(2, H, 9, 64).transpose(2, 3).reshape(2, H, 576)  # (p3, co) -> (co, p3)
                for t, w in enumerate(weights):
                    if w.grad is None:
                        w.grad = dW4[t].contiguous()
                    else:
                        w.grad.add_(dW4[t])

            torch.autograd.Variable._execution_engine.queue_callback(finish)
            dW4p = None
        elif side is not None:
            torch.cuda.current_stream(dz.device).wait_stream(side)
        return dQ, db3, dW4p, db4, dWa, dba, dWc.view_as(Wc), dbc, None, None, None, None

def tower_conv3(ac, plan: WindowPlan, mb: MinibatchWindows, rows: int | None = None) -> torch.Tensor:
    """relu(conv3(relu(conv2(relu(conv1(frame)))))) of both towers of CNNActorCritic `ac` for the
    minibatch's distinct frames: [2, U*9, 64], rows (u, p3), channels last ([2, rows*9, 64] with
    zero rows past U when rows is given)."""
    from .gemm_tuning import padded_windows

    ea, ec = ac.actor_extractor.network, ac.critic_extractor.network
    Z2w = _WindowConv2.apply(ac.conv2_tables(), plan, padded_windows(plan.num_windows))
    a2w = _BiasRelu.apply(Z2w, torch.stack([ea[2].bias, ec[2].bias]))
    W3 = torch.stack([ea[4].weight, ec[4].weight])  # [2, co, ci, ky, kx]
    Q = _TunedBmm.apply(a2w, W3.permute(0, 2, 3, 4, 1).reshape(2, 64, 576))  # [2, windows, (ky, kx, co)]
    return _WindowConv3.apply(Q, torch.stack([ea[4].bias, ec[4].bias]), plan, mb, rows)


def window_tower_head_x6(ac, plan: WindowPlan, mb: MinibatchWindows, head_bias: bool = True):
    """(logits [U, act_dim], value [U]) of the minibatch's distinct frames: conv2 / conv3 through
    the windows, fc1 on the matrix cores (_WindowTowerHeadX6, ac.fc1_impl "h3" or "x6").  The
    window GEMMs take PyTorch's default hipBLASLt path (no TunableOp: merlin/gemm_tuning.py)."""
    ea, ec = ac.actor_extractor.network, ac.critic_extractor.network
    Z2w = _WindowConv2.apply(ac.conv2_tables(), plan, plan.num_windows)
    a2w = _BiasRelu.apply(Z2w, torch.stack([ea[2].bias, ec[2].bias]))
    W3 = torch.stack([ea[4].weight, ec[4].weight])  # [2, co, ci, ky, kx]
    Q = _WindowGemm.apply(a2w, W3.permute(0, 2, 3, 4, 1).reshape(2, 64, 576))  # [2, windows, (ky, kx, co)]
    fa, fc = ac.actor[0], ac.critic[0]
    W4 = torch.stack([fa.weight, fc.weight])  # [2, hidden, 576] in (co, p3) order
    W4p = W4.view(2, W4.shape[1], 64, 9).transpose(2, 3).reshape(2, W4.shape[1], 576)
    ba, bc = (ac.actor[2].bias, ac.critic[2].bias) if head_bias else (None, None)
    # deferred fc1 weight gradient only for a caller that opted in (deferred_fc1_wgrad) and only when
    # both weights take plain .grad accumulation
    defer = _defer_active() and fa.weight.requires_grad and fc.weight.requires_grad and torch.is_grad_enabled()
    return _WindowTowerHeadX6.apply(Q, torch.stack([ea[4].bias, ec[4].bias]), W4p, torch.stack([fa.bias, fc.bias]),
                                    ac.actor[2].weight, ba, ac.critic[2].weight, bc, plan, mb,
                                    (fa.weight, fc.weight) if defer else None, ac.fc1_impl)
