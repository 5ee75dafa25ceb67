"""PPO.update's minibatch step on the window path (fc1 on the h3 or x6 GEMMs) with the launch sequence written out
(src/ppo.py:136-156: forward, loss, backward, clip_grad_norm_(0.5), Adam).

The autograd engine walked ~95 kernels per optimizer step, ~60 of them small torch ops, and the host
needed ~2 ms per step to queue them: at the bench state the GPU sat idle for ~20 % of every update
waiting for the host (scripts/busy_union.py on a rocprofv3 kernel trace: 67-75 ms of ~300-365 ms).
Here the step is the same kernels with the same operands in the same order, issued directly:

  * WeightStage -- everything that depends on the parameters alone (the conv1 / conv2 tables T2,
    the stacked and permuted conv3 / fc1 weights, fc1's weight planes (and their scale) for the forward and the
    input gradient) is one captured HIP graph, and the backward of that subgraph (the table / stacking
    adjoints down to every parameter's gradient, written into a flat gradient buffer) a second one.
    Parameters keep their storage for the whole run (the optimizer updates them in place), so the
    graphs replay on live weights.
  * the per-minibatch bookkeeping (slot / inv / order / offs / live-patch maps) comes as views of
    update-wide arrays (WindowPlan.update_minibatches(bulk=True)): no launches of its own.
  * the data-dependent part (window tables, conv3, fc1, heads, loss, their backward passes, conv3's
    segmented sums) calls the same library entry points as merlin/windows.py's autograd Functions,
    writing the gradients the stage's backward graph consumes straight into its input buffers.

Same arithmetic as the autograd path (tests/test_gpu_fast_step.py compares a whole update bit for bit).
"""
from __future__ import annotations

import weakref

import torch

from . import _native as nat
from .actor_critic import _splitk_bmm_tn


def flatten_parameters(module: torch.nn.Module) -> torch.Tensor:
    """Re-home every parameter of `module` into one contiguous buffer (parameter order), each parameter a view of
    it: the weight stage gathers all its derived weights with one indexed read, and the optimizer / all-reduce see
    one block.  Values are unchanged; call before anything captures parameter addresses (the rollout graph)."""
    params = list(module.parameters())
    flat = torch.empty(sum(p.numel() for p in params), dtype=params[0].dtype, device=params[0].device)
    off = 0
    with torch.no_grad():
        for p in params:
            n = p.numel()
            v = flat[off:off + n].view_as(p)
            v.copy_(p.data)
            p.data = v
            off += n
    return flat


class WeightStage:
    """Parameter-only forward / backward of the minibatch step as two captured HIP graphs.

    The derived weights are one indexed read of the flat parameter buffer, laid out as D = [W1 [2, 32, 3, 8, 8],
    b1 [2, 32], W2 [2, 64, 32, 4, 4], b2 [2, 64], W3r [2, 64, 576], b3 [2, 64], b4 [2, H], W4p [2, H, 576],
    W4p^T [2, 576, H]] (the towers stacked, conv3's and fc1's weights in the (ky, kx, co) / (p3, co) orders the
    window kernels read); then T2 from (W1, b1, W2) (CNNActorCritic.conv2_tables_from) and fc1's x6 planes of W4p
    and W4p^T in one split.  forward() -> (T2, b2, W3r, b3, W4p, b4); self.planes = (planes of W4p, of W4p^T).
    The backward graph maps dT2 (self.gT2) through the table adjoints to dW1 / db1 / dW2, puts them beside the
    gradients the step wrote into self.grads (db2, dW3r, db3, dW4p, db4: views of the derived-gradient buffer),
    and scatters the whole buffer onto the stage parameters' slots of the flat gradient (one launch)."""

    def __init__(self, ac, flat_params: torch.Tensor, flat_grad: torch.Tensor, impl: str = "hip", fc1: str = "h3"):
        self.ac = ac
        # fc1's GEMM form: "h3" (f16 two-plane; the weight planes' per-tower scale amaxW is computed by this graph,
        # the activations' by the step's producer kernels, merlin.fast_step.WindowStep.step) or "x6" (bf16
        # three-plane)
        self.fc1 = fc1
        # "hip": T2 and its adjoint by csrc/merlin_stage.hip (2 launches each way); "torch": the same tables by
        # CNNActorCritic.conv2_tables_from and autograd (the autograd path's exact arithmetic)
        self.impl = impl
        self.flat_params, self.flat_grad = flat_params, flat_grad
        self.ptr = flat_params.data_ptr()
        ea, ec = ac.actor_extractor.network, ac.critic_extractor.network
        fa, fc = ac.actor[0], ac.critic[0]
        H = fa.weight.shape[0]
        # the flat parameter offsets, as index tensors shaped like the parameters
        idx, off = {}, 0
        for p in ac.parameters():
            n = p.numel()
            idx[p] = torch.arange(off, off + n, dtype=torch.int64).view(p.shape)
            off += n
        st = lambda a, b: torch.stack([idx[a], idx[b]])  # noqa: E731
        W4 = st(fa.weight, fc.weight)  # [2, H, 576] in (co, p3) order
        W4p = W4.view(2, H, 64, 9).transpose(2, 3).reshape(2, H, 576)
        segs = [("W1", st(ea[0].weight, ec[0].weight)), ("b1", st(ea[0].bias, ec[0].bias)),
                ("W2", st(ea[2].weight, ec[2].weight)), ("b2", st(ea[2].bias, ec[2].bias)),
                ("W3r", st(ea[4].weight, ec[4].weight).permute(0, 2, 3, 4, 1).reshape(2, 64, 576)),
                ("b3", st(ea[4].bias, ec[4].bias)), ("b4", st(fa.bias, fc.bias)), ("W4p", W4p),
                ("W4pT", W4p.transpose(1, 2).contiguous())]
        W3r = segs[4][1]
        segs.append(("W3rT", W3r.transpose(1, 2).contiguous()))  # [2, 576, 64]: the window GEMM's B rows
        self.shapes, self.offs, o = {}, {}, 0
        for name, t in segs:
            self.shapes[name], self.offs[name] = tuple(t.shape), o
            o += t.numel()
        dev = flat_params.device
        self.amaxW = torch.zeros(2, dtype=torch.int32, device=dev)
        self.amaxW3 = torch.zeros(2, dtype=torch.int32, device=dev)
        self.fwd_map = torch.cat([t.reshape(-1) for _, t in segs]).to(dev)
        self.n_grad = self.offs["W4pT"]  # every stage-parameter element once in D[:n_grad]
        assert int(self.fwd_map[:self.n_grad].unique().numel()) == self.n_grad
        self._capture()

    def seg(self, buf, name):
        o = self.offs[name]
        shape = self.shapes[name]
        n = 1
        for d in shape:
            n *= d
        return buf[o:o + n].view(shape)

    def _fwd(self):
        D = self.flat_params.index_select(0, self.fwd_map)  # every derived weight in one launch
        if self.impl == "hip":
            W1, b1, W2 = (self.seg(D, k) for k in ("W1", "b1", "W2"))
            HT, T2 = nat.stage_tables_fwd(W1, b1, W2, *self.ac.stage_consts(D.device)[:2])
            leaves = (W2, HT)
        else:
            leaves = W1, b1, W2 = tuple(self.seg(D, k).requires_grad_() for k in ("W1", "b1", "W2"))
            T2 = self.ac.conv2_tables_from(W1, b1, W2)
        o = self.offs["W4p"]
        H = self.shapes["W4p"][1]
        if self.fc1 == "h3":
            W4p, W4pT = self.seg(D, "W4p"), self.seg(D, "W4pT")
            nat.h3_amax(W4p, out=self.amaxW)  # W4p^T holds the same values: one scale for both
            planes = (nat.h3_split(W4p, self.amaxW), nat.h3_split(W4pT, self.amaxW))
            if WINDOW_H3:  # conv3's weights for the window GEMMs: W3r^T (forward), W3r (input gradient)
                W3r, W3rT = self.seg(D, "W3r"), self.seg(D, "W3rT")
                nat.h3_amax(W3r, out=self.amaxW3)
                planes += (nat.h3_split(W3rT, self.amaxW3), nat.h3_split(W3r, self.amaxW3))
            return D, leaves, T2, planes
        planes = nat.x6_split(D[o:self.offs["W3rT"]].view(-1, 8)).view(-1)  # W4p and W4p^T back to back
        n4 = 2 * H * 576 * 3
        return D, leaves, T2, (planes[:n4].view(2, H, 3 * 576), planes[n4:].view(2, 576, 3 * H))

    def _capture(self):
        main = torch.cuda.current_stream()
        side = torch.cuda.Stream()
        side.wait_stream(main)
        hip = self.impl == "hip"
        with torch.cuda.stream(side), torch.enable_grad():
            for _ in range(2):  # lazy initialisation (GEMM handles, cached gather matrices) outside the captures
                _, leaves, T2, _ = self._fwd()
                if not hip:
                    torch.autograd.grad(T2, leaves, grad_outputs=torch.ones_like(T2))
        main.wait_stream(side)
        torch.cuda.synchronize()
        self.pool = torch.cuda.graph_pool_handle()
        self.gfwd, self.gbwd = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        DG = torch.zeros(self.fwd_map.numel(), dtype=torch.float32, device=self.flat_params.device)
        self.gT2 = torch.zeros((2, nat.LUT2_ROWS, 64), dtype=torch.float32, device=DG.device)
        self._dH = torch.empty((2, 680, 32), dtype=torch.float32, device=DG.device)  # scratch of the HIP adjoint
        with torch.enable_grad(), nat.capture_guard():  # no GC finalisers inside the captures
            with torch.cuda.graph(self.gfwd, pool=self.pool):
                D, leaves, T2, planes = self._fwd()
            with torch.cuda.graph(self.gbwd, pool=self.pool):
                if hip:
                    gs = None
                    W2, HT = leaves
                    atlas, _, koff, kv = self.ac.stage_consts(DG.device)
                    nat.stage_tables_bwd(W2, HT, self.gT2, atlas, koff, kv, dW1=self.seg(DG, "W1"),
                                         db1=self.seg(DG, "b1"), dW2=self.seg(DG, "W2"), dH=self._dH)
                else:
                    gs = torch.autograd.grad(T2, leaves, grad_outputs=self.gT2, retain_graph=True)
                    for g, k in zip(gs, ("W1", "b1", "W2")):
                        self.seg(DG, k).copy_(g)
                self.flat_grad.index_copy_(0, self.fwd_map[:self.n_grad], DG[:self.n_grad])
        self._keep = (D, leaves, T2, gs)  # the saved tensors the backward graph reads stay allocated
        self.outs = (T2.detach(),) + tuple(self.seg(D, k) for k in ("b2", "W3r", "b3", "W4p", "b4"))
        self.planes = planes
        # the gradients the step writes for the backward graph: dT2, then views of DG
        self.grads = (self.gT2,) + tuple(self.seg(DG, k) for k in ("b2", "W3r", "b3", "W4p", "b4"))
        self.DG = DG
        torch.cuda.synchronize()

    def valid(self) -> bool:
        return self.flat_params.data_ptr() == self.ptr

    def forward(self):
        self.gfwd.replay()
        return self.outs

    def backward(self):
        self.gbwd.replay()


# fc1's weight gradient on the side stream from right after the heads' backward (True: beside the input gradient
# too) or from after the input gradient (False: beside conv3's segmented sums only)
WGRAD_EARLY = False
# the weight gradient on a side stream beside conv3's backward sums (True), or on the main stream after the input
# gradient (False, round 6): the LDS-DMA kernel's blocks hold a CU whole, so the two only time-share the chip, and
# serial was as fast or faster (scripts/ab_update.py 3 5 fast,fast_wgradmain: 167.1 vs 168.7 ms per update,
# profiles/r06a_ab.log; a CU-masked side stream was far slower, 229-388 ms) -- and each kernel's time is its own
WGRAD_SIDE = False
SIDE_PRIORITY = 0  # the side stream's priority (torch.cuda.Stream priority: lower = higher priority)
# the side stream restricted to this many of every 4 groups of 8 compute units (0: all CUs).  The LDS-DMA weight
# gradient's blocks hold a CU's LDS and registers whole, so beside it conv3's backward sums only get the CUs its
# retiring blocks free; a CU mask keeps the other groups for them
SIDE_CU_GROUPS = 0
# < 0: the step's main-stream kernels on a stream of that (higher) priority, so that conv3's backward chain gets CUs
# ahead of the side-stream weight gradient.  Off: on the high-priority queue every small kernel took 4-6x longer
# (k_zero_fill 44 vs 8 us, k_colsum 50 vs 7), 286 vs 168 ms per update (profiles/r05n_fast_mainhi_timeline.txt)
MAIN_PRIORITY = 0
# h3: the window GEMMs (conv3's Q = a2w W3r and its two backward products, ~6.6k rows) on the f16 two-plane kernels
# too (False: hipBLASLt's fp32 GEMMs, the split-K weight gradient and its torch sum).  Off: with their operand scales
# (two reductions per step) they measured 200.8 vs 199.5 ms per update (scripts/ab_update.py 4 6 fast,fast_nowh3,
# weight stage captured with the planes either way)
WINDOW_H3 = False
# the window GEMM (Q = a2w W3r, merlin_window_gemm_fwd) and its backward (da2w with conv2's ReLU mask and db2, dW3r,
# merlin_window_gemm_bwd) on exact-f32 MFMA kernels, the backward in one launch + a fold (False: hipBLASLt's GEMMs,
# the split-K weight gradient and its torch sum, the ReLU backward: 137.6 us standalone at the bench's 6,571 windows,
# scripts/probe_window_bwd.py)
WINDOW_BWD_HIP = True
# h3: the weight gradient over the planes the NT GEMMs left (False: it splits a3, dz itself).  Off: the planes cost the
# forward 60-100 us of writes (a3: 2 x U x 576 x 4 B) for 50 us saved in the weight gradient (scripts/probe_h3.py)
WGRAD_PLANES = False
# h3: the weight gradient's operand planes made by k_h3_split on the side stream, beside the forward and
# input-gradient GEMMs (which do not store them), so the weight gradient runs on planes (merlin_h3_gemm_tn_planes).
# Off: the splits take the GEMMs' CUs (scripts/ab_update.py 4 6 fast,fast_nosplit: 218.7 vs 189.9 ms per update)
WGRAD_SPLIT_SIDE = False
# conv3's forward computes each distinct 5x5-tile patch of the minibatch once (merlin_tower_window_conv3_reuse,
# MinibatchWindows.rep_row; same outputs): "gather" -- only the representative rows of a3 are written and fc1's
# forward and weight-gradient GEMMs read every row through rep_row (merlin_h3_gemm_{nt,tn}_gather; h3 only, else as
# "copy"); "copy" -- the other rows copied from theirs; False -- every row computed
PATCH_REUSE = "gather"
# with "gather": the other rows' mask words copied on the side stream beside the forward GEMM (False: right after the
# representatives, on the main stream).  Off: the 15-us copy beside the GEMM slowed the update, 194.8 vs 189.6 ms
# (scripts/ab_update.py 5 6 fast,fast_maskmain), as every side-stream kernel beside the NT GEMMs has
MASK_COPY_SIDE = False
# with "gather": the non-representative rows' mask words are not copied at all; the patch sums (R pass) read each row's
# word through rep_row (merlin_segment_sum_mask_rows)
MASK_ROWS = True
# h3 with gathered a3 rows: dz leaves k_head_bwd as h3 planes scaled by a bound on max |dz| known before the pass (the
# loss's per-output maxima of dlogits / dvalue through the heads' weights: merlin_ppo_loss_absmax,
# merlin_tower_head_bwd_planes) instead of fp32 + its max, so the input gradient runs on both operands as planes
# (merlin_h3_gemm_nt_planes, LDS-DMA staged, cfg H3_NT_CFG["dgrad_planes"]) and the weight gradient stages dz's
# planes as copies (merlin_h3_gemm_tn_gather_planes_a).  False: dz in fp32, split by the GEMMs.
DZ_PLANES = True
# conv3's backward chain's fills made before the side-stream weight gradient starts (_conv3_backward_prefill)
PREFILL = True
# with DZ_PLANES: conv3's representative rows leave k_window_conv3_reps as h3 planes too, scaled by a bound on max Y3
# from Q's column maxima (merlin_tower_window_conv3_planes), so the forward GEMM stages a3 as copies
# (merlin_h3_gemm_nt_heads_planes) and the weight gradient runs on both operands' planes
# (merlin_h3_gemm_tn_gather_planes; with both operands as planes, the LDS-DMA TN k_h3_tq, H3_TN_CFG_PLANES).  False:
# a3 in fp32, split by the GEMMs.  (Before k_h3_tq, with the register-staged TN: off -- kernel traces of one setting
# per process, profiles/r05n_*_timeline.txt, had the forward no faster in the loop, the weight gradient 732 vs 716 us
# and conv3's patch sums beside it 223 vs 192 us; 172.5 vs 169.9 ms per update.)
A3_PLANES = True


class WindowStep:
    """One optimizer step of PPO._sgd on the window + x6 path (see the module docstring)."""

    def __init__(self, agent):
        # weak: the agent holds this step (agent._wstep); a strong back-reference made every agent a reference
        # cycle that only the cyclic GC frees -- possibly in the middle of another agent's graph capture
        self._agent = weakref.ref(agent)
        ac = agent.ac
        self.params = list(ac.parameters())
        flat_params = agent._flat_params
        off = 0
        for p in self.params:  # the parameters are views of agent._flat_params in parameter order
            assert p.data_ptr() == flat_params.data_ptr() + 4 * off, "parameters moved off the flat buffer"
            off += p.numel()
        dp = agent.dp
        if dp.enabled:
            flat = dp._flat_grad  # the gradient RCCL all-reduces; every p.grad is a view of it
        else:
            flat = torch.zeros(off, dtype=torch.float32, device=agent.device)
        assert flat.numel() == off
        views, off = {}, 0
        for p in self.params:
            n = p.numel()
            views[p] = flat[off:off + n].view_as(p)
            off += n
        self.flat, self.views = flat, views
        self.fc1 = getattr(ac, "fc1_impl", "h3")
        self.stage = WeightStage(ac, flat_params, flat, impl=getattr(agent, "stage_impl", "hip"), fc1=self.fc1)
        self.head = (ac.actor[2].weight, ac.actor[2].bias, ac.critic[2].weight, ac.critic[2].bias)
        self._side = None
        # [0:2] max |a3|, [2:4] max |dz| (or its bound), [4:13] the loss's max |dlogits[:, j]| / |dvalue| (DZ_PLANES)
        self.amax_act = torch.zeros(16, dtype=torch.int32, device=agent.device)
        self.amax_win = torch.zeros(4, dtype=torch.int32, device=agent.device)  # a2w's and dQ's scales

    def valid(self) -> bool:
        if not (self.stage.valid() and all(p.requires_grad for p in self.params)):
            return False
        ag = self._agent()
        if ag is None or getattr(ag.ac, "fc1_impl", "h3") != self.fc1:
            return False
        off, base = 0, self.stage.flat_params.data_ptr()
        for p in self.params:
            if p.data_ptr() != base + 4 * off:
                return False
            off += p.numel()
        return True

    def bind_grads(self):
        """Every parameter's .grad is its view of the flat buffer (each step overwrites all of them)."""
        for p in self.params:
            v = self.views[p]
            if p.grad is None or p.grad.data_ptr() != v.data_ptr():
                p.grad = v

    def side_stream(self, device):
        key = (SIDE_PRIORITY, SIDE_CU_GROUPS)
        if self._side is None or getattr(self, "_side_key", None) != key:
            if SIDE_CU_GROUPS:  # the weight gradient on SIDE_CU_GROUPS of every 4 groups of 8 CUs
                self._side = nat.cu_masked_stream(device, lambda i: (i // 8) % 4 < SIDE_CU_GROUPS)
            else:
                self._side = torch.cuda.Stream(device=device, priority=SIDE_PRIORITY)
            self._side_key = key
        return self._side

    def step(self, plan, mb, mb_idx, actions, logp_old, adv, ret, totals):
        """Forward, loss (statistics added to `totals`), backward of one minibatch: every parameter's gradient
        is left in its .grad view (the optimizer step follows in PPO._sgd)."""
        if MAIN_PRIORITY >= 0:
            return self._step(plan, mb, mb_idx, actions, logp_old, adv, ret, totals)
        # the step's main-stream work on a high-priority stream, so that conv3's backward chain gets CUs ahead of the
        # side stream's weight gradient when both are queued (torch's default stream has the lowest priority)
        cur = torch.cuda.current_stream()
        hp = getattr(self, "_hi", None)
        if hp is None:
            hp = self._hi = torch.cuda.Stream(device=cur.device, priority=MAIN_PRIORITY)
        hp.wait_stream(cur)
        with torch.cuda.stream(hp):
            self._step(plan, mb, mb_idx, actions, logp_old, adv, ret, totals)
        cur.wait_stream(hp)

    def _step(self, plan, mb, mb_idx, actions, logp_old, adv, ret, totals):
        ag = self._agent()
        Wa, ba, Wc, bc = self.head
        g = self.stage.grads  # (dT2, db2, dW3r, db3, dW4p, db4)
        # ---- forward (merlin/windows.py window_tower_head_x6)
        h3 = self.fc1 == "h3"
        # this step's operand scales [max |a3| per tower, max |dz| per tower], filled by atomics in the producer
        # kernels; zeroed here by a plain launch, not inside the captured forward graph: a zeroing captured as a
        # memset node replays with a wrong fill value on ROCm 7 (0x80808080: an exponent that overflows every plane,
        # NaN in the second update; scripts/probe_graph_then.py)
        am = self.amax_act
        if h3:
            am.zero_()
        T2, b2, W3r, b3, _, b4 = self.stage.forward()
        P4, P4t = self.stage.planes[:2]
        am3, amz, amW = am[0:2], am[2:4], self.stage.amaxW
        a2w = nat.window_lut(plan.rows, T2, bias=b2)  # relu(conv2) of every window (bias and ReLU fused)
        wh3 = h3 and WINDOW_H3 and len(self.stage.planes) == 4
        if wh3:
            P3t, P3 = self.stage.planes[2:]
            am2, amq, amW3 = self.amax_win[0:2], self.amax_win[2:4], self.stage.amaxW3
            nat.h3_amax(a2w, out=am2)
            Q = nat.h3_gemm_nt(a2w, am2, P3t, amW3, cfg=nat.H3_NT_CFG["qwin"], name="gemm_window_fwd")
        elif WINDOW_BWD_HIP:  # the same exact-f32 MFMA kernels as its backward (csrc/merlin_winbwd.hip)
            Q = nat.window_gemm_fwd(a2w, W3r)  # [2, windows, (ky, kx, co)]
        else:
            Q = torch.bmm(a2w, W3r)  # [2, windows, (ky, kx, co)]
        split_side = h3 and WGRAD_SPLIT_SIDE and WGRAD_SIDE and not WGRAD_EARLY
        rep_row = getattr(mb, "rep_row", None) if PATCH_REUSE else None
        # a3's rows through their patch representatives (the other rows never written)
        arows = rep_row if (PATCH_REUSE == "gather" and h3 and not WGRAD_PLANES and not split_side) else None
        # with gathered rows: the representatives only here; the other rows' mask words (read by the backward's patch
        # sums) are copied on the side stream beside the forward GEMM, joined by an event before that pass
        # MASK_ROWS: no copy at all, the patch sums read each row's mask word through its representative
        n = int(mb.groups.numel())
        a3p = (arows is not None and DZ_PLANES and A3_PLANES and MASK_ROWS and not MASK_COPY_SIDE
               and nat.H3_HEADS_EPILOGUE and int(Wa.shape[0]) <= 4)
        if a3p:  # the representatives as h3 planes, am3 = the bound they are scaled by
            Y3, bits = nat.window_conv3_planes(Q, plan.wid, mb.groups, b3, rep_row, am3,
                                               n_reps=getattr(mb, "n_reps", None))
            a3 = Y3.view(2, n, 1152)
        else:
            Y3, bits = nat.window_conv3(Q, plan.wid, mb.groups, b3, bits=True, amax=am3 if h3 else None,
                                        rep_row=rep_row,
                                        copy=(0 if (MASK_COPY_SIDE or MASK_ROWS) else 2) if arows is not None else 3,
                                        n_reps=getattr(mb, "n_reps", None))
            a3 = Y3.view(2, n, 576)
        pa3 = pdz = None
        main = torch.cuda.current_stream()
        side = self.side_stream(a3.device)
        masks_ready = None
        if arows is not None and MASK_COPY_SIDE and not MASK_ROWS:
            side.wait_stream(main)
            with torch.cuda.stream(side):
                nat.window_conv3_copy_masks(Y3, bits, rep_row)
                masks_ready = torch.cuda.Event()
                masks_ready.record(side)
            bits.record_stream(side)
            Y3.record_stream(side)
        if split_side:  # a3's planes for the weight gradient, on the side stream beside the forward GEMM
            side.wait_stream(main)
            with torch.cuda.stream(side):
                pa3 = nat.h3_split(a3, am3)
        if h3:
            # the forward and input-gradient GEMMs leave their fp32 operand's planes (a3's, dz's) for the weight
            # gradient, which then stages copies instead of splitting both operands again
            if WGRAD_PLANES and not split_side:
                pa3 = torch.empty((2, n, 1152), dtype=torch.int16, device=a3.device)
            if (pa3 is None and nat.H3_HEADS_EPILOGUE
                    and nat.lib().merlin_h3_heads_parts(P4.shape[1], nat.H3_NT_CFG["fwd"]) > 0):
                # both heads in the GEMM's epilogue (the loss adds their biases)
                h, logits, value = nat.h3_gemm_nt_heads(a3, am3, P4, amW, b4, Wa, Wc,
                                                        cfg=nat.H3_NT_CFG["fwd_planes" if a3p else "fwd"],
                                                        rows=arows, name="gemm_fc1_fwd")
            else:
                h = nat.h3_gemm_nt(a3, am3, P4, amW, bias=b4, cfg=nat.H3_NT_CFG["fwd"], name="gemm_fc1_fwd",
                                   planes_out=pa3, rows=arows)
                logits, value = nat.heads_fwd(h, Wa, Wc)  # both heads in one pass over h (the loss adds the biases)
        else:
            h = nat.x6_gemm_nt(a3, P4, bias=b4, cfg=nat.X6_NT_CFG["fwd"], name="gemm_fc1_fwd")
            logits, value = nat.heads_fwd(h, Wa, Wc)  # both heads in one pass over h (the loss adds their biases)
        # ---- loss and its gradient per frame (merlin.ppo._PPOLoss); the head-bias gradients land in .grad
        dzp = h3 and DZ_PLANES and arows is not None and pa3 is None and int(Wa.shape[0]) <= 8
        assert dzp or not a3p
        dmax = am[4:13] if dzp else None
        _, dlogits, dvalue, _, _ = nat.ppo_loss(
            logits, value, mb.offs, mb.order, mb.inv, mb_idx, actions, logp_old, adv, ret, ag.clip_eps, ag.vf_coef,
            ag.ent_coef, totals, bias_actor=ba, bias_critic=bc, out_bias_actor=self.views[ba],
            out_bias_critic=self.views[bc], grad_absmax=dmax)
        # ---- backward (_WindowTowerHeadX6.backward, _WindowGemm / _BiasRelu / _WindowConv2 backward)
        # (dzp: dz is its h3 planes, int16 [2, n, 1024], scaled by the bound left in amz)
        dz, _, _, _ = nat.head_bwd(h, dlogits, dvalue, Wa, Wc, out_bias=g[5], out_w_actor=self.views[Wa],
                                   out_w_critic=self.views[Wc], amax=amz if h3 else None, grad_absmax=dmax)
        if split_side:  # and dz's beside the input-gradient GEMM
            side.wait_stream(main)
            with torch.cuda.stream(side):
                pdz = nat.h3_split(dz, amz)

        def wgrad():
            if h3 and pdz is not None:
                nat.h3_gemm_tn(pdz, amz, pa3, am3, name="gemm_wgrad", out=g[4])
            elif h3:
                nat.h3_gemm_tn(dz, amz, a3, am3, name="gemm_wgrad", out=g[4], rows=arows,
                               cfg=nat.H3_TN_CFG_PLANES if a3p else None)
            else:
                nat.x6_gemm_tn(dz, a3, name="gemm_wgrad", out=g[4])

        if WGRAD_EARLY:  # fc1's weight gradient beside the input gradient and conv3's segmented sums
            side.wait_stream(main)
            with torch.cuda.stream(side):
                wgrad()
        # conv3's backward chain's fills (the band marks preset to -1, the dQ table zeroed) ahead of the side-stream
        # weight gradient: launched beside it, a small fill waits for a CU the GEMM's blocks free (~90 us each with
        # the LDS-DMA weight gradient, whose blocks hold a CU's LDS and VGPRs whole; profiles/r05u_* trace)
        pre = _conv3_backward_prefill(plan, int(Q.shape[1]), dz.device) if PREFILL else None
        if dzp:
            da3 = nat.h3_gemm_nt_planes(dz, amz, P4t, amW, cfg=nat.H3_NT_CFG["dgrad_planes"], name="gemm_fc1_dgrad")
        elif h3:
            if pa3 is not None and not WGRAD_EARLY and not split_side:
                pdz = torch.empty((2, n, 1024), dtype=torch.int16, device=dz.device)
            da3 = nat.h3_gemm_nt(dz, amz, P4t, amW, cfg=nat.H3_NT_CFG["dgrad"], name="gemm_fc1_dgrad",
                                 planes_out=None if split_side else pdz)
        else:
            da3 = nat.x6_gemm_nt(dz, P4t, cfg=nat.X6_NT_CFG["dgrad"], name="gemm_fc1_dgrad")
        if not WGRAD_SIDE:
            wgrad()
        elif not WGRAD_EARLY:  # fc1's weight gradient beside conv3's segmented sums
            side.wait_stream(main)
            with torch.cuda.stream(side):
                wgrad()
        for x in (dz, a3, pdz, pa3):
            if x is not None:
                x.record_stream(side)
        if masks_ready is not None:
            main.wait_event(masks_ready)
        dQ = _conv3_backward_bulk(plan, mb, bits, da3.view(2, n * 9, 64), int(Q.shape[1]),
                                  mask_rows=arows if MASK_ROWS else None, pre=pre)
        if wh3 or not WINDOW_BWD_HIP:  # (else summed by merlin_window_gemm_bwd below)
            nat.colsum(dQ.view(2, -1, 9, 64)[:, :, 0], out=g[3])  # db3: every (u, p3) has one window at tap 0
        dQ = dQ.view(2, -1, 576)
        if wh3:
            nat.h3_amax(dQ, out=amq)
            da2w = nat.h3_gemm_nt(dQ, amq, P3, amW3, cfg=nat.H3_NT_CFG["qwin_dgrad"], name="gemm_window_dgrad")
            nat.h3_gemm_tn(a2w, am2, dQ, amq, cfg=nat.H3_TN_CFG_WIN, name="gemm_window_wgrad", out=g[2])
        elif WINDOW_BWD_HIP:  # both products, the ReLU mask and db2 in one launch + an ordered fold
            da2w, _, _ = nat.window_gemm_bwd(a2w, dQ, W3r, out_db2=g[1], out_dW3r=g[2], out_db3=g[3])
        else:
            da2w = torch.bmm(dQ, W3r.transpose(1, 2))
            chunks = max(1, a2w.shape[1] // 256)
            _splitk_bmm_tn(a2w, dQ, chunks, min_chunk=128, name="gemm_window_wgrad", out=g[2])
        if wh3 or not WINDOW_BWD_HIP:
            nat.relu_bwd(a2w, da2w, out=da2w, out_bias=g[1])
        nat.segment_sum(da2w, plan.hist, nat.LUT2_ROWS, name="k_seg_sum_dT2", out=g[0])
        main.wait_stream(side)
        self.stage.backward()


def _conv3_backward_prefill(plan, nw, device):
    """(band marks preset to -1, zeroed dQ table) for _conv3_backward_bulk, made ahead of the weight gradient."""
    bslot = getattr(plan, "_bslot", None)
    if bslot is None:
        bslot = plan._bslot = torch.empty(plan.num_bands, dtype=torch.int32, device=device)
    bslot.fill_(-1)
    dq = torch.zeros((2, nw * 9, 64), dtype=torch.float32, device=device)
    return bslot, dq


def _conv3_backward_bulk(plan, mb, bits, dY3, nw, mask_rows=None, pre=None):
    """dQ [T, nw*9, 64] of merlin.windows._conv3_backward with the minibatch's live-patch map taken from
    the update-wide array (mb.kmap, WindowPlan.update_minibatches(bulk=True)).  pre: (bslot preset to -1, zeroed
    dQ) from _conv3_backward_prefill."""
    R = nat.segment_sum(dY3.contiguous(), plan.patch_plan, plan.num_patches, slot=mb.slot, sub=9,
                        name="k_seg_sum_R", mask=bits, fill=False, mask_rows=mask_rows)
    # band sums over the live patches, marking the bands that got one (merlin_segment_sum_marked); dQ reads only
    # those: the dead bands' rows are never zeroed (a 128-MB fill per step) nor read
    if pre is None:
        bslot = getattr(plan, "_bslot", None)
        if bslot is None:
            bslot = plan._bslot = torch.empty(plan.num_bands, dtype=torch.int32, device=dY3.device)
        bslot.fill_(-1)
    else:
        bslot = pre[0]
    S = nat.segment_sum(R, plan.band_plan, plan.num_bands, slot=mb.kmap, sub=1, name="k_seg_sum_S", fill=False,
                        mark=bslot)
    if pre is not None:  # the table was zeroed ahead: only the sums are written
        return nat.segment_sum(S, plan.dq_plan, nw * 9, slot=bslot, sub=1, name="k_seg_sum_dQ", out=pre[1],
                               fill=False)
    return nat.segment_sum(S, plan.dq_plan, nw * 9, slot=bslot, sub=1, name="k_seg_sum_dQ")
