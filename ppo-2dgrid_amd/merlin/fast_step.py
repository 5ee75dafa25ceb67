"""PPO.update's minibatch step on the window + x6 path with the launch sequence written out
(src/ppo.py:136-156: forward, loss, backward, clip_grad_norm_(0.5), Adam).

The autograd engine walked ~95 kernels per optimizer step, ~60 of them small torch ops, and the host
needed ~2 ms per step to queue them: at the bench state the GPU sat idle for ~20 % of every update
waiting for the host (scripts/busy_union.py on a rocprofv3 kernel trace: 67-75 ms of ~300-365 ms).
Here the step is the same kernels with the same operands in the same order, issued directly:

  * WeightStage -- everything that depends on the parameters alone (the conv1 / conv2 tables T2,
    the stacked and permuted conv3 / fc1 weights, fc1's x6 planes for the forward and the input
    gradient) is one captured HIP graph, and the backward of that subgraph (the table / stacking
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

import torch

from . import _native as nat
from .actor_critic import _splitk_bmm_tn


class WeightStage:
    """Parameter-only forward / backward of the minibatch step as two captured HIP graphs.

    forward() -> (T2 [2, 2720, 64], b2 [2, 64], W3r [2, 64, 576], b3 [2, 64], W4p [2, H, 576], b4 [2, H]) and
    self.planes = (x6 planes of W4p, of W4p^T); backward() maps the gradients left in self.grads (same shapes
    as forward()'s outputs) to the gradients of the 16 tower / fc1 parameters, written into `grad_views`."""

    def __init__(self, ac, grad_views: dict):
        self.ac = ac
        ea, ec = ac.actor_extractor.network, ac.critic_extractor.network
        fa, fc = ac.actor[0], ac.critic[0]
        self.params = [ea[0].weight, ea[0].bias, ec[0].weight, ec[0].bias, ea[2].weight, ea[2].bias, ec[2].weight,
                       ec[2].bias, ea[4].weight, ea[4].bias, ec[4].weight, ec[4].bias, fa.weight, fa.bias, fc.weight,
                       fc.bias]
        self.views = [grad_views[p] for p in self.params]
        self.ptrs = [p.data_ptr() for p in self.params]
        self._capture()

    def _fwd(self):
        ac = self.ac
        ea, ec = ac.actor_extractor.network, ac.critic_extractor.network
        fa, fc = ac.actor[0], ac.critic[0]
        H = fa.weight.shape[0]
        T2 = ac.conv2_tables()
        b2 = torch.stack([ea[2].bias, ec[2].bias])
        W3 = torch.stack([ea[4].weight, ec[4].weight])  # [2, co, ci, ky, kx]
        W3r = W3.permute(0, 2, 3, 4, 1).reshape(2, 64, 576)  # [2, ci, (ky, kx, co)]
        b3 = torch.stack([ea[4].bias, ec[4].bias])
        W4 = torch.stack([fa.weight, fc.weight])  # [2, H, 576] in (co, p3) order
        W4p = W4.view(2, H, 64, 9).transpose(2, 3).reshape(2, H, 576)  # (p3, co): a3's column order
        b4 = torch.stack([fa.bias, fc.bias])
        planes = (nat.x6_split(W4p.detach()), nat.x6_split(W4p.detach().transpose(1, 2).contiguous()))
        return (T2, b2, W3r, b3, W4p, b4), planes

    def _capture(self):
        main = torch.cuda.current_stream()
        side = torch.cuda.Stream()
        side.wait_stream(main)
        with torch.cuda.stream(side), torch.enable_grad():
            for _ in range(2):  # lazy initialisation (GEMM handles, cached gather matrices) outside the captures
                outs, _ = self._fwd()
                torch.autograd.grad(outs, self.params, grad_outputs=[torch.ones_like(o) for o in outs])
        main.wait_stream(side)
        torch.cuda.synchronize()
        self.pool = torch.cuda.graph_pool_handle()
        self.gfwd, self.gbwd = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.enable_grad():
            with torch.cuda.graph(self.gfwd, pool=self.pool):
                outs, planes = self._fwd()
            self.grads = tuple(torch.zeros_like(o) for o in outs)
            with torch.cuda.graph(self.gbwd, pool=self.pool):
                gs = torch.autograd.grad(outs, self.params, grad_outputs=self.grads, retain_graph=True)
                for g, v in zip(gs, self.views):
                    v.copy_(g)
        self._keep = (outs, gs)  # the saved tensors the backward graph reads stay allocated
        self.outs = tuple(o.detach() for o in outs)
        self.planes = planes
        torch.cuda.synchronize()

    def valid(self) -> bool:
        return all(p.data_ptr() == q for p, q in zip(self.params, self.ptrs))

    def forward(self):
        self.gfwd.replay()
        return self.outs

    def backward(self):
        self.gbwd.replay()


class WindowStep:
    """One optimizer step of PPO._sgd on the window + x6 path (see the module docstring)."""

    def __init__(self, agent):
        self.agent = agent
        ac = agent.ac
        self.params = [p for p in ac.parameters() if p.requires_grad]
        dp = agent.dp
        if dp.enabled:
            flat = dp._flat_grad  # the gradient RCCL all-reduces; every p.grad is a view of it
        else:
            flat = torch.zeros(sum(p.numel() for p in self.params), dtype=torch.float32, device=agent.device)
        views, off = {}, 0
        for p in self.params:
            n = p.numel()
            views[p] = flat[off:off + n].view_as(p)
            off += n
        self.flat, self.views = flat, views
        self.stage = WeightStage(ac, views)
        self.head = (ac.actor[2].weight, ac.actor[2].bias, ac.critic[2].weight, ac.critic[2].bias)
        self._side = None

    def valid(self) -> bool:
        return self.stage.valid() and all(p.requires_grad for p in self.params)

    def bind_grads(self):
        """Every parameter's .grad is its view of the flat buffer (each step overwrites all of them)."""
        for p in self.params:
            v = self.views[p]
            if p.grad is None or p.grad.data_ptr() != v.data_ptr():
                p.grad = v

    def side_stream(self, device):
        if self._side is None:
            self._side = torch.cuda.Stream(device=device)
        return self._side

    def step(self, plan, mb, mb_idx, actions, logp_old, adv, ret, totals):
        """Forward, loss (statistics added to `totals`), backward of one minibatch: every parameter's gradient
        is left in its .grad view (the optimizer step follows in PPO._sgd)."""
        ag = self.agent
        Wa, ba, Wc, bc = self.head
        g = self.stage.grads  # (dT2, db2, dW3r, db3, dW4p, db4)
        # ---- forward (merlin/windows.py window_tower_head_x6)
        T2, b2, W3r, b3, _, b4 = self.stage.forward()
        P4, P4t = self.stage.planes
        a2w = nat.bias_relu_(nat.window_lut(plan.rows, T2), b2)  # relu(conv2) of every window
        Q = torch.bmm(a2w, W3r)  # [2, windows, (ky, kx, co)]
        Y3, bits = nat.window_conv3(Q, plan.wid, mb.groups, b3, bits=True)
        n = int(mb.groups.numel())
        a3 = Y3.view(2, n, 576)
        h = nat.x6_gemm_nt(a3, P4, bias=b4, cfg=nat.X6_NT_CFG["fwd"], name="gemm_fc1_fwd")
        logits = torch.mm(h[0], Wa.t())
        value = torch.mm(h[1], Wc.t()).squeeze(-1)
        # ---- loss and its gradient per frame (merlin.ppo._PPOLoss); the head-bias gradients land in .grad
        _, dlogits, dvalue, _, _ = nat.ppo_loss(
            logits, value, mb.offs, mb.order, mb.inv, mb_idx, actions, logp_old, adv, ret, ag.clip_eps, ag.vf_coef,
            ag.ent_coef, totals, bias_actor=ba, bias_critic=bc, out_bias_actor=self.views[ba],
            out_bias_critic=self.views[bc])
        # ---- backward (_WindowTowerHeadX6.backward, _WindowGemm / _BiasRelu / _WindowConv2 backward)
        dz, _, _, _ = nat.head_bwd(h, dlogits, dvalue, Wa, Wc, out_bias=g[5], out_w_actor=self.views[Wa],
                                   out_w_critic=self.views[Wc])
        da3 = nat.x6_gemm_nt(dz, P4t, cfg=nat.X6_NT_CFG["dgrad"], name="gemm_fc1_dgrad")
        main = torch.cuda.current_stream()
        side = self.side_stream(dz.device)
        side.wait_stream(main)  # fc1's weight gradient beside conv3's segmented sums
        with torch.cuda.stream(side):
            nat.x6_gemm_tn(dz, a3, name="gemm_wgrad", out=g[4])
        dz.record_stream(side)
        a3.record_stream(side)
        dQ = _conv3_backward_bulk(plan, mb, bits, da3.view(2, n * 9, 64), int(Q.shape[1]))
        nat.colsum(dQ.view(2, -1, 9, 64)[:, :, 0], out=g[3])  # db3: every (u, p3) has one window at tap 0
        dQ = dQ.view(2, -1, 576)
        da2w = torch.bmm(dQ, W3r.transpose(1, 2))
        chunks = max(1, a2w.shape[1] // 256)
        _splitk_bmm_tn(a2w, dQ, chunks, min_chunk=128, name="gemm_window_wgrad", out=g[2])
        nat.relu_bwd(a2w, da2w, out=da2w, out_bias=g[1])
        nat.segment_sum(da2w, plan.hist, nat.LUT2_ROWS, name="k_seg_sum_dT2", out=g[0])
        main.wait_stream(side)
        self.stage.backward()


def _conv3_backward_bulk(plan, mb, bits, dY3, nw):
    """dQ [T, nw*9, 64] of merlin.windows._conv3_backward with the minibatch's live-patch map taken from
    the update-wide array (mb.kmap, WindowPlan.update_minibatches(bulk=True))."""
    R = nat.segment_sum(dY3.contiguous(), plan.patch_plan, plan.num_patches, slot=mb.slot, sub=9,
                        name="k_seg_sum_R", mask=bits, fill=False)
    S = nat.segment_sum(R, plan.band_plan, plan.num_bands, slot=mb.kmap, sub=1, name="k_seg_sum_S")
    return nat.segment_sum(S, plan.dq_plan, nw * 9, name="k_seg_sum_dQ")
