"""The optimizer step of PPO.update on the device (src/ppo.py:153-156):

    nn.utils.clip_grad_norm_(self.policy.parameters(), 0.5)
    self.optimizer.step()                      # optim.Adam(lr=...)

as two HIP launches (merlin_clip_adam, csrc/merlin_optim.hip) instead of torch's ~10-launch
chain (foreach norm, stack, vector_norm, coefficient, clamp, foreach mul, step add, fused Adam).
The state lives in the wrapped torch.optim.Adam (exp_avg / exp_avg_sq / float32 `step` tensors on
the device, as Adam(fused=True) keeps them), so `optimizer.state_dict()` and checkpoints are
unchanged and the torch optimizer can take over again at any step.
"""
from __future__ import annotations

import torch

from . import _native as nat


class ClipAdam:
    def __init__(self, optimizer: torch.optim.Adam, max_norm: float):
        if len(optimizer.param_groups) != 1:
            raise ValueError("ClipAdam: one parameter group")
        g = optimizer.param_groups[0]
        if g.get("weight_decay", 0) or g.get("amsgrad") or g.get("maximize"):
            raise ValueError("ClipAdam: plain Adam only (no weight decay / amsgrad / maximize)")
        self.optimizer = optimizer
        self.max_norm = float(max_norm)
        self._ws = None
        self._norm = None

    def step(self) -> torch.Tensor:
        """clip_grad_norm_(params, max_norm) then Adam.step(); returns the pre-clip norm (0-d f32)."""
        g = self.optimizer.param_groups[0]
        ps = [p for p in g["params"] if p.grad is not None]
        if not ps:
            raise RuntimeError("ClipAdam.step: no parameter has a gradient")
        st = self.optimizer.state
        for p in ps:
            s = st[p]
            if len(s) == 0:  # what Adam(fused=True) creates on its first step
                s["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
                s["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                s["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        dev = ps[0].device
        if self._norm is None or self._norm.device != dev:
            self._norm = torch.empty((), dtype=torch.float32, device=dev)
        n_ws = int(nat.lib().merlin_clip_adam_workspace(len(ps), (nat.C.c_int64 * len(ps))(*[p.numel() for p in ps])))
        if self._ws is None or self._ws.numel() < n_ws or self._ws.device != dev:
            self._ws = torch.empty(n_ws, dtype=torch.float64, device=dev)
        b1, b2 = g["betas"]
        lr = g["lr"]
        if isinstance(lr, torch.Tensor):
            lr = float(lr)
        return nat.clip_adam(ps, [p.grad for p in ps], [st[p]["exp_avg"] for p in ps],
                             [st[p]["exp_avg_sq"] for p in ps], [st[p]["step"] for p in ps], lr, b1, b2, g["eps"],
                             self.max_norm, norm_out=self._norm, workspace=self._ws)
