"""Data parallelism over ranks = GPUs, one process per GPU.

Envs shard with no data-path collective: rank r owns envs [r*N, (r+1)*N) and seeds
them with the global index.  The PPO update keeps the reference's single-learner
semantics with two exchanges per iteration on the process group (RCCL on ROCm):
  * advantage moments (count, sum, sum of squares; f64[3]) all-reduced once, so
    normalisation uses the statistics of the concatenated batch (src/ppo.py:125);
  * the flat f32 gradient (744,772 params = 2.98 MB) all-reduced and averaged once
    per optimizer step, before clip_grad_norm_(0.5) and the replicated Adam step.
Parameters live as views of one flat buffer so the gradient goes to RCCL as a single
2.98 MB message (xGMI ring: per-link bound, one launch, no bucketing needed).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


class DataParallel:
    def __init__(self, group=None):
        self.group = group
        self.enabled = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
        self.world = dist.get_world_size(group) if self.enabled else 1
        self.rank = dist.get_rank(group) if self.enabled else 0
        self._flat_grad = None
        self._params = None

    @staticmethod
    def init_from_env(backend: str | None = None, device: torch.device | None = None) -> "DataParallel":
        """torchrun-style init (RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT)."""
        if int(os.environ.get("WORLD_SIZE", "1")) > 1 and not dist.is_initialized():
            if backend is None:
                backend = "nccl" if (device is not None and device.type == "cuda") else "gloo"
            kw = {}
            if backend == "nccl" and device is not None:
                kw["device_id"] = device
            dist.init_process_group(backend=backend, **kw)
        return DataParallel()

    def attach(self, module: torch.nn.Module) -> None:
        """Broadcast rank 0's parameters and back every .grad by one flat buffer.  The buffer spans every
        parameter in parameter order (frozen ones too, so it lines up with the flat parameter buffer of
        merlin/fast_step.py whatever is frozen later); only parameters that require grad get a .grad view."""
        params = list(module.parameters())
        self._params = params
        if not self.enabled:
            return
        with torch.no_grad():
            flat = torch.cat([p.detach().reshape(-1) for p in params])
            dist.broadcast(flat, src=0, group=self.group)
            off = 0
            for p in params:
                n = p.numel()
                p.copy_(flat[off:off + n].view_as(p))
                off += n
        self._flat_grad = torch.zeros(sum(p.numel() for p in params), dtype=params[0].dtype,
                                      device=params[0].device)
        self._bind_grads()

    def _bind_grads(self):
        off = 0
        for p in self._params:
            n = p.numel()
            p.grad = self._flat_grad[off:off + n].view_as(p) if p.requires_grad else None
            off += n

    def zero_grad(self, optimizer) -> None:
        if self.enabled:
            self._flat_grad.zero_()
            self._bind_grads()
        else:
            optimizer.zero_grad(set_to_none=True)

    def allreduce_grads(self) -> None:
        if not self.enabled:
            return
        dist.all_reduce(self._flat_grad, op=dist.ReduceOp.SUM, group=self.group)
        self._flat_grad.div_(self.world)

    def allreduce_sum_(self, t: torch.Tensor) -> torch.Tensor:
        if self.enabled:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t
