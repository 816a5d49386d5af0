"""
The training step of the hot path, without host synchronisation.

Mirrors ``train_step`` of the reference (noisy_src/train.py:68-119) plus the
``scheduler.step()`` of its loop (train.py:461): render coarse+fine, MSE losses,
backward through the HIP kernels, joint gradient clip at 1.0 fused into Adam,
LambdaLR 0.1^(step/(lr_decay*1000)).  Losses stay on the device; callers that
log them call ``.item()`` themselves (the reference syncs four times a step).
For data parallelism the flat gradients are all-reduced (RCCL) before the
optimizer step.
"""

from __future__ import annotations

from typing import Dict, Optional

import torch

from . import ops
from .optim import FusedAdam
from .rendering import render_rays


def lr_lambda_factory(lr_decay: int):
    decay_steps = lr_decay * 1000

    def lr_lambda(step):
        return 0.1 ** (step / decay_steps)

    return lr_lambda


class Trainer:
    def __init__(self, model_coarse, model_fine, render_config, lr: float = 5e-4, lr_decay: int = 250,
                 max_norm: float = 1.0, process_group=None):
        self.model_coarse = model_coarse
        self.model_fine = model_fine
        self.render_config = render_config
        params = list(model_coarse.parameters())
        if model_fine is not None:
            params += list(model_fine.parameters())
        self.params = params
        self.max_norm = max_norm
        self.optimizer = FusedAdam(params, lr=lr)
        self.scheduler = torch.optim.lr_scheduler.LambdaLR(self.optimizer, lr_lambda_factory(lr_decay))
        self.process_group = process_group

    def _allreduce_grads(self):
        import torch.distributed as dist
        world = dist.get_world_size(self.process_group)
        for net in (self.model_coarse, self.model_fine):
            if net is None:
                continue
            g = _flat_grad_of(net)
            dist.all_reduce(g, op=dist.ReduceOp.SUM, group=self.process_group)
            if world > 1:
                g.mul_(1.0 / world)

    def step(self, rays_o: torch.Tensor, rays_d: torch.Tensor, target_rgb: torch.Tensor,
             t_rand: Optional[torch.Tensor] = None, u: Optional[torch.Tensor] = None) -> Dict[str, torch.Tensor]:
        self.optimizer.zero_grad(set_to_none=True)
        out = render_rays(self.model_coarse, self.model_fine, rays_o, rays_d, self.render_config, is_train=True,
                          t_rand=t_rand, u=u)
        loss_c = ops.mse_loss(out["rgb_coarse"], target_rgb)
        loss = loss_c
        metrics = {"loss_coarse": loss_c}
        if "rgb_fine" in out:
            loss_f = ops.mse_loss(out["rgb_fine"], target_rgb)
            loss = loss_c + loss_f
            metrics["loss_fine"] = loss_f
        loss.backward()
        if self.process_group is not None:
            self._allreduce_grads()
        self.optimizer.step(clip_groups=[(self.params, self.max_norm)])
        self.scheduler.step()
        metrics["loss"] = loss.detach()
        metrics["rgb_fine"] = out.get("rgb_fine", out["rgb_coarse"]).detach()
        return metrics


def _flat_grad_of(net) -> torch.Tensor:
    """The network's gradient as ONE flat tensor (the MLP backward writes it that way)."""
    from .optim import _contiguous_run
    grads = [p.grad for p in net.parameters()]
    flat = _contiguous_run(grads)
    if flat is None:
        flat = torch.cat([g.reshape(-1) for g in grads])
        off = 0
        for p in net.parameters():
            n = p.numel()
            p.grad = flat[off:off + n].view(p.shape)
            off += n
    return flat
