"""
Optimizer tail on HIP: Adam + global-norm gradient clipping.

Replaces the reference's ``torch.optim.Adam`` + ``clip_grad_norm_`` sequence
(noisy_src/train.py:112-117, noisy_src/train_pose_opt.py:398-409) with the
fused kernel ``nr_adam_step`` (csrc/optim.hip): one launch per run of
parameters that are contiguous in one flat buffer (a NeRF network is one run),
with the clip coefficient computed on the device from ``nr_sumsq`` — no host
synchronisation.  ``FusedAdam`` is a ``torch.optim.Optimizer``, so
``LambdaLR``/``state_dict`` work as with torch's Adam.
"""

from __future__ import annotations

import weakref
from typing import Iterable, List, Optional, Sequence, Tuple

import torch

from . import ops


def _contiguous_run(ts: Sequence[torch.Tensor]) -> Optional[torch.Tensor]:
    """A 1-D view covering ``ts`` if they lie back to back in one storage, else None."""
    if not ts:
        return None
    base = ts[0]
    st = base.untyped_storage()
    off = base.storage_offset()
    n = 0
    for t in ts:
        if (t.untyped_storage().data_ptr() != st.data_ptr() or t.storage_offset() != off + n
                or not t.is_contiguous() or t.dtype != torch.float32):
            return None
        n += t.numel()
    return torch.empty(0, dtype=torch.float32, device=base.device).set_(st, off, (n,), (1,))


def _runs(params: List[torch.Tensor]) -> List[List[torch.Tensor]]:
    """Split params into maximal runs that are contiguous in memory."""
    runs, cur = [], []
    for p in params:
        if cur and _contiguous_run(cur + [p]) is None:
            runs.append(cur)
            cur = []
        cur.append(p)
    if cur:
        runs.append(cur)
    return runs


def grad_sumsq(params: Iterable[torch.Tensor], out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Device scalar sum of squares of all gradients (HIP reduction, no host sync)."""
    params = [p for p in params if p.grad is not None]
    if out is None:
        out = torch.zeros((), device=params[0].device, dtype=torch.float32)
    for run in _runs([p.grad for p in params]):
        flat = _contiguous_run(run)
        if flat is None or flat.data_ptr() % 16:
            flat = torch.cat([g.reshape(-1) for g in run])
        ops.sumsq_into(flat, out)
    return out


def clip_grad_norm_(parameters, max_norm: float) -> torch.Tensor:
    """torch.nn.utils.clip_grad_norm_ semantics (coef = min(1, max_norm/(norm+1e-6)))."""
    if isinstance(parameters, torch.Tensor):
        parameters = [parameters]
    params = [p for p in parameters if p.grad is not None]
    if not params:
        return torch.zeros(())
    total = grad_sumsq(params).sqrt()
    coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
    for p in params:
        p.grad.mul_(coef)
    return total


class FusedAdam(torch.optim.Optimizer):
    """torch.optim.Adam (amsgrad=False, weight_decay=0) on the HIP fused kernel.

    ``step(clip_groups=[(params, max_norm), ...])`` folds clip_grad_norm_ of each
    group into the update (train.py:115 joint clip; train_pose_opt.py:398-404
    per-network clips)."""

    def __init__(self, params, lr: float = 1e-3, betas: Tuple[float, float] = (0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, amsgrad: bool = False, *, maximize: bool = False, foreach=None,
                 capturable: bool = False, differentiable: bool = False, fused=None,
                 decoupled_weight_decay: bool = False, refresh_images: bool = True):
        # the reference's Adam (train.py:402, train_pose_opt.py:788-789) uses the defaults;
        # the fused kernel implements exactly that configuration
        if weight_decay != 0.0 or amsgrad or maximize or differentiable or decoupled_weight_decay:
            raise ValueError("FusedAdam implements torch.optim.Adam with weight_decay=0, amsgrad=False, "
                             "maximize=False, differentiable=False only")
        # the full torch.optim.Adam param-group keys, so state_dict() loads into torch's Adam
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=0.0, amsgrad=False,
                                      maximize=False, foreach=foreach, capturable=capturable,
                                      differentiable=False, fused=fused, decoupled_weight_decay=False))
        self._flat_state = {}
        # refresh a NeRF's packed MFMA images inside the Adam launch (False: the next
        # forward re-packs them, the pre-fusion behaviour; tests compare the two)
        self.refresh_images = refresh_images
        # graph mode (engine.GraphedTrainer): a device fp32 pair {lr/bc1, sqrt(bc2)} the
        # Adam launch reads, so a captured step replays with the schedule advanced
        self.device_sched: Optional[torch.Tensor] = None
        # parameter lists that are whole NeRF networks, by the parameters' identities:
        # [(net, start, end)] (False: not such a list) -- the per-step fast path
        self._nerf_plans = {}

    def load_state_dict(self, state_dict) -> None:
        """torch's load, then drop the flat m/v buffers so the next step adopts the loaded
        exp_avg / exp_avg_sq (instead of updating stale buffers)."""
        super().load_state_dict(state_dict)
        self._flat_state.clear()

    def _state_run(self, run: List[torch.nn.Parameter]):
        key = tuple(id(p) for p in run)
        cached = self._flat_state.get(key)
        if cached is not None:
            return cached
        n = sum(p.numel() for p in run)
        dev = run[0].device
        m = torch.zeros(n, device=dev, dtype=torch.float32)
        v = torch.zeros(n, device=dev, dtype=torch.float32)
        off = 0
        for p in run:
            st = self.state[p]
            k = p.numel()
            if "exp_avg" in st:  # e.g. restored from a state_dict
                m[off:off + k].copy_(st["exp_avg"].reshape(-1))
                v[off:off + k].copy_(st["exp_avg_sq"].reshape(-1))
            st["exp_avg"] = m[off:off + k].view(p.shape)
            st["exp_avg_sq"] = v[off:off + k].view(p.shape)
            st.setdefault("step", torch.zeros((), dtype=torch.float32))
            off += k
        self._flat_state[key] = (m, v)
        return m, v

    def _nerf_runs(self, params: List[torch.Tensor]):
        """[(run, pflat, gflat, net)] when ``params`` is a concatenation of whole NeRF
        networks' parameter lists (in their order) whose gradients are the views of the
        network's last backward's flat gradient: each network's flat parameter and
        gradient buffers, with O(parameters) pointer checks instead of rebuilding the
        runs (the generic path costs ~1 ms of host time per step).  None otherwise."""
        from .model import flat_owner
        key = tuple(map(id, params))
        plan = self._nerf_plans.get(key)
        if plan and any(ref() is None for ref, _, _, _ in plan):
            plan = None  # a network of this plan is gone (its ids may be reused)
        if plan is None:
            plan, i = [], 0
            while i < len(params):
                net = flat_owner(params[i])
                plist = net._param_list if net is not None else None
                if (not plist or len(params) - i < len(plist)
                        or any(a is not b for a, b in zip(params[i:i + len(plist)], plist))):
                    plan = False
                    break
                offs, off = [], 0
                for p in plist:
                    offs.append(off)
                    off += p.numel()
                # a weak reference: the cache must not keep a network (and its buffers) alive
                plan.append((weakref.ref(net), i, i + len(plist), offs))
                i += len(plist)
            self._nerf_plans[key] = plan
        if not plan:
            return None
        out = []
        for ref, i0, i1, offs in plan:
            net = ref()
            if net is None:
                return None
            run = params[i0:i1]
            flat, g = net._flat, net._last_gflat
            if flat is None or g is None or run[0].data_ptr() != flat.data_ptr() or g.numel() != flat.numel():
                return None
            gp = g.data_ptr()
            for p, off in zip(run, offs):
                if p.grad is None or p.grad.data_ptr() != gp + 4 * off or p.data_ptr() != flat.data_ptr() + 4 * off:
                    return None
            out.append((run, flat, g, net))
        return out

    @torch.no_grad()
    def step(self, closure=None, clip_groups=None):
        """One Adam step of every parameter with a gradient; ``clip_groups`` folds
        clip_grad_norm_ of each group into it.  The whole tail is one nr_sumsq_partials
        launch per clip group and one nr_adam_multi launch per param group (up to 8
        flat buffers each); a NeRF network's packed MFMA images are refreshed inside
        that launch, so its next forward does not re-pack."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        from .model import flat_owner
        clip_of, partials = {}, []
        for plist, max_norm in clip_groups or ():
            plist = [p for p in plist if p.grad is not None]
            if not plist:
                continue
            fast = self._nerf_runs(plist)
            if fast is not None:
                flats = [g for _, _, g, _ in fast]
            else:
                flats = []
                for run in _runs([p.grad for p in plist]):
                    flat = _contiguous_run(run)
                    if flat is None or flat.data_ptr() % 16:
                        flat = torch.cat([g.reshape(-1) for g in run])
                    flats.append(flat)
            if len(flats) > ops.MAX_ADAM_SPANS:  # one buffer per network in practice
                acc = grad_sumsq(plist)
                flats = None
            gi = len(partials)
            partials.append(ops.sumsq_partials(flats) if flats is not None else acc)
            for p in plist:
                clip_of[id(p)] = (gi, float(max_norm), flats is not None)
        for group in self.param_groups:
            b1, b2 = group["betas"]
            params = [p for p in group["params"] if p.grad is not None]
            # runs must agree on memory layout AND on the clip group
            fast = self._nerf_runs(params)
            if fast is not None and any(len({clip_of.get(id(p), (None,))[0] for p in run}) != 1
                                        for run, _, _, _ in fast):
                fast = None
            if fast is not None:
                runs = [(run, pflat, gflat) for run, pflat, gflat, _ in fast]
            else:
                runs = []
                for run in _runs(params):
                    cur = [run[0]]
                    for p in run[1:]:
                        if clip_of.get(id(p), (None,))[0] == clip_of.get(id(cur[0]), (None,))[0]:
                            cur.append(p)
                        else:
                            runs.append((cur, None, None))
                            cur = [p]
                    runs.append((cur, None, None))
            by_step = {}
            for run, pflat, gflat in runs:
                if pflat is None:
                    ops._check(run[0])
                    pflat = _contiguous_run(run)
                    if pflat is None or pflat.data_ptr() % 16:
                        raise RuntimeError("FusedAdam: parameters must be fp32 ROCm tensors (NeRF flat buffers)")
                    gflat = _contiguous_run([p.grad for p in run])
                    if gflat is None or gflat.data_ptr() % 16:
                        gflat = torch.cat([p.grad.reshape(-1) for p in run])
                m, v = self._state_run(run)
                st = self.state[run[0]]
                st["step"] += 1
                step = int(st["step"].item()) if st["step"].device.type == "cpu" else int(st["step"])
                for p in run[1:]:
                    self.state[p]["step"] = st["step"]
                span = {"p": pflat, "g": gflat, "m": m, "v": v}
                clip = clip_of.get(id(run[0]))
                if clip is not None:
                    gi, max_norm, is_partials = clip
                    if is_partials:
                        span["partials"], span["max_norm"] = partials[gi], max_norm
                    else:  # a clip group of more than 8 buffers: the legacy accumulator path
                        span["sumsq"], span["max_norm"] = partials[gi], max_norm
                net = flat_owner(pflat) if ("sumsq" not in span and self.refresh_images) else None
                target = net._fused_pack_target(pflat, run) if net is not None else None
                if target is not None:
                    span["table"], span["packed"] = target
                by_step.setdefault(step, []).append((span, run, net if target is not None else None))
            for step, items in by_step.items():
                fused = [it for it in items if "sumsq" not in it[0]]
                for k in range(0, len(fused), ops.MAX_ADAM_SPANS):
                    ops.adam_multi([sp for sp, _, _ in fused[k:k + ops.MAX_ADAM_SPANS]], group["lr"], b1, b2,
                                   group["eps"], step, sched=self.device_sched)
                for sp, _, _ in items:
                    if "sumsq" in sp:
                        ops.adam_step(sp["p"], sp["g"], sp["m"], sp["v"], group["lr"], b1, b2, group["eps"], step,
                                      sumsq=sp["sumsq"], max_norm=sp["max_norm"])
                for _, run, net in items:
                    for p in run:  # parameters changed behind autograd's back: bump versions
                        torch.autograd.graph.increment_version(p)
                    if net is not None:  # ... and its images were refreshed in the same launch
                        net._mark_packed_fresh(run)
        # the step consumed the networks' flat gradients: drop the extra reference, so
        # zero_grad(set_to_none=True) frees them
        for plan in self._nerf_plans.values():
            for ref, _, _, _ in plan or ():
                net = ref()
                if net is not None:
                    net._last_gflat = None
        return loss
