"""
The training step of the hot path, without host synchronisation.

Mirrors ``train_step`` of the reference (noisy_src/train.py:68-119) plus the
``scheduler.step()`` of its loop (train.py:461): render coarse+fine, MSE losses,
backward through the HIP kernels, joint gradient clip at 1.0 fused into Adam,
LambdaLR 0.1^(step/(lr_decay*1000)).  Losses stay on the device; callers that
log them call ``.item()`` themselves (the reference syncs four times a step).
For data parallelism each network's flat gradient is all-reduced (RCCL) as soon
as its backward has produced it (the fine net's overlaps the coarse backward),
and the optimizer step waits for both.
"""

from __future__ import annotations

from typing import Dict, Optional

import torch

from . import ops
from .optim import FusedAdam
from .rendering import render_rays


def init_distributed(device: str = "cuda"):
    """One process per GPU under ``torch.distributed.run``: reads RANK / LOCAL_RANK /
    WORLD_SIZE, binds the local GPU and joins the default group (backend "nccl" = RCCL
    on ROCm; "gloo" for CPU-device runs).  Returns (process_group or None, rank, world,
    device string).  Without the torchrun environment it is a single process."""
    import os
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if device.startswith("cuda") and torch.cuda.is_available():
        # one GPU per rank; ranks beyond the visible GPUs share them (gloo test mode)
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        device = f"cuda:{local}"
    if world <= 1:
        return None, 0, 1, device
    import torch.distributed as dist
    if not dist.is_initialized():
        if device.startswith("cuda") and os.environ.get("NR_DIST_BACKEND", "nccl") == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(device))
        else:
            dist.init_process_group("gloo")
    return dist.group.WORLD, rank, world, device


def rank_slice(n_global: int, rank: int, world: int) -> slice:
    """Rank r's contiguous share [r*B/N, (r+1)*B/N) of a global batch."""
    if n_global % world:
        raise ValueError(f"global batch {n_global} is not divisible by world size {world}")
    per = n_global // world
    return slice(rank * per, (rank + 1) * per)


def check_run_args(config, world: int, train_data, val_data) -> None:
    """Fail before any work for arguments the loops cannot honour: a global batch the
    ranks cannot split evenly (every batch would be skipped), or only one of
    train_data / val_data (the loops validate on val_data and train on train_data)."""
    if world > 1 and config.data.batch_size % world:
        raise ValueError(f"batch_size {config.data.batch_size} is not divisible by the {world} data-parallel ranks")
    if (train_data is None) != (val_data is None):
        raise ValueError("train_data and val_data must be given together (or neither: load the scene from disk)")


def mean_over_ranks(values, process_group=None):
    """Average a list of device scalars over the group (the logged global-batch losses)."""
    t = torch.stack([v.detach().float().reshape(()) for v in values])
    if process_group is not None:
        import torch.distributed as dist
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=process_group)
        t = t / dist.get_world_size(process_group)
    return t


class LaggedScalars:
    """Logged device scalars read back one iteration late.  ``push`` queues a pinned copy
    of this iteration's values and returns the previous iteration's (synchronising on its
    event only), so the host queues step i+1 while step i still runs instead of idling on
    a per-step ``.item()``/``.tolist()`` as the reference's loops do (train.py:386-420).
    ``flush`` returns the pending values now (before a validation / checkpoint)."""

    def __init__(self, n_max: int = 8):
        self._buf = [torch.zeros(n_max, dtype=torch.float32, pin_memory=True) for _ in range(2)]
        self._k = 0
        self._pending = None

    def push(self, values: torch.Tensor, meta=None):
        n = values.numel()
        host = self._buf[self._k % 2]  # the slot's previous values were resolved by the last push
        self._k += 1
        host[:n].copy_(values.reshape(-1), non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        prev, self._pending = self._pending, (host, n, ev, meta)
        return self._resolve(prev)

    def flush(self):
        prev, self._pending = self._pending, None
        return self._resolve(prev)

    @staticmethod
    def _resolve(p):
        if p is None:
            return None
        host, n, ev, meta = p
        ev.synchronize()
        return host[:n].tolist(), meta


def lr_lambda_factory(lr_decay: int):
    decay_steps = lr_decay * 1000

    def lr_lambda(step):
        return 0.1 ** (step / decay_steps)

    return lr_lambda


class GradAllReducer:
    """Bucketed data-parallel gradient averaging: one async all-reduce (SUM) per flat
    gradient buffer, launched when the buffer is ready; ``finish`` waits.  With
    ``average`` it then divides by the world size; the trainers instead pre-scale the
    backward seed by 1/world (``prescale``), so the SUM already is the mean and no
    multiply kernel runs per buffer.  Backend-agnostic (RCCL on the GPU box, gloo in
    the CPU tests)."""

    def __init__(self, process_group=None, average: bool = True):
        import torch.distributed as dist
        self.dist = dist
        self.group = process_group
        self.world = dist.get_world_size(process_group)
        self.average = average
        self.pending = []
        # timing (bench.py): per eager step, HIP events on the compute stream at the first
        # launch, before ``finish`` waits and after it: (launch -> done) is the collective's
        # span beside the rest of the backward, (wait -> done) what the step is exposed to
        self.timing = None
        self._t_launch = None

    @property
    def prescale(self) -> float:
        """The factor the backward seed carries when ``average`` is off."""
        return 1.0 if self.average else 1.0 / self.world

    def launch(self, flat: torch.Tensor) -> None:
        if flat.is_cuda and torch.cuda.is_current_stream_capturing():
            # inside a hipGraph capture (GraphedTrainer): the stream-ordered form, captured
            # as the collective's kernel plus the stream dependencies around it
            self.dist.all_reduce(flat, op=self.dist.ReduceOp.SUM, group=self.group)
            self.pending.append((None, flat))
            return
        if self.timing is not None and flat.is_cuda and not self.pending:
            self._t_launch = torch.cuda.Event(enable_timing=True)
            self._t_launch.record()
        work = self.dist.all_reduce(flat, op=self.dist.ReduceOp.SUM, group=self.group, async_op=True)
        self.pending.append((work, flat))

    def finish(self) -> None:
        timed = self.timing is not None and self._t_launch is not None
        if timed:
            t_wait = torch.cuda.Event(enable_timing=True)
            t_wait.record()
        for work, flat in self.pending:
            if work is not None:
                work.wait()
            if self.average and self.world > 1:
                flat.mul_(1.0 / self.world)
        if timed:
            t_done = torch.cuda.Event(enable_timing=True)
            t_done.record()
            self.timing.append((self._t_launch, t_wait, t_done))
        self._t_launch = None
        self.pending.clear()

    def timing_summary(self) -> Optional[Dict[str, float]]:
        """Means over the recorded steps (ms): ``span`` = first launch -> all reduced,
        ``exposed`` = the compute stream's wait in ``finish``; None without records."""
        if not self.timing:
            return None
        torch.cuda.synchronize()
        span = [a.elapsed_time(c) for a, _, c in self.timing]
        exposed = [b.elapsed_time(c) for _, b, c in self.timing]
        return {"steps": len(span), "span_ms": sum(span) / len(span), "exposed_ms": sum(exposed) / len(exposed)}


class Trainer:
    """One reference training iteration (train.py:68-119) on the HIP kernels.
    ``coarse_stream``: run the coarse network's forward, compositing, loss and backward on
    a second stream; the coarse backward starts as soon as the coarse forward ends and
    runs beside the fine sampling, forward and backward (the fine samples depend on the
    coarse weights only through detached z values, rays.py:325, so d(loss_c + loss_f)
    reaches the coarse net as d loss_c alone).  Bit-identical to the one-stream step.  It
    pays where one chain does not fill the GPU and the host is out of the way: inside a
    GraphedTrainer capture (the two chains become two branches of the graph) at up to
    ``AUTO_COARSE_STREAM_RAYS`` rays per step (BASELINE cfg #4's 512 rays per rank: 0.856
    -> 0.802 ms per replay; 1024 rays 1.36 -> 1.34 ms; 2048 and 4096 rays no gain or a
    loss; eager steps lose to the second stream's host cost, profiles/r05_coarse_early_ab.txt).
    ``coarse_stream="auto"`` applies exactly that rule per step; True / False force it."""

    AUTO_COARSE_STREAM_RAYS = 1024

    def __init__(self, model_coarse, model_fine, render_config, lr: float = 5e-4, lr_decay: int = 250,
                 max_norm: float = 1.0, process_group=None, coarse_stream=False):
        if coarse_stream not in (True, False, "auto"):
            raise ValueError(f"coarse_stream must be True, False or 'auto', not {coarse_stream!r}")
        self.coarse_stream = coarse_stream if coarse_stream == "auto" else bool(coarse_stream)
        self._cstream = None
        self.last_step_coarse_stream = False  # whether the last step (or capture) used it
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
        self.reducer = None
        if process_group is not None:
            self.reducer = GradAllReducer(process_group, average=False)
            for net in (model_coarse, model_fine):
                if net is not None:
                    net._grad_ready_hook = self.reducer.launch

    def step(self, rays_o: torch.Tensor, rays_d: torch.Tensor, target_rgb: torch.Tensor,
             t_rand: Optional[torch.Tensor] = None, u: Optional[torch.Tensor] = None) -> Dict[str, torch.Tensor]:
        self.optimizer.zero_grad(set_to_none=True)
        cs = None
        if (self.coarse_stream is not False and self.model_fine is not None and rays_o.is_cuda
                and self.render_config.use_hierarchical):
            # created on the first eager step (a GraphedTrainer warms up eagerly), not
            # inside a capture
            if self._cstream is None or self._cstream.device != rays_o.device:
                self._cstream = torch.cuda.Stream(device=rays_o.device)
            if self.coarse_stream is True or (rays_o.shape[0] <= self.AUTO_COARSE_STREAM_RAYS
                                              and torch.cuda.is_current_stream_capturing()):
                cs = self._cstream
        self.last_step_coarse_stream = cs is not None
        gs = self.reducer.prescale if self.reducer is not None else 1.0  # DP: 1/world in the seed
        early = {}

        def coarse_backward(out_c):
            # on the coarse stream: the coarse loss's backward, beside the fine forward
            # (loss = loss_c + loss_f sends exactly d loss_c to the coarse net)
            early["loss_c"] = out_c["loss"]
            early["loss_c"].backward(ops.unit_grad(rays_o.device))

        # the MSE losses (train.py:89/98) come out of the compositing (ops.composite_mse)
        out = render_rays(self.model_coarse, self.model_fine, rays_o, rays_d, self.render_config, is_train=True,
                          t_rand=t_rand, u=u, coarse_stream=cs,
                          coarse_backward=coarse_backward if cs is not None else None,
                          target_rgb=target_rgb, loss_scale=gs)
        if cs is not None:
            main = torch.cuda.current_stream(rays_o.device)
            loss_f = out["loss_fine"]
            loss_c = early["loss_c"].detach()
            lf = loss_f.detach()
            fine_done = main.record_event()
            loss_f.backward(ops.unit_grad(rays_o.device))
            # the summed value on the coarse stream, beside the fine backward (the backward
            # already ran for loss_c; d(loss_c + loss_f) = d loss_f for the fine net).
            # Captured after the fine backward, so that a graph replay keeps the fine
            # chain on one hardware queue (a hop between queues costs ~10 us)
            cs.wait_event(fine_done)
            lf.record_stream(cs)
            with torch.cuda.stream(cs):
                loss = loss_c + lf
            loss.record_stream(main)
            main.wait_stream(cs)  # join the coarse chain
            metrics = {"loss_coarse": loss_c, "loss_fine": lf}
        else:
            loss_c = out["loss_coarse"]
            loss = loss_c
            metrics = {"loss_coarse": loss_c.detach()}  # metrics hold no autograd graph
            if "loss_fine" in out:
                loss_f = out["loss_fine"]
                loss = loss_c + loss_f
                metrics["loss_fine"] = loss_f.detach()
            loss.backward(ops.unit_grad(loss.device))
        if self.reducer is not None:
            flats = [flat for _, flat in self.reducer.pending]
            self.reducer.finish()
            for net in (self.model_coarse, self.model_fine):
                if net is not None:
                    _adopt_reduced_grad(net, flats)
        self.optimizer.step(clip_groups=[(self.params, self.max_norm)])
        self.scheduler.step()
        metrics["loss"] = loss.detach()
        metrics["rgb_fine"] = out.get("rgb_fine", out["rgb_coarse"]).detach()
        return metrics


class GraphedTrainer:
    """``Trainer.step`` captured once into a hipGraph (``torch.cuda.graph``) and replayed:
    the ~23 kernels of a step become one graph launch, so a step costs its GPU time even
    where the host's Python dispatch (autograd, the optimizer's bookkeeping: ~1.3 ms per
    step) exceeds it -- small per-GPU batches such as BASELINE cfg #4's 512 rays per rank.

    Everything the replay needs is on the device: the rays go through static input
    buffers, the jitter / inverse-CDF uniforms are drawn by torch.rand into static
    buffers before each replay (or the caller passes them; torch's graph-safe RNG inside
    the graph when the step also draws noise), the fused Adam launch rewrites the packed
    images, and the two step-dependent Adam scalars come from an 8-byte device pair
    written before each replay (``FusedAdam.device_sched``); the LR schedule and the
    optimizer's step counters advance on the host exactly as in ``Trainer.step``.
    Data parallel: the trainer's RCCL all-reduces (one per network) are captured inside
    the graph in their stream-ordered form, so a replay is the whole DP step.

    The graph holds raw device addresses: every network's packed images and pack table
    and the optimizer's flat m / v buffers.  Those tensors are pinned here, and a replay
    after any of them was replaced (a checkpoint load, ``FusedAdam.load_state_dict``)
    raises instead of writing into freed memory."""

    def __init__(self, trainer: "Trainer", rays_o: torch.Tensor, rays_d: torch.Tensor, target_rgb: torch.Tensor,
                 t_rand: Optional[torch.Tensor] = None, u: Optional[torch.Tensor] = None, warmup: int = 2):
        self.trainer = trainer
        opt = trainer.optimizer
        if not isinstance(opt, FusedAdam) or len(opt.param_groups) != 1:
            raise ValueError("GraphedTrainer needs the trainer's single-group FusedAdam")
        self.static = [t.detach().clone() for t in (rays_o, rays_d, target_rgb)]
        self.static_rand = [None if t is None else t.detach().clone() for t in (t_rand, u)]
        dev = rays_o.device
        # randoms the caller does not inject are drawn into static buffers right before
        # each step (eager warm-ups and every replay) rather than inside the graph: the
        # same torch.rand calls in the same order as the eager step makes them, so the
        # numbers are the eager step's, and a replay skips torch's graph-RNG prologue
        # (two fill launches before every replay of a graph that draws).  Only when the
        # step draws nothing else (raw_noise_std == 0), which would interleave with them
        rc = trainer.render_config
        self._predraw = []
        if t_rand is None and u is None and rc.perturb and not rc.raw_noise_std:
            B = rays_o.shape[0]
            self.static_rand[0] = torch.empty(B, rc.num_samples, device=dev)
            self._predraw.append(self.static_rand[0])
            if rc.use_hierarchical and trainer.model_fine is not None:
                self.static_rand[1] = torch.empty(B, rc.num_samples_fine, device=dev)
                self._predraw.append(self.static_rand[1])
        self.sched = torch.zeros(2, device=dev, dtype=torch.float32)
        # pinned staging ring for the per-step pair: a slot is rewritten only after the
        # copy that read it has run (its event), however far the host runs ahead
        self._ring = torch.zeros(64, 2, dtype=torch.float32).pin_memory()
        self._ring_ev = [None] * 64
        self._k = 0
        # eager warm-up steps on a side stream (allocator pools, optimizer state, packed
        # images and pack tables exist before the capture); they are real training steps.
        # warmup=0 is accepted once the trainer has stepped eagerly (the state exists):
        # the capture then trains on nothing, so a caller's step sequence is unchanged
        if warmup < 1 and not self._step_states():
            warmup = 1
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self._draw()
                trainer.step(*self.static, *self.static_rand)
        torch.cuda.current_stream(dev).wait_stream(side)
        # capture one step; its host-side bookkeeping (Adam step counters, LR scheduler)
        # ran once without device work, so it is rolled back afterwards
        self._common_step()
        steps = [(st, st["step"].clone()) for st in self._step_states()]
        sched_state = trainer.scheduler.state_dict()
        lr = [g["lr"] for g in opt.param_groups]
        opt.device_sched = self.sched
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.out = trainer.step(*self.static, *self.static_rand)
        for st, v in steps:
            st["step"].copy_(v)
        trainer.scheduler.load_state_dict(sched_state)
        for g, v in zip(opt.param_groups, lr):
            g["lr"] = v
        # the graph holds the pair's address; eager steps between replays (a batch of
        # another shape, see train.train) use the host scalars again
        opt.device_sched = None
        self._bound = self._bound_buffers()

    def _draw(self) -> None:
        for t in self._predraw:
            t.uniform_()  # torch.rand(shape) of the eager step, into the static buffer

    def _bound_buffers(self):
        """The device tensors whose addresses the captured graph holds (strong references)."""
        nets = [n for n in (self.trainer.model_coarse, self.trainer.model_fine) if n is not None]
        out = [t for n in nets for t in (n._packed, n._table, n._flat) if t is not None]
        for m, v in self.trainer.optimizer._flat_state.values():
            out += [m, v]
        return out

    def _check_bound(self) -> None:
        now = self._bound_buffers()
        if len(now) != len(self._bound) or any(a is not b for a, b in zip(now, self._bound)):
            raise RuntimeError("GraphedTrainer: a buffer the captured graph writes was replaced (packed images, "
                               "pack table, parameters or Adam state, e.g. by a checkpoint load); "
                               "build a new GraphedTrainer")

    def _common_step(self) -> int:
        """The one Adam step count every buffer shares (one pair of bias corrections
        drives every span of the captured launch)."""
        vals = {int(st["step"]) for st in self._step_states()}
        if len(vals) != 1:
            raise RuntimeError(f"GraphedTrainer: the optimizer's buffers are at different steps {sorted(vals)}")
        return vals.pop()

    def _step_states(self):
        opt = self.trainer.optimizer
        seen, out = set(), []
        for p in opt.param_groups[0]["params"]:
            st = opt.state.get(p)
            if st and "step" in st and id(st["step"]) not in seen:
                seen.add(id(st["step"]))
                out.append(st)
        return out

    def step(self, rays_o: Optional[torch.Tensor] = None, rays_d: Optional[torch.Tensor] = None,
             target_rgb: Optional[torch.Tensor] = None, t_rand: Optional[torch.Tensor] = None,
             u: Optional[torch.Tensor] = None) -> Dict[str, torch.Tensor]:
        """Replay one training step on these rays (copied into the static buffers; None:
        the buffers as they are).  Returns the captured metrics (device tensors that every
        replay overwrites).  Eager ``trainer.step`` calls may be interleaved (same state)."""
        if self._predraw and (t_rand is None) != (u is None) and len(self._predraw) == 2:
            raise ValueError("GraphedTrainer: inject both t_rand and u, or neither")
        dsts, srcs = [], []
        for dst, src in zip(self.static + self.static_rand, (rays_o, rays_d, target_rgb, t_rand, u)):
            if src is not None:
                if dst is None:
                    raise ValueError("GraphedTrainer: t_rand / u were drawn in the graph at capture")
                dsts.append(dst)
                srcs.append(src)
        if dsts and all(x.is_cuda and x.device == d.device and x.dtype == d.dtype and x.shape == d.shape
                        for d, x in zip(dsts, srcs)):
            torch._foreach_copy_(dsts, srcs)  # one launch for all the static inputs
        else:
            for d, x in zip(dsts, srcs):
                d.copy_(x)
        if self._predraw and t_rand is None:
            self._draw()
        self._check_bound()
        opt = self.trainer.optimizer
        group = opt.param_groups[0]
        b1, b2 = group["betas"]
        states = self._step_states()
        nxt = self._common_step() + 1
        a, b = ops.adam_sched_values(group["lr"], b1, b2, nxt)
        slot = self._k % len(self._ring_ev)
        if self._ring_ev[slot] is not None:
            self._ring_ev[slot].synchronize()
        self._ring[slot, 0], self._ring[slot, 1] = a, b  # fp32 rounding, as the host path's
        self.sched.copy_(self._ring[slot], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._ring_ev[slot] = ev
        self._k += 1
        self.graph.replay()
        for st in states:
            st["step"] += 1
        self.trainer.scheduler.step()
        return self.out


class PoseTrainer:
    """The joint pose-optimisation step without host synchronisation (BASELINE cfg #3).

    Mirrors ``train_step_with_poses`` of the reference (noisy_src/train_pose_opt.py:290-411)
    plus the two ``scheduler.step()`` of its loop (:876-880): all poses from the SE(3)
    kernel, the batch's rays from (image, pixel) and those poses, render coarse+fine, MSE
    losses plus the pose regulariser (0.01 mean w^2 + 0.001 mean dt^2, :377-389, weights
    :621-622), backward, separate clips (coarse 1.0, fine 1.0, poses 0.1, :398-404) fused
    into the Adams, the pose Adam and its LambdaLR only once ``optimize_poses``.  The
    reference's ``.item()`` metrics are left to the caller (losses stay on the device).
    Data parallel: the network gradients all-reduce as in ``Trainer``; the pose gradient
    (each rank touches its own images) is one more all-reduce of 2 x 3 x n_poses floats.
    Every gradient is AVERAGED over the ranks: each rank's loss is the mean over its
    equal share of the global batch plus the replicated pose regulariser, so the mean
    of the rank gradients is the single-process gradient.  The 1/world
    rides in the backward seed (the MSE kernels' gradient scale and the regulariser's
    factor), so the all-reduced SUM is that mean without a multiply per buffer.
    Before the pose-optimisation delay (``optimize_poses=False``) the poses enter the
    step detached: the reference lets their gradient accumulate unused until the first
    optimising step's ``zero_grad``, so skipping it changes
    nothing and saves the MLP's input-gradient pass."""

    def __init__(self, model_coarse, model_fine, camera_params, pixel_sampler, render_config,
                 lr: float = 5e-4, pose_lr: float = 1e-4, lr_decay: int = 250,
                 rotation_reg_weight: float = 0.01, translation_reg_weight: float = 0.001, process_group=None):
        self.model_coarse, self.model_fine = model_coarse, model_fine
        self.camera_params, self.pixel_sampler, self.render_config = camera_params, pixel_sampler, render_config
        self.coarse = list(model_coarse.parameters())
        self.fine = list(model_fine.parameters()) if model_fine is not None else []
        self.poses = list(camera_params.parameters())
        self.rot_w, self.trans_w = rotation_reg_weight, translation_reg_weight
        self.optimizer_nerf = FusedAdam(self.coarse + self.fine, lr=lr)
        self.optimizer_poses = FusedAdam(self.poses, lr=pose_lr) if self.poses else None
        lam = lr_lambda_factory(lr_decay)
        self.scheduler_nerf = torch.optim.lr_scheduler.LambdaLR(self.optimizer_nerf, lam)
        self.scheduler_poses = (torch.optim.lr_scheduler.LambdaLR(self.optimizer_poses, lam)
                                if self.optimizer_poses is not None else None)
        self.reducer = None
        if process_group is not None:
            self.reducer = GradAllReducer(process_group, average=False)
            for net in (model_coarse, model_fine):
                if net is not None:
                    net._grad_ready_hook = self.reducer.launch

    def step(self, pixel_batch, optimize_poses: bool = True, t_rand: Optional[torch.Tensor] = None,
             u: Optional[torch.Tensor] = None) -> Dict[str, torch.Tensor]:
        cam = self.camera_params
        optimize_poses = optimize_poses and self.optimizer_poses is not None
        self.optimizer_nerf.zero_grad(set_to_none=True)
        if optimize_poses:
            self.optimizer_poses.zero_grad(set_to_none=True)
        poses = cam.get_all_poses()
        if not optimize_poses:
            poses = poses.detach()
        rays_o, rays_d = self.pixel_sampler.get_rays_for_batch(pixel_batch, poses)
        target = pixel_batch.target_rgb
        gs = self.reducer.prescale if self.reducer is not None else 1.0  # DP: 1/world in the seed
        # the MSE losses (train_pose_opt.py:355-370) come out of the compositing
        out = render_rays(self.model_coarse, self.model_fine, rays_o, rays_d, self.render_config, is_train=True,
                          t_rand=t_rand, u=u, target_rgb=target, loss_scale=gs)
        loss_c = out["loss_coarse"]
        loss = loss_c
        metrics = {"loss_coarse": loss_c.detach()}  # metrics hold no autograd graph
        if "loss_fine" in out:
            loss_f = out["loss_fine"]
            loss = loss_c + loss_f
            metrics["loss_fine"] = loss_f.detach()
        bwd = loss
        if optimize_poses:
            # the regulariser is replicated on every rank: its gradient carries the seed's
            # 1/world too, so the SUM over the ranks counts it once
            reg = []
            if self.rot_w > 0 and cam.learn_rotation:
                reg.append(self.rot_w * torch.mean(cam.rotation_deltas ** 2))
            if self.trans_w > 0 and cam.learn_translation:
                reg.append(self.trans_w * torch.mean(cam.translation_deltas ** 2))
            for r in reg:
                loss = loss + r
                bwd = bwd + (r * gs if gs != 1.0 else r)
        bwd.backward(ops.unit_grad(loss.device))
        if self.reducer is not None:
            flats = [flat for _, flat in self.reducer.pending]
            pg = [p.grad for p in self.poses if p.grad is not None] if optimize_poses else []
            pflat = torch.cat([g.reshape(-1) for g in pg]) if pg else None
            if pflat is not None:
                self.reducer.launch(pflat)
            self.reducer.finish()
            for net in (self.model_coarse, self.model_fine):
                if net is not None:
                    _adopt_reduced_grad(net, flats)
            off = 0
            for g in pg:
                g.copy_(pflat[off:off + g.numel()].view(g.shape))
                off += g.numel()
        groups = [(self.coarse, 1.0)] + ([(self.fine, 1.0)] if self.fine else [])
        self.optimizer_nerf.step(clip_groups=groups)
        self.scheduler_nerf.step()
        if optimize_poses:
            self.optimizer_poses.step(clip_groups=[(self.poses, 0.1)])
            self.scheduler_poses.step()
        metrics["loss"] = loss.detach()
        metrics["rgb_fine"] = out.get("rgb_fine", out["rgb_coarse"]).detach()
        return metrics


def _adopt_reduced_grad(net, flats) -> None:
    """The MLP backward hands autograd views of its flat gradient, which AccumulateGrad
    normally adopts as ``.grad``; if it copied them instead, copy the reduced values."""
    from .optim import _contiguous_run
    g = _contiguous_run([p.grad for p in net.parameters()])
    if g is not None and any(g.data_ptr() == f.data_ptr() for f in flats):
        return
    # this net's own flat gradient (the coarse and fine nets have equal sizes, and with a
    # coarse stream the coarse all-reduce may be launched first)
    last = getattr(net, "_last_gflat", None)
    mine = [f for f in flats if last is not None and f.data_ptr() == last.data_ptr()]
    for f in mine or flats:
        if f.numel() == net._param_count:
            off = 0
            for p in net.parameters():
                n = p.numel()
                p.grad.copy_(f[off:off + n].view(p.shape))
                off += n
            del flats[next(i for i, x in enumerate(flats) if x is f)]  # by identity (== is elementwise)
            return


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
