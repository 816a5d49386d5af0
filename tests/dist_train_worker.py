"""Worker of tests/test_distributed_gpu.py: the data-parallel Trainer step on the GPU.

Every rank builds the same two networks (seed 42), takes its contiguous slice of one
global batch (SURVEY.md §8e partitioning) and runs the engine.Trainer step whose
per-network gradient all-reduce hooks into the MLP backward.  The ranks share one
GPU here, so the collective is gloo over device tensors (RCCL refuses two ranks on
one device); the hook/launch/finish path is the one bench.py runs over RCCL.
Writes its final flat parameters to <out>/rank<r>.pt.
"""

import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "robust-nerf_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    out = Path(sys.argv[1])
    steps = int(sys.argv[2])
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    pg = None
    if world > 1:
        dist.init_process_group("gloo")
        pg = dist.group.WORLD
    from noisy_src.config import ModelConfig, RenderConfig
    from noisy_src.engine import PoseTrainer, Trainer
    from noisy_src.model import create_nerf
    from bench import lego_rays, pose_opt_setup

    pose_mode = len(sys.argv) > 3 and sys.argv[3] == "pose"
    torch.manual_seed(42)
    mc, mf = create_nerf(ModelConfig(precision="fp32"))
    mc, mf = mc.to(dev), mf.to(dev)
    rc = RenderConfig()
    B = 256
    per = B // world
    sl = slice(rank * per, (rank + 1) * per)
    pose_grads = []
    if pose_mode:
        # joint pose optimisation (cfg #3): the pose gradient is one more all-reduce
        cam, sampler = pose_opt_setup(64, 64, dev)
        trainer = PoseTrainer(mc, mf, cam, sampler, rc, process_group=pg)
        orig = trainer.optimizer_poses.step

        def capture(*a, **k):  # the (all-reduced) pose gradient right before the pose Adam
            pose_grads.append(torch.cat([p.grad.reshape(-1) for p in cam.parameters()]).cpu())
            return orig(*a, **k)

        trainer.optimizer_poses.step = capture
    else:
        trainer = Trainer(mc, mf, rc, process_group=pg)
    # the (all-reduced) flat network gradients right before the first Adam step: Adam is
    # invariant to the gradient's scale, so the parameters alone cannot show a wrong
    # 1/world; the test compares these with one process's gradients
    net_grads = []
    nopt = trainer.optimizer_nerf if pose_mode else trainer.optimizer
    nstep = nopt.step

    def capture_net(*a, **k):
        if not net_grads:
            net_grads.append(torch.cat([p.grad.reshape(-1) for n in (mc, mf) for p in n.parameters()]).cpu())
        return nstep(*a, **k)

    nopt.step = capture_net
    for k in range(steps):
        g = torch.Generator().manual_seed(900 + k)
        tr = torch.rand(B, rc.num_samples, generator=g).to(dev)
        u = torch.rand(B, rc.num_samples_fine, generator=g).to(dev)
        if pose_mode:
            batch = sampler.sample_batch(generator=torch.Generator(device=dev).manual_seed(700 + k))
            trainer.step(batch.slice(sl), optimize_poses=True, t_rand=tr[sl], u=u[sl])
        else:
            o, d, t = lego_rays(B, 500 + k, dev)
            trainer.step(o[sl], d[sl], t[sl], t_rand=tr[sl], u=u[sl])
    torch.cuda.synchronize()
    flat = torch.cat([mc.flat_params().cpu(), mf.flat_params().cpu()])
    if pose_mode:
        flat = torch.cat([flat, torch.cat([p.detach().reshape(-1).cpu() for p in cam.parameters()])])
        torch.save(torch.stack(pose_grads), out / f"pose_grads_rank{rank}_of{world}.pt")
    torch.save(flat, out / f"{'pose_' if pose_mode else ''}rank{rank}_of{world}.pt")
    torch.save(net_grads[0], out / f"{'pose_' if pose_mode else ''}net_grads_rank{rank}_of{world}.pt")
    if pg is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
