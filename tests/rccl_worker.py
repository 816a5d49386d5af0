"""Worker of tests/test_rccl.py: the data-parallel step over RCCL on one MI355X.

Run as ``torch.distributed.run --nproc-per-node=1`` (world 1): the process joins a
backend-"nccl" (= RCCL) group before anything touches the GPU, then checks, for the
bf16 Trainer step, the fp32 PoseTrainer step and the hipGraph-captured Trainer step,
that the step with the all-reduce hooks active (RCCL kernels launched from the MLP
backward) is bit-identical to the step without a process group.
At world 1 the SUM over the group is the identity and the backward seed's 1/world is
1, so any difference is a bug of the DP path, not of summation order.
Writes ``<out>/rccl_report.json``.
"""

import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "robust-nerf_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def _batches(n, B, rc, dev, seed):
    from bench import lego_rays
    out = []
    for k in range(n):
        g = torch.Generator().manual_seed(seed + k)
        tr = torch.rand(B, rc.num_samples, generator=g).to(dev)
        u = torch.rand(B, rc.num_samples_fine, generator=g).to(dev)
        o, d, t = lego_rays(B, seed + 100 + k, dev)
        out.append((o, d, t, tr, u))
    return out


def _nets(precision, dev):
    from noisy_src.config import ModelConfig
    from noisy_src.model import create_nerf
    torch.manual_seed(42)
    mc, mf = create_nerf(ModelConfig(precision=precision))
    return mc.to(dev), mf.to(dev)


def _flat(*nets):
    return torch.cat([n.flat_params() for n in nets]).cpu()


def train_case(pg, dev, precision="bf16", steps=3):
    from noisy_src.config import RenderConfig
    from noisy_src.engine import Trainer
    rc = RenderConfig()
    data = _batches(steps, 512, rc, dev, 900)
    res = {}
    for name, group in (("plain", None), ("rccl", pg)):
        mc, mf = _nets(precision, dev)
        tr = Trainer(mc, mf, rc, process_group=group)
        grads, losses = [], []
        nstep = tr.optimizer.step

        def cap(*a, **k):
            grads.append(torch.cat([p.grad.reshape(-1) for n in (mc, mf) for p in n.parameters()]).cpu())
            return nstep(*a, **k)

        tr.optimizer.step = cap
        for b in data:
            losses.append(float(tr.step(*b)["loss"]))
        torch.cuda.synchronize()
        res[name] = (_flat(mc, mf), torch.stack(grads), losses)
    return {"losses_equal": res["plain"][2] == res["rccl"][2],
            "grads_equal": bool(torch.equal(res["plain"][1], res["rccl"][1])),
            "params_equal": bool(torch.equal(res["plain"][0], res["rccl"][0])),
            "grad_norm": float(res["plain"][1][0].norm())}


def pose_case(pg, dev, steps=2):
    from bench import pose_opt_setup
    from noisy_src.config import RenderConfig
    from noisy_src.engine import PoseTrainer
    rc = RenderConfig()
    res = {}
    for name, group in (("plain", None), ("rccl", pg)):
        mc, mf = _nets("fp32", dev)
        cam, sampler = pose_opt_setup(64, 64, dev)
        sampler.batch_size = 256
        tr = PoseTrainer(mc, mf, cam, sampler, rc, process_group=group)
        for k in range(steps):
            g = torch.Generator().manual_seed(700 + k)
            t_rand = torch.rand(256, rc.num_samples, generator=g).to(dev)
            u = torch.rand(256, rc.num_samples_fine, generator=g).to(dev)
            batch = sampler.sample_batch(generator=torch.Generator(device=dev).manual_seed(800 + k))
            tr.step(batch, optimize_poses=True, t_rand=t_rand, u=u)
        torch.cuda.synchronize()
        res[name] = torch.cat([_flat(mc, mf), torch.cat([p.detach().reshape(-1).cpu() for p in cam.parameters()])])
    return {"params_and_poses_equal": bool(torch.equal(res["plain"], res["rccl"])),
            "poses_moved": float(res["plain"][-600:].abs().max())}


def graph_case(pg, dev, steps=4):
    """GraphedTrainer of a DP trainer: the RCCL all-reduces are captured in the graph;
    the replayed steps equal the eager DP trainer's bit for bit."""
    from noisy_src.config import RenderConfig
    from noisy_src.engine import GraphedTrainer, Trainer
    rc = RenderConfig()
    data = _batches(steps + 1, 512, rc, dev, 300)
    eager = Trainer(*_nets("bf16", dev), rc, process_group=pg)
    mc, mf = _nets("bf16", dev)
    tr = Trainer(mc, mf, rc, process_group=pg)
    try:
        graphed = GraphedTrainer(tr, *data[0], warmup=1)
    except Exception as e:  # noqa: BLE001 -- recorded for the report
        return {"captured": False, "error": f"{type(e).__name__}: {e}"}
    eager.step(*data[0])
    le, lg = [], []
    for b in data[1:]:
        le.append(float(eager.step(*b)["loss"]))
        lg.append(float(graphed.step(*b)["loss"]))
    torch.cuda.synchronize()
    same = bool(torch.equal(_flat(eager.model_coarse, eager.model_fine), _flat(mc, mf)))
    # a replay after the Adam state was replaced must refuse
    tr.optimizer.load_state_dict(tr.optimizer.state_dict())
    try:
        graphed.step(*data[1])
        refused = False
    except RuntimeError:
        refused = True
    return {"captured": True, "losses_equal": le == lg, "params_equal": same, "stale_replay_refused": refused}


def main():
    out = Path(sys.argv[1])
    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    dist.init_process_group("nccl", device_id=dev)  # before any other GPU work
    torch.cuda.set_device(dev)
    pg = dist.group.WORLD
    rep = {"world": world, "backend": dist.get_backend(pg),
           "rccl_version": ".".join(map(str, torch.cuda.nccl.version())) if hasattr(torch.cuda, "nccl") else None}
    # one collective first: RCCL initialises its communicator on it
    t = torch.ones(4, device=dev)
    dist.all_reduce(t)
    rep["allreduce_ok"] = bool(torch.equal(t.cpu(), torch.full((4,), float(world))))
    rep["train_bf16"] = train_case(pg, dev)
    rep["pose_fp32"] = pose_case(pg, dev)
    rep["graph_bf16"] = graph_case(pg, dev)
    if rank == 0:
        (out / "rccl_report.json").write_text(json.dumps(rep, indent=1))
        print(json.dumps(rep))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
