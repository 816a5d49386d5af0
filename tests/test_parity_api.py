"""GPU parity of the reference-level entry points built on the HIP path:
train.train_step / render_image, data.RayDataset / RaySampler,
data_pose_opt.PixelDataset / PixelSampler and train_pose_opt.CameraPoseParameters /
train_step_with_poses, each against the oracle composition of the reference code."""
from pathlib import Path

import numpy as np
import pytest
import torch

from oracle import refimpl as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
GOLDEN = Path(__file__).resolve().parent / "golden"


def _gt_poses():
    return torch.from_numpy(np.load(sorted(GOLDEN.glob("final_poses_*.npz"))[0])["ground_truth_poses"])


def _nets(seed=0):
    from noisy_src.config import ModelConfig
    from noisy_src.model import create_nerf
    cfg = ModelConfig(precision="fp32")
    torch.manual_seed(seed)
    oc, of = ref.create_nerf(cfg)
    mc, mf = create_nerf(cfg)
    mc.load_state_dict(oc.state_dict())
    mf.load_state_dict(of.state_dict())
    return oc, of, mc.to(DEV), mf.to(DEV)


def test_ray_dataset_and_epoch_sampler():
    """RayDataset rays equal get_rays of every image (data.py:202-240); one epoch of the
    RaySampler visits every ray exactly once (data.py:285-309)."""
    from noisy_src.data import RayDataset, RaySampler, synthetic_blender_data
    poses = _gt_poses()[:3]
    data = synthetic_blender_data(poses, H=12, W=10, device=DEV)
    ds = RayDataset(data)
    dirs = ref.get_ray_directions(12, 10, data.focal)
    for i in range(3):
        o, d = ref.get_rays(dirs, poses[i])
        assert (ds.rays_o[i * 120:(i + 1) * 120].cpu() - o.reshape(-1, 3)).abs().max() < 1e-6
        assert (ds.rays_d[i * 120:(i + 1) * 120].cpu() - d.reshape(-1, 3)).abs().max() < 1e-6
    sampler = RaySampler(ds, batch_size=64)
    seen = torch.cat([b["target_rgb"] for b in sampler])
    assert seen.shape[0] == 360 and len(sampler) == 6
    want = ds.colors.cpu()
    assert torch.equal(torch.sort(seen.cpu().sum(1))[0], torch.sort(want.sum(1))[0])
    assert sampler.sample_batch()["rays_o"].shape == (64, 3)


def test_pixel_dataset_rays_match_reference_loop():
    """PixelSampler.get_rays_for_batch (one gather kernel) == the reference's per-unique-
    image loop (data_pose_opt.py:83-148, oracle get_rays_from_pixels); PixelDataset's
    unique-pose form agrees with it."""
    from noisy_src.data import synthetic_blender_data
    from noisy_src.data_pose_opt import PixelDataset, PixelSampler
    poses = _gt_poses()[:5]
    data = synthetic_blender_data(poses, H=20, W=16, device=DEV)
    ds = PixelDataset(data)
    sampler = PixelSampler(ds, batch_size=300)
    torch.manual_seed(3)
    batch = sampler.sample_batch()
    o, d = sampler.get_rays_for_batch(batch, data.poses)
    ro, rd = ref.get_rays_from_pixels(batch.image_indices.cpu(), batch.pixel_coords.cpu(), poses, 20, 16, data.focal)
    assert (o.cpu() - ro).abs().max() < 1e-6 and (d.cpu() - rd).abs().max() < 1e-6
    uniq = torch.unique(batch.image_indices)
    o2, d2 = ds.get_rays_from_pixels(batch, data.poses[uniq])
    assert torch.equal(o2, o) and torch.equal(d2, d)
    assert torch.equal(batch.target_rgb, data.images.reshape(-1, 3)[
        batch.image_indices * 320 + batch.pixel_coords[:, 1].long() * 16 + batch.pixel_coords[:, 0].long()])


def test_axis_angle_to_rotation_matrix():
    """train_pose_opt.py:122-163 incl. the theta < 1e-6 -> I rule."""
    from noisy_src.train_pose_opt import CameraPoseParameters
    g = torch.Generator().manual_seed(0)
    aa = torch.randn(7, 3, generator=g) * 0.3
    aa[2] = 0.0
    aa[3] = 1e-8
    cam = CameraPoseParameters(_gt_poses()[:2].to(DEV))
    got = cam.axis_angle_to_rotation_matrix(aa.to(DEV)).cpu()
    want = ref.CameraPoseParameters(_gt_poses()[:2]).axis_angle_to_rotation_matrix(aa)
    assert (got - want).abs().max() < 1e-6


def test_train_step_api_matches_oracle():
    """train.train_step(renderer, optimizer, batch) (train.py:68-119) with the fused Adam
    and with torch's Adam, vs the oracle step."""
    from noisy_src.config import RenderConfig
    from noisy_src.optim import FusedAdam
    from noisy_src.rendering import NeRFRenderer
    from noisy_src.train import train_step
    rc = RenderConfig()
    g = torch.Generator().manual_seed(5)
    poses = _gt_poses()
    dirs = ref.get_ray_directions(40, 40, 44.4).reshape(-1, 3)
    o, d = ref.get_rays(dirs[torch.randint(0, 1600, (256,), generator=g)], poses[0])
    tgt = torch.rand(256, 3, generator=g)
    tr, u = torch.rand(256, 64, generator=g), torch.rand(256, 128, generator=g)
    for opt_kind in ("fused", "torch"):
        oc, of, mc, mf = _nets()
        state = ref.TrainState(oc, of)
        renderer = NeRFRenderer(mc, mf, rc)
        opt = FusedAdam(renderer.parameters(), lr=5e-4) if opt_kind == "fused" else \
            torch.optim.Adam(renderer.parameters(), lr=5e-4)
        batch = {"rays_o": o.to(DEV), "rays_d": d.to(DEV), "target_rgb": tgt.to(DEV)}
        for _ in range(2):
            want = ref.train_step(oc, of, state, o, d, tgt, rc, t_rand=tr, u=u)
            got = train_step(renderer, opt, batch, t_rand=tr.to(DEV), u=u.to(DEV))
            assert abs(got["loss"] - want["loss"]) < 1e-5, opt_kind
            assert set(got) >= {"loss", "loss_coarse", "loss_fine", "psnr", "psnr_coarse", "psnr_fine"}


def test_train_step_with_poses_matches_oracle():
    """train_pose_opt.train_step_with_poses (train_pose_opt.py:290-411): rays from the
    learnable poses, L2 pose regularisers, separate clips (1.0 / 1.0 / 0.1), NeRF and pose
    Adams.  Two steps vs the oracle composition; rotation deltas never move."""
    from noisy_src.config import RenderConfig
    from noisy_src.data import synthetic_blender_data
    from noisy_src.data_pose_opt import PixelDataset, PixelSampler
    from noisy_src.optim import FusedAdam
    from noisy_src.train_pose_opt import CameraPoseParameters, train_step_with_poses
    rc = RenderConfig()
    init = _gt_poses()[:4]
    init = init.clone()
    init[:, :3, 3] += 0.05  # a noisy start
    data = synthetic_blender_data(init, H=24, W=24, device=DEV)
    sampler = PixelSampler(PixelDataset(data), batch_size=256)
    oc, of, mc, mf = _nets()
    cam = CameraPoseParameters(init.to(DEV))
    ocam = ref.CameraPoseParameters(init.clone())
    opt_n = FusedAdam(list(mc.parameters()) + list(mf.parameters()), lr=5e-4)
    opt_p = FusedAdam(cam.parameters(), lr=1e-4)
    oopt_n = torch.optim.Adam(list(oc.parameters()) + list(of.parameters()), lr=5e-4)
    oopt_p = torch.optim.Adam(ocam.parameters(), lr=1e-4)
    for step in range(2):
        torch.manual_seed(20 + step)
        batch = sampler.sample_batch()
        g = torch.Generator().manual_seed(30 + step)
        tr, u = torch.rand(256, 64, generator=g), torch.rand(256, 128, generator=g)
        got = train_step_with_poses(mc, mf, cam, sampler, opt_n, opt_p, batch, rc, optimize_poses=True,
                                    rotation_reg_weight=0.01, translation_reg_weight=0.001,
                                    t_rand=tr.to(DEV), u=u.to(DEV))
        # oracle composition of the same step
        oopt_n.zero_grad()
        oopt_p.zero_grad()
        ro, rd = ref.get_rays_from_pixels(batch.image_indices.cpu(), batch.pixel_coords.cpu(), ocam.get_all_poses(),
                                          24, 24, data.focal)
        out = ref.render_rays(oc, of, ro, rd, rc, t_rand=tr, u=u)
        t = batch.target_rgb.cpu()
        loss = ((out["rgb_coarse"] - t) ** 2).mean() + ((out["rgb_fine"] - t) ** 2).mean()
        loss = loss + 0.01 * (ocam.rotation_deltas ** 2).mean() + 0.001 * (ocam.translation_deltas ** 2).mean()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(oc.parameters(), 1.0)
        torch.nn.utils.clip_grad_norm_(of.parameters(), 1.0)
        torch.nn.utils.clip_grad_norm_(ocam.parameters(), 0.1)
        oopt_n.step()
        oopt_p.step()
        assert abs(got["loss"] - loss.item()) < 1e-5, step
    assert torch.count_nonzero(cam.rotation_deltas.detach()) == 0
    dt = cam.translation_deltas.detach().cpu()
    want = ocam.translation_deltas.detach()
    # Adam normalises each coordinate (step 1 moves every one by exactly lr*sign(g)), so
    # fp32 differences in small per-image pose gradients show up as ~1 % of the step
    assert ((dt - want).norm() / want.norm()).item() < 0.03
    assert dt.abs().max() > 1e-5  # translations did move


def test_render_image_matches_render_rays():
    """train.render_image (train.py:122-160) == the oracle's deterministic render of
    every pixel; evaluate() returns finite metrics."""
    from noisy_src.config import RenderConfig
    from noisy_src.data import synthetic_blender_data
    from noisy_src.rendering import NeRFRenderer
    from noisy_src.train import evaluate, render_image
    rc = RenderConfig()
    oc, of, mc, mf = _nets()
    pose = _gt_poses()[7]
    got = render_image(NeRFRenderer(mc, mf, rc), pose.to(DEV), 12, 10, 13.0, chunk_size=50)
    dirs = ref.get_ray_directions(12, 10, 13.0)
    o, d = ref.get_rays(dirs, pose)
    with torch.no_grad():
        want = ref.render_rays(oc, of, o.reshape(-1, 3), d.reshape(-1, 3), rc, is_train=False)
    assert (got["rgb"].reshape(-1, 3).cpu() - want["rgb_fine"]).abs().max() < 1e-4
    assert (got["acc"].reshape(-1).cpu() - want["acc_fine"]).abs().max() < 1e-4
    val = synthetic_blender_data(_gt_poses()[:2], H=12, W=10, device=DEV)
    m = evaluate(NeRFRenderer(mc, mf, rc), val, num_images=2)
    assert np.isfinite(m.psnr) and 0 < m.ssim <= 1 and len(m.per_image_psnr) == 2


def test_pose_trainer_matches_train_step_with_poses():
    """engine.PoseTrainer (the sync-free cfg #3 step bench.py --pose-opt times) performs
    the same update as train_pose_opt.train_step_with_poses + its schedulers."""
    from noisy_src.config import RenderConfig
    from noisy_src.data import synthetic_blender_data
    from noisy_src.data_pose_opt import PixelDataset, PixelSampler
    from noisy_src.engine import PoseTrainer, lr_lambda_factory
    from noisy_src.optim import FusedAdam
    from noisy_src.train_pose_opt import CameraPoseParameters, train_step_with_poses
    rc = RenderConfig()
    init = _gt_poses()[:4].clone()
    init[:, :3, 3] += 0.05
    data = synthetic_blender_data(init, H=24, W=24, device=DEV)
    sampler = PixelSampler(PixelDataset(data), batch_size=256)
    _, _, mc_a, mf_a = _nets()
    _, _, mc_b, mf_b = _nets()
    cam_a, cam_b = CameraPoseParameters(init.to(DEV)), CameraPoseParameters(init.to(DEV))
    opt_n = FusedAdam(list(mc_a.parameters()) + list(mf_a.parameters()), lr=5e-4)
    opt_p = FusedAdam(cam_a.parameters(), lr=1e-4)
    sch_n = torch.optim.lr_scheduler.LambdaLR(opt_n, lr_lambda_factory(250))
    sch_p = torch.optim.lr_scheduler.LambdaLR(opt_p, lr_lambda_factory(250))
    trainer = PoseTrainer(mc_b, mf_b, cam_b, sampler, rc)
    for step in range(3):
        now = step >= 1  # the first step stands for the pose-opt delay
        batch = sampler.sample_batch(generator=torch.Generator(device=DEV).manual_seed(40 + step))
        g = torch.Generator().manual_seed(50 + step)
        tr, u = torch.rand(256, 64, generator=g).to(DEV), torch.rand(256, 128, generator=g).to(DEV)
        got = train_step_with_poses(mc_a, mf_a, cam_a, sampler, opt_n, opt_p if now else None, batch, rc,
                                    optimize_poses=now, rotation_reg_weight=0.01 if now else 0.0,
                                    translation_reg_weight=0.001 if now else 0.0, t_rand=tr, u=u)
        sch_n.step()
        if now:
            sch_p.step()
        m = trainer.step(batch, optimize_poses=now, t_rand=tr, u=u)
        assert abs(float(m["loss"]) - got["loss"]) < 1e-6, step
    assert torch.equal(mc_a.flat_params(), mc_b.flat_params())
    assert torch.equal(mf_a.flat_params(), mf_b.flat_params())
    # the pose gradient is a fixed-order segmented reduction: bit-identical
    assert torch.equal(cam_a.translation_deltas.detach(), cam_b.translation_deltas.detach())
    assert cam_b.translation_deltas.detach().abs().max() > 1e-6
    assert opt_p.param_groups[0]["lr"] == trainer.optimizer_poses.param_groups[0]["lr"]
