"""GPU parity at the BENCHMARKED sizes (VERDICT r1 "parity never runs at the benchmarked
size"): one full training step of the HIP engine vs the oracle (the reference's
algorithm, oracle/refimpl.py) run through torch on the same GPU, on identical rays,
weights and injected random draws (t_rand, u).

* cfg #2: lego 800x800 rays, 4096 rays, 64c+128f, bf16 MFMA (fine M = 786,432).  The
  oracle runs the reference algorithm through ``refimpl.MfmaEmulatedNeRF``, a value-by-value
  model of the 16-bit arithmetic (16-bit MFMA operands, fp32 accumulation, fp32 heads,
  16-bit dz storage), so that only summation order differs;
* cfg #5: 4096 rays, 128c+256f, fp16 MFMA (fine M = 1,572,864; sample_hier_kernel<6>);
* cfg #3: the joint pose-optimisation step at 4096 rays, bf16, SE(3) translation grads;
* cfg #1: coarse-only 64 samples, 256 rays, fp32 (the reference's own numerics).

Compared: rgb_coarse / rgb_fine maps, both losses, and the flat gradient of each network
captured inside ``Trainer.step`` right before the fused clip + Adam (relative L2 error).
Weights: the reference's nn.Linear init with the sigma-head bias set to +1 (a field with
positive density, like a trained one).  At the bare init on random targets the fine net
is nearly inactive: sigma = relu(.) sits within ~1e-9 of the kink for many samples, and
the reference's last interval delta = 1e10 (rendering.py:67-72) turns that into
dL/dsigma ~ 1e10 exp(-1e10 sigma) -- a gradient decided by the last bits of a
near-zero sum, which no two summation orders agree on (fine-net gradient norm 4e-5 vs
0.3 for the coarse net; 18 % apart between the bf16 kernels and the bf16 model, 60 %
between the fp32 reference and its own bf16 rounding).  The fp32 kernels still match the
fp32 oracle there to 1.2e-5 (test_cfg2_fp32_step_4096 uses the bare init).
Tolerances: 16-bit configs 2e-3 relative on gradients, maps 1e-4 abs; fp32 1e-3 / 1e-5.
The drift of the 16-bit step from the plain fp32 oracle (the reference's own arithmetic)
is bounded too: by its recorded value (profiles/r02_fullsize_parity.jsonl,
r03_v2_parity.jsonl; unchanged since) times a 1.5 margin, so a change that makes the 16-bit
path less accurate fails even when it stays self-consistent with the numerics model.
Measured errors are printed and, with NR_PARITY_OUT set, appended there as JSON lines.
"""
import json
import math
import os
from pathlib import Path

import numpy as np
import pytest
import torch

from oracle import refimpl as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
ROOT = Path(__file__).resolve().parents[1]
GOLDEN = ROOT / "tests" / "golden"


def _record(name, rec):
    print(name, json.dumps(rec))
    out = os.environ.get("NR_PARITY_OUT")
    if out:
        with open(out, "a") as fh:
            fh.write(json.dumps({"test": name, **rec}) + "\n")


def _lego_rays(B, seed):
    """Rays of the lego 800x800 training cameras (the reference's GT pose fixture)."""
    g = torch.Generator().manual_seed(seed)
    poses = torch.from_numpy(np.load(sorted(GOLDEN.glob("final_poses_*.npz"))[0])["ground_truth_poses"])
    H = W = 800
    focal = 0.5 * W / math.tan(0.5 * 0.6911112070083618)
    dirs = ref.get_ray_directions(H, W, focal).reshape(-1, 3)
    img = torch.randint(0, 100, (B,), generator=g)
    pix = torch.randint(0, H * W, (B,), generator=g)
    d = torch.einsum("bij,bj->bi", poses[img, :3, :3], dirs[pix])
    d = d / d.norm(dim=-1, keepdim=True)
    return poses[img, :3, 3].contiguous().to(DEV), d.to(DEV), torch.rand(B, 3, generator=g).to(DEV)


def _nets(precision, seed=0, sigma_bias=1.0):
    """(oracle coarse, oracle fine, HIP coarse, HIP fine, fp32 oracle coarse, fine): the
    oracle nets are the numerics model of ``precision`` over the fp32 oracle weights.
    ``sigma_bias`` (None: the bare init) is written into both sigma heads."""
    from noisy_src.config import ModelConfig
    from noisy_src.model import create_nerf
    cfg = ModelConfig(precision=precision)
    torch.manual_seed(seed)
    oc, of = ref.create_nerf(cfg)
    if sigma_bias is not None:
        with torch.no_grad():
            for n in (oc, of):
                n.sigma_linear.bias.fill_(sigma_bias)
    mc, mf = create_nerf(cfg)
    mc.load_state_dict(oc.state_dict())
    mf.load_state_dict(of.state_dict())
    oc, of = oc.to(DEV), of.to(DEV)
    if precision == "fp32":
        return oc, of, mc.to(DEV), mf.to(DEV), oc, of
    return (ref.mfma_emulated_nerf(oc, precision), ref.mfma_emulated_nerf(of, precision), mc.to(DEV), mf.to(DEV),
            oc, of)


def _flat_grad(net):
    return torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1) for p in net.parameters()])


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


def _capture_grads(optimizer, nets, store):
    """Wrap optimizer.step so the flat network gradients are captured right before it."""
    orig = optimizer.step

    def step(*a, **k):
        store.extend(_flat_grad(n).clone() for n in nets if n is not None)
        return orig(*a, **k)

    optimizer.step = step


def _train_step_parity(name, precision, Nc, Nf, B, hierarchical=True, seed=0, sigma_bias=1.0):
    from noisy_src.config import RenderConfig
    from noisy_src.engine import Trainer
    from noisy_src.rendering import render_rays
    rc = RenderConfig(num_samples=Nc, num_samples_fine=Nf, use_hierarchical=hierarchical)
    oc, of, mc, mf, pc, pf = _nets(precision, seed, sigma_bias)
    if not hierarchical:
        of = mf = pf = None
    o, d, tgt = _lego_rays(B, 100 + seed)
    g = torch.Generator(device=DEV).manual_seed(200 + seed)
    tr = torch.rand(B, Nc, device=DEV, generator=g)
    u = torch.rand(B, Nf, device=DEV, generator=g)

    # oracle: the reference's train_step math through torch on the GPU
    want = ref.render_rays(oc, of, o, d, rc, is_train=True, t_rand=tr, u=u)
    loss_c = torch.mean((want["rgb_coarse"] - tgt) ** 2)
    loss = loss_c
    if hierarchical:
        loss_f = torch.mean((want["rgb_fine"] - tgt) ** 2)
        loss = loss + loss_f
    loss.backward()
    want_g = [_flat_grad(oc)] + ([_flat_grad(of)] if hierarchical else [])
    drift = None
    if precision != "fp32":  # the same step in the reference's own fp32 arithmetic
        for n in (pc, pf):
            if n is not None:
                n.zero_grad(set_to_none=True)
        w32 = ref.render_rays(pc, pf, o, d, rc, is_train=True, t_rand=tr, u=u)
        l32 = torch.mean((w32["rgb_coarse"] - tgt) ** 2)
        if hierarchical:
            l32 = l32 + torch.mean((w32["rgb_fine"] - tgt) ** 2)
        l32.backward()
        drift = {"g32": [_flat_grad(pc)] + ([_flat_grad(pf)] if hierarchical else []), "w32": w32}

    with torch.no_grad():
        got = render_rays(mc, mf, o, d, rc, is_train=True, t_rand=tr, u=u)
    trainer = Trainer(mc, mf, rc)
    grads = []
    _capture_grads(trainer.optimizer, (mc, mf), grads)
    m = trainer.step(o, d, tgt, t_rand=tr, u=u)
    rec = {"precision": precision, "Nc": Nc, "Nf": Nf, "rays": B, "sigma_bias": sigma_bias,
           "M_fine": B * (Nc + Nf) if hierarchical else 0,
           "loss_rel": abs(m["loss"].item() - loss.item()) / loss.item()}
    keys = ["rgb_coarse"] + (["rgb_fine"] if hierarchical else [])
    for k in keys:
        diff = (got[k] - want[k].detach()).abs()
        rec[f"{k}_max_abs"] = diff.max().item()
        rec[f"{k}_mean_abs"] = diff.mean().item()
    rec["grad_rel"] = [_rel(a, b) for a, b in zip(grads, want_g)]
    rec["grad_norm"] = [b.norm().item() for b in want_g]
    # per-tensor relative error of the last network's gradient (diagnostic)
    net, wg = (mf, want_g[-1]) if hierarchical else (mc, want_g[0])
    off, per = 0, {}
    for (pname, prm) in net.named_parameters():
        k = prm.numel()
        per[pname] = round(_rel(grads[-1][off:off + k], wg[off:off + k]), 6)
        off += k
    rec["last_net_per_param_rel"] = per
    if hierarchical:
        rec["rgb_fine_trainer_vs_render"] = (m["rgb_fine"] - got["rgb_fine"]).abs().max().item()
    if drift is not None:
        rec["vs_fp32_oracle"] = {"grad_rel": [_rel(a, b) for a, b in zip(grads, drift["g32"])],
                                 **{f"{k}_max_abs": (got[k] - drift["w32"][k].detach()).abs().max().item()
                                    for k in keys}}
    _record(name, rec)
    return rec


def _assert(rec, map_tol, grad_tol, loss_tol):
    assert rec["loss_rel"] < loss_tol, rec
    for k, v in rec.items():
        if k.endswith("_max_abs"):
            assert v < map_tol, (k, v)
    for r in rec["grad_rel"]:
        assert r < grad_tol, rec["grad_rel"]
    if "rgb_fine_trainer_vs_render" in rec:
        assert rec["rgb_fine_trainer_vs_render"] == 0.0  # the step's forward is the render's forward


# recorded drift of the 16-bit step from the fp32 oracle (gradient relative L2 of the
# coarse / fine nets, rgb maps max abs) and the 1.5x margin it is held to
DRIFT_MARGIN = 1.5
DRIFT_RECORDED = {
    "cfg2": {"grad_rel": (2.006e-3, 1.844e-3), "rgb_max_abs": 1.038e-4},
    "cfg5": {"grad_rel": (3.958e-4, 3.190e-4), "rgb_max_abs": 1.448e-5},
    "cfg4": {"grad_rel": (4.219e-3, 3.623e-3), "rgb_max_abs": 9.221e-5},
}


def _assert_drift(rec, cfg):
    """The 16-bit step's distance from the fp32 oracle stays within DRIFT_MARGIN of the
    recorded one (a precision regression fails here)."""
    ref_d, got = DRIFT_RECORDED[cfg], rec["vs_fp32_oracle"]
    for g, r in zip(got["grad_rel"], ref_d["grad_rel"]):
        assert g < DRIFT_MARGIN * r, (cfg, got, ref_d)
    for k in ("rgb_coarse_max_abs", "rgb_fine_max_abs"):
        assert got[k] < DRIFT_MARGIN * ref_d["rgb_max_abs"], (cfg, k, got, ref_d)


def test_cfg2_fullsize_bf16_step():
    rec = _train_step_parity("cfg2_bf16_4096x(64+128)", "bf16", 64, 128, 4096)
    assert rec["M_fine"] == 786432
    _assert(rec, map_tol=1e-4, grad_tol=2e-3, loss_tol=1e-5)
    _assert_drift(rec, "cfg2")


def test_cfg5_fullsize_fp16_step():
    rec = _train_step_parity("cfg5_fp16_4096x(128+256)", "fp16", 128, 256, 4096)
    assert rec["M_fine"] == 1572864
    _assert(rec, map_tol=1e-4, grad_tol=2e-3, loss_tol=1e-5)
    _assert_drift(rec, "cfg5")


def test_cfg1_coarse_only_fp32_step():
    rec = _train_step_parity("cfg1_fp32_256x64_coarse_only", "fp32", 64, 128, 256, hierarchical=False)
    _assert(rec, map_tol=1e-5, grad_tol=1e-4, loss_tol=1e-5)


def test_cfg2_fp32_step_4096():
    """The fp32 parity mode at the benchmarked batch (north star: rgb within 1e-4 abs)."""
    rec = _train_step_parity("cfg2_fp32_4096x(64+128)", "fp32", 64, 128, 4096, sigma_bias=None)
    _assert(rec, map_tol=1e-4, grad_tol=1e-3, loss_tol=1e-5)


def test_cfg2_fp32_step_4096_active_fine_net():
    """the fp32 parity mode at the benchmarked batch with the sigma-head
    bias at +1, so the fine net is active (at the bare init its gradient norm is ~3e-5
    and the comparison degenerate): both networks' gradients within 1e-3 relative of the
    fp32 oracle, with a fine-net gradient norm of at least 1e-3."""
    rec = _train_step_parity("cfg2_fp32_4096x(64+128)_active", "fp32", 64, 128, 4096, sigma_bias=1.0)
    assert rec["grad_norm"][1] >= 1e-3, rec["grad_norm"]
    _assert(rec, map_tol=1e-4, grad_tol=1e-3, loss_tol=1e-5)


def test_cfg4_per_rank_bf16_step_512():
    """BASELINE cfg #4's strong-scaling per-rank workload -- 512 rays of
    the 4096-ray global batch on each of 8 GPUs, coarse M = 32,768, fine M = 98,304 (the
    size that may not fill 256 CUs) -- one bf16 training step vs the numerics model."""
    rec = _train_step_parity("cfg4_rank_bf16_512x(64+128)", "bf16", 64, 128, 512)
    assert rec["M_fine"] == 98304
    _assert(rec, map_tol=1e-4, grad_tol=2e-3, loss_tol=1e-5)
    _assert_drift(rec, "cfg4")


def _pose_step(precision):
    """One joint pose-optimisation step at 4096 rays: rays from (image, pixel) and the
    learnable SE(3) poses, render, loss + pose regulariser, backward to the networks AND
    the translation deltas; rotation gradients are exactly 0 (the reference's quirk)."""
    from noisy_src.config import RenderConfig
    from noisy_src.data import synthetic_blender_data
    from noisy_src.data_pose_opt import create_pixel_dataset
    from noisy_src.engine import PoseTrainer
    from noisy_src.train_pose_opt import CameraPoseParameters
    fix = sorted(GOLDEN.glob("final_poses_*rot5.0deg_trans5.0pct_*.npz"))[0]
    z = np.load(fix)
    init = torch.from_numpy(z["initial_poses"])
    data = synthetic_blender_data(torch.from_numpy(z["ground_truth_poses"]), H=800, W=800, device=DEV)
    _, sampler = create_pixel_dataset(data)
    sampler.batch_size = 4096
    batch = sampler.sample_batch(generator=torch.Generator(device=DEV).manual_seed(5))
    rc = RenderConfig()
    oc, of, mc, mf, pc, pf = _nets(precision)
    g = torch.Generator(device=DEV).manual_seed(6)
    tr = torch.rand(4096, 64, device=DEV, generator=g)
    u = torch.rand(4096, 128, device=DEV, generator=g)

    def oracle(c, f, dtype=torch.float32):
        cam_o = ref.CameraPoseParameters(init.to(DEV, dtype)).to(dtype)
        ro, rd = ref.get_rays_from_pixels(batch.image_indices, batch.pixel_coords.to(dtype), cam_o.get_all_poses(),
                                          800, 800, data.focal)
        want = ref.render_rays(c, f, ro, rd, rc, t_rand=tr.to(dtype), u=u.to(dtype))
        t = batch.target_rgb.to(dtype)
        loss = torch.mean((want["rgb_coarse"] - t) ** 2) + torch.mean((want["rgb_fine"] - t) ** 2)
        loss = loss + 0.01 * torch.mean(cam_o.rotation_deltas ** 2) + 0.001 * torch.mean(cam_o.translation_deltas ** 2)
        loss.backward()
        return cam_o, want, loss

    cam_o, want, loss = oracle(oc, of)
    g_model = [_flat_grad(oc), _flat_grad(of)]
    if precision != "fp32":
        for n in (pc, pf):
            n.zero_grad(set_to_none=True)
        cam_32, want32, _ = oracle(pc, pf)
    else:  # the fp64 truth: dL/d(translation) is a sum over ~7.9k samples per image with
        # heavy cancellation, so fp32 implementations are compared by their error vs fp64
        import copy
        c64, f64 = copy.deepcopy(pc).double(), copy.deepcopy(pf).double()
        for n in (c64, f64):
            n.zero_grad(set_to_none=True)
        cam_64, _, _ = oracle(c64, f64, torch.float64)

    cam = CameraPoseParameters(init.to(DEV))
    trainer = PoseTrainer(mc, mf, cam, sampler, rc)
    grads = []
    orig = trainer.optimizer_poses.step

    def pose_step(*a, **k):
        grads.append(cam.translation_deltas.grad.clone())
        grads.append(cam.rotation_deltas.grad.clone())
        return orig(*a, **k)

    trainer.optimizer_poses.step = pose_step
    _capture_grads(trainer.optimizer_nerf, (mc, mf), grads)
    m = trainer.step(batch, optimize_poses=True, t_rand=tr, u=u)
    gc, gf, gt, gr = grads  # the NeRF Adam steps before the pose Adam
    rec = {"precision": precision, "rays": 4096, "loss_rel": abs(m["loss"].item() - loss.item()) / loss.item(),
           "grad_rel": [_rel(gc, g_model[0]), _rel(gf, g_model[1])],
           "trans_grad_rel": _rel(gt, cam_o.translation_deltas.grad),
           "rot_grad_nonzero": int(torch.count_nonzero(gr).item()) + int(torch.count_nonzero(cam_o.rotation_deltas.grad)),
           "rgb_fine_max_abs": (m["rgb_fine"] - want["rgb_fine"].detach()).abs().max().item()}
    if precision == "fp32":
        t64 = cam_64.translation_deltas.grad
        rec["trans_err_hip_vs_fp64"] = _rel(gt, t64)
        rec["trans_err_torch_fp32_vs_fp64"] = _rel(cam_o.translation_deltas.grad, t64)
    if precision != "fp32":
        rec["grad_rel_vs_fp32_oracle"] = [_rel(gc, _flat_grad(pc)), _rel(gf, _flat_grad(pf))]
        rec["rgb_fine_max_abs_vs_fp32_oracle"] = (m["rgb_fine"] - want32["rgb_fine"].detach()).abs().max().item()
        rec["trans_grad_rel_vs_fp32_oracle"] = _rel(gt, cam_32.translation_deltas.grad)
        rec["model_trans_grad_rel_vs_fp32_oracle"] = _rel(cam_o.translation_deltas.grad, cam_32.translation_deltas.grad)
    _record(f"cfg3_pose_opt_{precision}_4096", rec)
    return rec


def test_cfg3_fullsize_pose_opt_step_fp32():
    rec = _pose_step("fp32")
    assert rec["rot_grad_nonzero"] == 0
    assert rec["loss_rel"] < 1e-5 and rec["rgb_fine_max_abs"] < 1e-4
    assert max(rec["grad_rel"]) < 1e-3, rec
    # as close to the fp64 truth as torch's own fp32 evaluation of the reference is
    assert rec["trans_err_hip_vs_fp64"] < 2 * rec["trans_err_torch_fp32_vs_fp64"] + 1e-3, rec


def test_cfg3_fullsize_pose_opt_step_bf16():
    """bf16 (the benchmarked cfg #3 precision).  The network gradients match the numerics
    model like cfg #2; the translation gradient is a sum of dL/dpts over every sample of
    an image, and dL/dpts inherits the 16-bit path's per-sample rounding-boundary flips
    (the hardware-sine positional encoding lands a few x_enc values one bf16 ulp away
    from torch's sin): it must stay well inside the model's own distance from fp32."""
    rec = _pose_step("bf16")
    assert rec["rot_grad_nonzero"] == 0
    assert rec["loss_rel"] < 1e-5 and rec["rgb_fine_max_abs"] < 1e-4
    assert max(rec["grad_rel"]) < 2e-3, rec
    assert rec["trans_grad_rel"] < 3e-2, rec
    assert rec["trans_grad_rel_vs_fp32_oracle"] < 2 * rec["model_trans_grad_rel_vs_fp32_oracle"] + 1e-2, rec
    # drift from the fp32 oracle within DRIFT_MARGIN of the recorded values (translation:
    # 0.0775, profiles/r03_v2_parity.jsonl; networks 2.249e-3 / 1.913e-3 and rgb_fine
    # 1.100e-4: profiles/r06_fullsize_parity.jsonl)
    assert rec["trans_grad_rel_vs_fp32_oracle"] < DRIFT_MARGIN * 0.0775, rec
    for g, r in zip(rec["grad_rel_vs_fp32_oracle"], (2.249e-3, 1.913e-3)):
        assert g < DRIFT_MARGIN * r, rec
    assert rec["rgb_fine_max_abs_vs_fp32_oracle"] < DRIFT_MARGIN * 1.100e-4, rec


def test_eval_render_image_fullsize_800_fp32():
    """VERDICT r2 5 / SURVEY §8f-2: ``train.render_image`` of a WHOLE 800x800 lego view
    (640,000 rays) at the reference's eval chunk of 4096 (train.py:122-160,
    inference.py:75-105; deterministic: det=True, no perturbation), fp32 parity mode, vs
    the oracle's render_rays run through torch on the same GPU chunk by chunk.  North
    star: rendered RGB within 1e-4 abs."""
    from noisy_src.config import RenderConfig
    from noisy_src.rendering import NeRFRenderer
    from noisy_src.train import render_image
    rc = RenderConfig()
    oc, of, mc, mf, _, _ = _nets("fp32", seed=3, sigma_bias=1.0)
    poses = torch.from_numpy(np.load(sorted(GOLDEN.glob("final_poses_*.npz"))[0])["ground_truth_poses"])
    pose = poses[11].to(DEV)
    H = W = 800
    focal = 0.5 * W / math.tan(0.5 * 0.6911112070083618)
    got = render_image(NeRFRenderer(mc, mf, rc), pose, H, W, focal, chunk_size=4096)
    dirs = ref.get_ray_directions(H, W, focal).to(DEV)
    o, d = ref.get_rays(dirs, pose)
    o, d = o.reshape(-1, 3), d.reshape(-1, 3)
    want_rgb, want_acc = [], []
    with torch.no_grad():
        for i in range(0, H * W, 4096):
            w = ref.render_rays(oc, of, o[i:i + 4096], d[i:i + 4096], rc, is_train=False)
            want_rgb.append(w["rgb_fine"])
            want_acc.append(w["acc_fine"])
    want_rgb, want_acc = torch.cat(want_rgb), torch.cat(want_acc)
    err = (got["rgb"].reshape(-1, 3) - want_rgb).abs()
    rec = {"rays": H * W, "rgb_max_abs": err.max().item(), "rgb_mean_abs": err.mean().item(),
           "acc_max_abs": (got["acc"].reshape(-1) - want_acc).abs().max().item(),
           "acc_mean": want_acc.mean().item(), "pixels_over_1e-4": int((err.max(-1).values > 1e-4).sum())}
    _record("eval_render_image_800x800_fp32", rec)
    assert rec["acc_mean"] > 0.05  # the view sees density: a non-trivial image
    assert rec["rgb_max_abs"] < 1e-4, rec
    assert rec["acc_max_abs"] < 1e-4, rec
