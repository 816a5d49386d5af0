"""The oracle (oracle/refimpl.py) against the reference's own artifacts and
analytic known-answer tests.  CPU only."""
import json
import math
from pathlib import Path
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from oracle import refimpl as ref

GOLDEN = Path(__file__).resolve().parent / "golden"
ART = json.loads((GOLDEN / "reference_artifacts.json").read_text())
RC = SimpleNamespace(near=2.0, far=6.0, num_samples=64, num_samples_fine=128, use_hierarchical=True,
                     perturb=True, raw_noise_std=0.0, white_background=True)


def _final_poses():
    for f in sorted(GOLDEN.glob("final_poses_*.npz")):
        yield f.stem[len("final_poses_"):], dict(np.load(f))


# ---- pins against the reference's run artifacts -------------------------------------------
def test_reference_rotation_never_moves_and_translation_does():
    """outputs/*/final_poses.pt: R_opt == R_init bit for bit in every run (the dead rotation
    gradient of train_pose_opt.py:143-161); t moved in the noisy-translation runs."""
    n = 0
    for run, p in _final_poses():
        assert np.array_equal(p["optimized_poses"][:, :3, :3], p["initial_poses"][:, :3, :3]), run
        if "trans" in run:
            assert np.abs(p["optimized_poses"][:, :3, 3] - p["initial_poses"][:, :3, 3]).max() > 1e-3
        n += 1
    assert n == 5


def test_oracle_pose_error_matches_reference_summary():
    """noise.py:237-268 restated; mean errors of the final poses equal the pickled ones."""
    for run, p in _final_poses():
        gt = torch.from_numpy(p["ground_truth_poses"])
        opt = torch.from_numpy(p["optimized_poses"])
        errs = [ref.compute_pose_error(gt[i], opt[i]) for i in range(100)]
        want = ART["final_poses"][run]["pose_errors"]
        t_mean = float(np.mean([e["translation_error"] for e in errs]))
        r_mean = float(np.mean([e["rotation_error_deg"] for e in errs]))
        assert t_mean == pytest.approx(want["translation_error_mean"], rel=1e-5, abs=1e-7), run
        assert r_mean == pytest.approx(want["rotation_error_mean"], rel=1e-3, abs=2e-3), run


def test_oracle_rotation_gradient_is_dead_at_zero():
    """The oracle CameraPoseParameters reproduces the reference quirk: dL/domega == 0 exactly,
    so Adam leaves R bit-identical (as in every final_poses.pt) while t moves."""
    run, p = next(_final_poses())
    init = torch.from_numpy(p["initial_poses"][:8])
    cam = ref.CameraPoseParameters(init)
    opt = torch.optim.Adam(cam.parameters(), lr=1e-4)
    g = torch.Generator().manual_seed(0)
    img = torch.randint(0, 8, (256,), generator=g)
    pix = torch.stack([torch.randint(0, 40, (256,), generator=g), torch.randint(0, 40, (256,), generator=g)], -1).float()
    for _ in range(3):
        opt.zero_grad()
        o, d = ref.get_rays_from_pixels(img, pix, cam.get_all_poses(), 40, 40, 50.0)
        loss = ((o + 2.0 * d) ** 2).sum() + 0.01 * torch.mean(cam.rotation_deltas ** 2)
        loss.backward()
        assert torch.count_nonzero(cam.rotation_deltas.grad) == 0
        assert torch.count_nonzero(cam.translation_deltas.grad) > 0
        opt.step()
    poses = cam.get_all_poses().detach()
    assert torch.equal(poses[:, :3, :3], init[:, :3, :3])
    assert not torch.equal(poses[:, :3, 3], init[:, :3, 3])


def test_oracle_lr_schedule_matches_logged_lr():
    """train.py:405-411 LambdaLR: the CSV logs lr after scheduler.step() (row 0 = step 1)."""
    for run, info in ART["runs"].items():
        for step, logged in enumerate(info["learning_rate_first_rows"], start=1):
            assert 5e-4 * ref.lr_lambda(step) == pytest.approx(logged, rel=1e-12), run


def test_oracle_param_count_and_flops():
    """summary.json model_coarse_total_params = 595,844; §8d MACs/sample = 593,408."""
    torch.manual_seed(0)
    assert ref.num_params(ref.NeRF()) == 595844
    for info in ART["runs"].values():
        assert info["params_per_net"] == 595844
    assert ref.mlp_flops_per_sample() == 593408


# ---- analytic known-answer tests ------------------------------------------------------------
def test_pe_known_answer():
    pe = ref.PositionalEncoding(10)
    out = pe(torch.zeros(1, 3))
    want = torch.tensor([0.0] * 3 + ([0.0] * 3 + [1.0] * 3) * 10)
    assert torch.equal(out[0], want)
    x = torch.tensor([[0.3, -1.7, 2.5]])
    out = pe(x)[0]
    for k in range(10):
        f = 2.0 ** k
        assert torch.allclose(out[3 + 6 * k: 6 + 6 * k], torch.sin(f * x[0]))
        assert torch.allclose(out[6 + 6 * k: 9 + 6 * k], torch.cos(f * x[0]))


def test_ray_directions_identity_pose():
    d = ref.get_ray_directions(2, 2, 1.0)
    assert torch.equal(d[1, 0], torch.tensor([-1.0, 0.0, -1.0]))  # (i=0,j=1): ((0-1)/1, -(1-1), -1)
    o, rd = ref.get_rays(d, torch.eye(4))
    assert torch.allclose(rd, d / d.norm(dim=-1, keepdim=True))
    assert torch.equal(o, torch.zeros_like(o))


def test_composite_constant_sigma_closed_form():
    B, S, s = 4, 16, 0.7
    z = torch.linspace(2, 6, S).expand(B, S)
    rd = torch.tensor([[0.0, 0.0, -1.0]]).expand(B, 3)
    rgb = torch.rand(B, S, 3)
    out = ref.raw2outputs(rgb, torch.full((B, S, 1), s), z, rd)
    delta = (4.0 / (S - 1))
    a = 1 - math.exp(-s * delta)
    w = [a * (1 - a + 1e-10) ** i for i in range(S - 1)]
    w.append((1.0) * (1 - a + 1e-10) ** (S - 1))  # last delta is 1e10 -> alpha = 1
    assert torch.allclose(out["weights"][0], torch.tensor(w), atol=1e-6)
    assert torch.allclose(out["acc_map"], torch.ones(B), atol=1e-5)


def test_composite_zero_sigma_is_white():
    B, S = 3, 8
    out = ref.raw2outputs(torch.rand(B, S, 3), torch.zeros(B, S, 1), torch.linspace(2, 6, S).expand(B, S),
                          torch.randn(B, 3))
    assert torch.equal(out["rgb_map"], torch.ones(B, 3))
    assert torch.equal(out["acc_map"], torch.zeros(B))


def test_sample_pdf_uniform_det_is_lerp():
    bins = torch.linspace(2, 6, 9).expand(2, 9)
    s = ref.sample_pdf(bins, torch.ones(2, 8), 5, det=True)
    assert torch.allclose(s, torch.linspace(2, 6, 5).expand(2, 5), atol=1e-5)


def test_sample_pdf_spike_concentrates():
    bins = torch.linspace(0, 8, 9)[None]
    w = torch.zeros(1, 8)
    w[0, 3] = 100.0
    s = ref.sample_pdf(bins, w, 64, det=False, u=torch.rand(1, 64))
    inside = ((s >= 3.0) & (s <= 4.0)).float().mean()
    assert inside > 0.99


def test_shapes_like_reference_test_baseline():
    """noisy_src/test_baseline.py:12-146 shape and range checks, on the oracle."""
    torch.manual_seed(0)
    pe = ref.PositionalEncoding(10)
    assert pe(torch.randn(100, 3)).shape == (100, 63)
    m = ref.NeRF()
    rgb, sigma = m(torch.randn(1024, 3), torch.randn(1024, 3))
    assert rgb.shape == (1024, 3) and sigma.shape == (1024, 1)
    assert rgb.min() >= 0 and rgb.max() <= 1 and sigma.min() >= 0
    dirs = ref.get_ray_directions(100, 100, 50.0)
    assert dirs.shape == (100, 100, 3)
    c2w = torch.eye(4)
    c2w[2, 3] = 4.0
    o, d = ref.get_rays(dirs, c2w)
    o, d = o.reshape(-1, 3)[:100], d.reshape(-1, 3)[:100]
    pts, z = ref.sample_along_rays(o, d, 2.0, 6.0, 64)
    assert pts.shape == (100, 64, 3)
    pf, zf = ref.sample_hierarchical(o, d, z, torch.rand(100, 64), 128)
    assert pf.shape == (100, 192, 3)
    assert torch.all(zf[:, 1:] >= zf[:, :-1])
    out = ref.raw2outputs(torch.rand(100, 64, 3), torch.rand(100, 64, 1) * 10,
                          torch.linspace(2, 6, 64).expand(100, 64), d)
    assert out["rgb_map"].shape == (100, 3) and out["weights"].shape == (100, 64)
    rc = SimpleNamespace(**{**RC.__dict__, "num_samples": 32, "num_samples_fine": 64})
    mc, mf = ref.create_nerf()
    res = ref.render_rays(mc, mf, o[:50], d[:50], rc)
    assert res["rgb_fine"].shape == (50, 3)
