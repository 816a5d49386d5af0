"""Diagnostic: per-sample g_x error vs fp64 across M."""
import sys, torch
sys.path[:0] = [".", "robust-nerf_amd"]
from oracle import refimpl as ref
from noisy_src.config import ModelConfig
from noisy_src.model import NeRF
cfg = ModelConfig(precision="fp32")
torch.manual_seed(0); o = ref.NeRF(cfg); sd = o.state_dict(); o64 = o.double()
net = NeRF(cfg); net.load_state_dict(sd); net = net.cuda()
for M in (64, 128, 160, 256, 777):
    g = torch.Generator().manual_seed(1)
    x = torch.rand(M, 3, generator=g) * 3 - 1.5
    d = torch.nn.functional.normalize(torch.randn(M, 3, generator=g), dim=-1)
    gr = torch.randn(M, 3, generator=g); gs = torch.randn(M, 1, generator=g)
    xh = x.cuda().requires_grad_(True); r, s = net(xh, d.cuda()); ((r * gr.cuda()).sum() + (s * gs.cuda()).sum()).backward()
    x6 = x.double().requires_grad_(True); r6, s6 = o64(x6, d.double()); ((r6 * gr.double()).sum() + (s6 * gs.double()).sum()).backward()
    e = ((xh.grad.double().cpu() - x6.grad).norm(dim=-1) / x6.grad.norm(dim=-1).clamp_min(1e-12))
    bad = (e > 1e-4).nonzero().flatten().tolist()
    print(f"M={M} max rel {e.max().item():.2e} n_bad {len(bad)} tiles {sorted(set(b//32 for b in bad))[:20]} lanes {sorted(set(b%32 for b in bad))[:32]}")
    print("   fwd max", (r.detach().double().cpu() - r6.detach()).abs().max().item(), (s.detach().double().cpu() - s6.detach()).abs().max().item())
