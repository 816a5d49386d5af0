"""Diagnostic: isolate the sigma-path vs rgb-path contribution to trunk grads."""
import sys, torch
sys.path[:0] = [".", "robust-nerf_amd"]
from oracle import refimpl as ref
from noisy_src.config import ModelConfig
from noisy_src.model import NeRF
cfg = ModelConfig(precision="fp32")
torch.manual_seed(0); o64 = ref.NeRF(cfg)
sd = o64.state_dict()
o64 = o64.double()
net = NeRF(cfg); net.load_state_dict(sd); net = net.cuda()
g = torch.Generator().manual_seed(1)
M = 64
x = torch.rand(M, 3, generator=g) * 3 - 1.5
d = torch.nn.functional.normalize(torch.randn(M, 3, generator=g), dim=-1)
def run(model, x, d, gr, gs):
    for p in model.parameters(): p.grad = None
    r, s = model(x, d); ((r * gr).sum() + (s * gs).sum()).backward()
    return [p.grad.detach().double().cpu() for p in model.parameters()], r.detach().double().cpu(), s.detach().double().cpu()
names = [n for n, _ in net.named_parameters()]
for label, grs, gss in (("rgb only", 1.0, 0.0), ("sigma only", 0.0, 1.0)):
    gr = torch.randn(M, 3, generator=g) * grs; gs = torch.randn(M, 1, generator=g) * gss
    ph, rh, sh = run(net, x.cuda(), d.cuda(), gr.cuda(), gs.cuda())
    p6, r6, s6 = run(o64, x.double(), d.double(), gr.double(), gs.double())
    print(label, "fwd rgb", (rh - r6).abs().max().item(), "sigma", (sh - s6).abs().max().item())
    for n, a, c in zip(names, ph, p6):
        if "bias" in n:
            print(f"   {n:24s} rel {((a-c).norm()/c.norm().clamp_min(1e-30)).item():.2e}  |c| {c.norm().item():.3e}")
# sigma-only, per-sample check of dz7 via bias grad with single samples
gr = torch.zeros(M, 3); gs = torch.zeros(M, 1)
for m in range(4):
    gs.zero_(); gs[m] = 1.0
    ph, rh, sh = run(net, x.cuda(), d.cuda(), gr.cuda(), gs.cuda())
    p6, r6, s6 = run(o64, x.double(), d.double(), gr.double(), gs.double())
    i7 = names.index("pts_linears.7.bias")
    a, c = ph[i7], p6[i7]
    diff = (a - c).abs()
    print("sample", m, "sigma", s6[m].item(), "max|dz7 diff|", diff.max().item(), "max|dz7|", c.abs().max().item(),
          "argmax", diff.argmax().item(), "ratio at argmax", (a[diff.argmax()] / c[diff.argmax()]).item())
