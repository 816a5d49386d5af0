"""Diagnostic: HIP fp32 MLP gradients vs torch-fp32 and torch-fp64 oracles."""
import sys, torch
sys.path[:0] = [".", "robust-nerf_amd"]
from oracle import refimpl as ref
from noisy_src.config import ModelConfig
from noisy_src.model import NeRF
cfg = ModelConfig(precision="fp32")
torch.manual_seed(0); o32 = ref.NeRF(cfg)
o64 = ref.NeRF(cfg).double(); o64.load_state_dict({k: v.double() for k, v in o32.state_dict().items()})
net = NeRF(cfg); net.load_state_dict(o32.state_dict()); net = net.cuda()
g = torch.Generator().manual_seed(1)
M = 777
x = torch.rand(M, 3, generator=g) * 3 - 1.5
d = torch.nn.functional.normalize(torch.randn(M, 3, generator=g), dim=-1)
gr = torch.randn(M, 3, generator=g); gs = torch.randn(M, 1, generator=g)
def run(model, x, d, gr, gs):
    x = x.clone().requires_grad_(True); d = d.clone().requires_grad_(True)
    r, s = model(x, d); ((r * gr).sum() + (s * gs).sum()).backward()
    return [p.grad.detach().double().cpu() for p in model.parameters()], x.grad.double().cpu(), d.grad.double().cpu()
p32, x32, d32 = run(o32, x, d, gr, gs)
p64, x64, d64 = run(o64, x.double(), d.double(), gr.double(), gs.double())
ph, xh, dh = run(net, x.cuda(), d.cuda(), gr.cuda(), gs.cuda())
names = [n for n, _ in o32.named_parameters()]
for n, a, b, c in zip(names, ph, p32, p64):
    print(f"{n:28s} hip-vs64 {((a-c).norm()/c.norm()).item():.2e}  torch32-vs64 {((b-c).norm()/c.norm()).item():.2e}  maxrel hip {((a-c).abs().max()/c.abs().max()).item():.2e} t32 {((b-c).abs().max()/c.abs().max()).item():.2e}")
print("g_x", ((xh-x64).norm()/x64.norm()).item(), ((x32-x64).norm()/x64.norm()).item())
print("g_d", ((dh-d64).norm()/d64.norm()).item(), ((d32-d64).norm()/d64.norm()).item())
