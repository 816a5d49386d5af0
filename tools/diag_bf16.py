"""Diagnostic: HIP bf16 MLP grads vs fp64, next to a bf16-operand emulation in torch."""
import sys, torch
sys.path[:0] = [".", "robust-nerf_amd"]
from oracle import refimpl as ref
from noisy_src.config import ModelConfig
from noisy_src.model import NeRF
import torch.nn.functional as F
cfg = ModelConfig(precision="bf16")
torch.manual_seed(0); o = ref.NeRF(cfg); sd = o.state_dict()
o64 = ref.NeRF(cfg).double(); o64.load_state_dict({k: v.double() for k, v in sd.items()})
net = NeRF(cfg); net.load_state_dict(sd); net = net.cuda()
# bf16-operand emulation: linear layers round input and weight to bf16, accumulate fp32
class EmuLinear(torch.nn.Module):
    def __init__(self, lin): super().__init__(); self.lin = lin
    def forward(self, x):
        return F.linear(x.bfloat16().float(), self.lin.weight.bfloat16().float(), self.lin.bias)
emu = ref.NeRF(cfg); emu.load_state_dict(sd)
for i in range(len(emu.pts_linears)): emu.pts_linears[i] = EmuLinear(emu.pts_linears[i])
emu.feature_linear = EmuLinear(emu.feature_linear); emu.dir_linear = EmuLinear(emu.dir_linear)
g = torch.Generator().manual_seed(1); M = 1500
x = torch.rand(M, 3, generator=g) * 3 - 1.5
d = torch.nn.functional.normalize(torch.randn(M, 3, generator=g), dim=-1)
gr = torch.randn(M, 3, generator=g); gs = torch.randn(M, 1, generator=g)
def run(model, dev, dt):
    for p in model.parameters(): p.grad = None
    r, s = model(x.to(dev, dt), d.to(dev, dt)); ((r * gr.to(dev, dt)).sum() + (s * gs.to(dev, dt)).sum()).backward()
    return [p.grad.double().cpu() for p in model.parameters()], r.double().detach().cpu(), s.double().detach().cpu()
ph, rh, sh = run(net, "cuda", torch.float32)
p6, r6, s6 = run(o64, "cpu", torch.float64)
pe, re_, se = run(emu, "cpu", torch.float32)
print("fwd rgb max: hip", (rh - r6).abs().max().item(), "emu", (re_ - r6).abs().max().item())
print("fwd sig max: hip", (sh - s6).abs().max().item(), "emu", (se - s6).abs().max().item(), "|sig|max", s6.abs().max().item())
names = [n for n, _ in o64.named_parameters()]
for n, a, b, c in zip(names, ph, pe, p6):
    print(f"{n:26s} hip {((a-c).norm()/c.norm()).item():.3e}  emu {((b-c).norm()/c.norm()).item():.3e}")
