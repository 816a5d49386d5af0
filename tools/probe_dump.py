import sys, numpy as np, torch
sys.path.insert(0, "robust-nerf_amd")
from noisy_src import _hip
_hip.load(require_all=False)
out = {}
for kind, K in ((2, 16), (3, 2)):
    g = torch.Generator().manual_seed(7)
    A = torch.randint(-4, 5, (32, K), generator=g).float()
    B = torch.randint(-4, 5, (K, 32), generator=g).float()
    D = torch.zeros(64 * 16, device="cuda")
    Ad, Bd = A.cuda(), B.cuda()
    _hip.call("nr_probe_mfma", kind, _hip.ptr(Ad), _hip.ptr(Bd), _hip.ptr(D), _hip.stream_ptr())
    torch.cuda.synchronize()
    out[f"A{kind}"] = A.numpy(); out[f"B{kind}"] = B.numpy(); out[f"D{kind}"] = D.cpu().numpy().reshape(64, 16)
np.savez("gpurun_out/probe_dump.npz", **out)
print("saved")
