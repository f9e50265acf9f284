"""Which rounding does torch's flat.div_(3) use on this GPU (diagnostic for the fused K-AVG apply)."""
import torch
from kubeml_amd.ops import kernels as K
dev = torch.device("cuda")
torch.manual_seed(19)
n = 4099
x = torch.randn(n, device=dev)
flat = x * 3 + torch.randn_like(x)
snap = x.clone()
x2 = x + torch.randn_like(x) * 0.01
ref = x2.clone().add_(flat.clone().div_(3).sub_(snap))
div_t = flat / torch.full_like(flat, 3.0)
mul_r = flat * torch.full_like(flat, 1.0 / 3.0)
d3 = flat.clone().div_(3)
print("div_(3) == tensor div:", torch.equal(d3, div_t), " == mul recip:", torch.equal(d3, mul_r))
out = x2.clone()
K.kavg_async_apply_(out, flat, snap, None, 3, 0)
torch.cuda.synchronize()
bad = (out != ref).nonzero().flatten()
print("mismatches vs torch ref:", bad.numel(), "first idx", bad[:8].tolist())
for name, q in (("div", div_t), ("mul", mul_r), ("d3", d3)):
    r = x2 + (q - snap)
    print(name, "mismatch:", int((out != r).sum()))
