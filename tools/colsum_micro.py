import torch, sys
sys.path.insert(0, '.')
from kubeml_amd.ops import kernels as K
dev = torch.device('cuda', 0)
for C in (768, 2304, 3072):
    x = torch.randn(16384, C, device=dev).bfloat16(); out = torch.zeros(C, device=dev)
    for _ in range(3): K.colsum_(x, out)
    torch.cuda.synchronize(); a, b = torch.cuda.Event(True), torch.cuda.Event(True); a.record()
    for _ in range(50): K.colsum_(x, out)
    b.record(); torch.cuda.synchronize(); t = a.elapsed_time(b) / 50 * 1e3
    print(f"colsum M=16384 C={C}: {t:.1f} us  {x.numel()*2/t/1e6:.2f} TB/s", flush=True)
