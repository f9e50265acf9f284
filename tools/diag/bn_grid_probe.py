"""Graph-timed BN apply / BN backward apply on ResNet-50's largest maps (run per KUBEML_BN_GRID_CAP)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from kubeml_amd.ops import kernels as K
from tools.conv_micro import gtime

dev = "cuda"
for (M, C) in [(401408, 256), (401408, 64), (100352, 512), (25088, 1024)]:
    x = torch.randn(M, C, device=dev).to(torch.bfloat16)
    r = torch.randn(M, C, device=dev).to(torch.bfloat16)
    stats = torch.zeros(2 * C, device=dev)
    K.bn_stats(x, stats)
    g, b = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)
    y = torch.empty_like(x)
    t1 = gtime(lambda: K.bn_apply(x, stats, g, b, res=r, y=y, relu=True), reps=20)
    t0 = gtime(lambda: K.bn_apply(x, stats, g, b, y=y, relu=True), reps=20)
    mean, rstd = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    dres = torch.empty_like(x)
    tb = gtime(lambda: K.bn_bwd(r, y, x, mean, rstd, g, dg, db, dres=dres), reps=20)
    mb = M * C * 2 / 1e6
    print(f"cap={os.environ.get('KUBEML_BN_GRID_CAP', '1024')} M={M} C={C}: apply+res {t1:.1f}us "
          f"({3 * mb / t1:.2f} TB/s)  apply {t0:.1f}us ({2 * mb / t0:.2f} TB/s)  bwd(+dres) {tb:.1f}us", flush=True)
