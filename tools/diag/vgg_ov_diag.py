import sys, torch
sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
from test_engine_gpu import _vgg_adam_run
for steps in (1, 2):
    ua, spa, oa, la, sa = _vgg_adam_run(True, steps)
    ub, spb, ob, lb, sb = _vgg_adam_run(False, steps)
    net_ranges = None
    print("steps", steps, "losses", la, lb)
    from kubeml_amd.models.vgg import vgg11_bn
    for name, (s, e) in (("all", (0, spa.numel)),):
        d = (ua[s:e] - ub[s:e]).norm() / ub[s:e].norm()
        print(name, float(d))
    # per-parameter
    worst = []
    for i, (o, n) in enumerate(spa.offsets):
        a, b = ua[o:o + n], ub[o:o + n]
        r = float((a - b).norm() / (b.norm() + 1e-30))
        worst.append((r, i, o, n, float(a.abs().max()), float(b.abs().max())))
    worst.sort(reverse=True)
    for w in worst[:6]:
        print("  param", w)
