"""The classifier-dgrad hand-off of the last block's BN partial rows (nn/modules.py _LinearFn,
models/resnet.py forward) against the block's own BN reduction: same model, same batch, one
backward with the hand-off and one with it disabled (fc._kml_bnf_block cleared after the
forward); prints the relative gradient difference per parameter group."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def run(arch, classes, B, handoff):
    from kubeml_amd.models import resnet as R
    from kubeml_amd.nn import backward_loss, cross_entropy, flatten_module
    torch.manual_seed(0)
    m = getattr(R, arch)(classes).cuda()
    m.train()
    sp = flatten_module(m)
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.randn(B, 32, 32, 8, device="cuda", generator=g).to(torch.bfloat16)
    x[..., 3:] = 0
    y = torch.randint(0, classes, (B,), device="cuda", generator=g)
    sp.zero_grad()
    out = m(x)
    if not handoff:
        object.__setattr__(m.fc, "_kml_bnf_block", None)
    backward_loss(cross_entropy(out, y))
    sp.finish_grads()
    torch.cuda.synchronize()
    named = {n: sp.grad_view([p]).clone() for n, p in m.named_parameters()}
    return named


def main():
    for arch, classes, B in (("resnet18", 10, 32), ("resnet34", 1000, 256)):
        a = run(arch, classes, B, True)
        b = run(arch, classes, B, False)
        worst = sorted(((float((a[n] - b[n]).norm() / (b[n].norm() + 1e-30)), n) for n in a), reverse=True)[:6]
        print(arch, classes, B, "worst rel diffs:", [(n, f"{r:.2e}") for r, n in worst], flush=True)


if __name__ == "__main__":
    main()
