"""conv_bwd (the grouped dgrad+wgrad launch training uses) against an fp64 reference at
the ResNet-18 / 32x32 shapes for several batch sizes, repeated to expose run-to-run
differences (split-K tickets, atomics) — per conv: max rel error of dw and dx, and the
spread of dw over repeats."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

dev = torch.device("cuda", 0)


def main():
    from kubeml_amd.ops import kernels as K
    torch.manual_seed(0)
    convs = [((32, 32, 8), 64, 7, 2, 3), ((8, 8, 64), 64, 3, 1, 1), ((8, 8, 64), 128, 3, 2, 1), ((4, 4, 128), 128, 3, 1, 1),
             ((8, 8, 64), 128, 1, 2, 0), ((4, 4, 128), 256, 3, 2, 1), ((2, 2, 256), 256, 3, 1, 1),
             ((4, 4, 128), 256, 1, 2, 0), ((2, 2, 256), 512, 3, 2, 1), ((1, 1, 512), 512, 3, 1, 1),
             ((2, 2, 256), 512, 1, 2, 0)]
    bad = 0
    for B in (20, 32, 256):
        for (H, W, C), Kc, k, s, p in convs:
            x = torch.randn(B, H, W, C, device=dev).to(torch.bfloat16)
            w = (torch.randn(Kc, k, k, C, device=dev) * 0.05).to(torch.bfloat16)
            OH = (H + 2 * p - k) // s + 1
            OW = (W + 2 * p - k) // s + 1
            dy = torch.randn(B, OH, OW, Kc, device=dev).to(torch.bfloat16)
            xd = x.double().permute(0, 3, 1, 2).contiguous().requires_grad_(True)
            wd = w.double().permute(0, 3, 1, 2).contiguous().requires_grad_(True)
            yd = F.conv2d(xd, wd, stride=s, padding=p)
            yd.backward(dy.double().permute(0, 3, 1, 2))
            ref_dw = wd.grad.permute(0, 2, 3, 1)
            ref_dx = xd.grad.permute(0, 2, 3, 1)
            dws = []
            for _ in range(4):
                dw = torch.zeros(Kc, k, k, C, device=dev)
                dx = K.conv_bwd(dy, w, x, dw, k, k, (s, s), (p, p))
                torch.cuda.synchronize()
                dws.append(dw.clone())
            e_dw = float((dws[0].double() - ref_dw).norm() / ref_dw.norm())
            e_dx = float((dx.double() - ref_dx).norm() / ref_dx.norm())
            spread = max(float((d - dws[0]).abs().max()) for d in dws)
            plans = K.bwd_plans((B, H, W, C), Kc, k, k, (s, s), (p, p))
            flag = "BAD" if (e_dw > 1e-3 or e_dx > 1e-2) else ""
            bad += bool(flag)
            print(f"B={B} in={H}x{W}x{C} K={Kc} k={k} s={s}: dw_err {e_dw:.2e} dx_err {e_dx:.2e} "
                  f"dw_spread {spread:.2e} plans {plans} {flag}", flush=True)
    print("bad", bad)


if __name__ == "__main__":
    main()
