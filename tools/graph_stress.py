"""Graph-replay stress test for the conv kernels (stale-data / race detector).

Captures [inputs <- sources (copy kernels)] -> memset(dw) -> conv_fwd -> conv_wgrad into
one hipGraph, then replays it with new source data every time and compares every
replay against an eager recomputation.  A kernel that reads stale data across graph
replays, or races inside a launch, shows up as a mismatch on some replay.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from kubeml_amd.ops import kernels as K


def rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


ZERO = os.environ.get("ZERO", "memset")


def main(reps=20):
    dev = torch.device("cuda")
    torch.manual_seed(0)
    cases = [
        # (B,H,W,Ci,Co,k,s,p, fwd cfg, wgrad cfg)
        (256, 32, 32, 8, 64, 7, 2, 3, (128, 32, 64, 1, 1), (64, 32, 64, 32, 0)),
        (256, 8, 8, 64, 64, 3, 1, 1, (128, 32, 64, 1, 1), (32, 32, 64, 32, 0)),
        (256, 8, 8, 64, 128, 3, 2, 1, (64, 32, 64, 1, 1), (32, 32, 64, 8, 0)),
        (256, 1, 1, 512, 512, 3, 1, 1, (32, 32, 64, 1, 0), (32, 32, 64, 2, 0)),
    ]
    bad = 0
    for (B, H, W, Ci, Co, k, s, p, cf, cw) in cases:
        OH, OW = K.out_hw(H, W, k, k, s, s, p, p)
        src_x = torch.randn(B, H, W, Ci, device=dev).to(torch.bfloat16)
        src_w = (torch.randn(Co, k, k, Ci, device=dev) * 0.05).to(torch.bfloat16)
        src_dy = torch.randn(B, OH, OW, Co, device=dev).to(torch.bfloat16)
        x, w, dy = src_x.clone(), src_w.clone(), src_dy.clone()
        dw = torch.zeros(Co, k, k, Ci, device=dev)
        y = torch.empty(B, OH, OW, Co, dtype=torch.bfloat16, device=dev)

        def body():
            x.copy_(src_x)
            w.copy_(src_w)
            dy.copy_(src_dy)
            if ZERO == "memset":
                K.memset_(dw)
            elif ZERO == "fill":
                K.fill_(dw, 0.0)
            else:
                dw.zero_()
            K.conv_fwd(x, w, k, k, (s, s), (p, p), out=y, cfg=cf)
            K.conv_wgrad(x, dy, dw, k, k, (s, s), (p, p), cfg=cw)

        for _ in range(2):
            body()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            with torch.cuda.graph(g, stream=st):
                body()
        torch.cuda.current_stream().wait_stream(st)
        torch.cuda.synchronize()
        for r in range(reps):
            src_x.copy_(torch.randn_like(src_x, dtype=torch.float32).to(torch.bfloat16))
            src_w.copy_((torch.randn_like(src_w, dtype=torch.float32) * 0.05).to(torch.bfloat16))
            src_dy.copy_(torch.randn_like(src_dy, dtype=torch.float32).to(torch.bfloat16))
            g.replay()
            torch.cuda.synchronize()
            y_ref = K.conv_fwd(src_x, src_w, k, k, (s, s), (p, p), cfg=(32, 32, 32, 1, 0))
            dw_ref = torch.zeros_like(dw)
            K.conv_wgrad(src_x, src_dy, dw_ref, k, k, (s, s), (p, p), cfg=(32, 32, 32, 1, 0))
            torch.cuda.synchronize()
            ey, ew = rel(y, y_ref), rel(dw, dw_ref)
            if ey > 1e-2 or ew > 1e-2 or not (ey == ey and ew == ew):
                bad += 1
                print(f"MISMATCH case {(B, H, W, Ci, Co, k, s, p)} replay {r}: fwd {ey:.3e} wgrad {ew:.3e}", flush=True)
        print(f"case {(H, W, Ci, Co, k, s)} fwd {cf} wgrad {cw}: done", flush=True)
    print("TOTAL_BAD", bad)


if __name__ == "__main__":
    main()
