"""Measure the per-kernel floor inside a replayed hipGraph (tiny kernels back to back).

Prints us/kernel for: tiny 1-block kernels, a 2 MB streaming kernel, and the same
under eager launch.  Used to decide between fusing kernels vs speeding them up.
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from kubeml_amd.ops import kernels as K


def timed(fn, n_inner, graph=True, reps=20):
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        fn()
    torch.cuda.synchronize()
    if graph:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(st):
            with torch.cuda.graph(g, stream=st):
                fn()
        torch.cuda.synchronize()
        run = g.replay
    else:
        run = fn
    run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps / n_inner * 1e6


def main():
    dev = torch.device("cuda")
    ctr = torch.zeros(3, device=dev)
    big = torch.zeros(512 * 1024, device=dev)  # 2 MB
    bf = torch.zeros(16384, 64, dtype=torch.bfloat16, device=dev)
    N = 200
    for graph in (True, False):
        tag = "graph" if graph else "eager"
        print(tag, "tiny advance  us/kernel %.2f" % timed(lambda: [K.advance_counter_(ctr, 256, 50000) for _ in range(N)], N, graph))
        print(tag, "zero 2MB      us/kernel %.2f" % timed(lambda: [K.memset_(big) for _ in range(N)], N, graph))
        print(tag, "scale 2MB     us/kernel %.2f" % timed(lambda: [K.scale_(big, 0.5) for _ in range(N)], N, graph))
        print(tag, "relu 2MB bf16 us/kernel %.2f" % timed(lambda: [K.relu_fwd(bf) for _ in range(N)], N, graph))


if __name__ == "__main__":
    main()
