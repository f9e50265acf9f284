"""Do forked capture streams run concurrently inside one hipGraph replay?

Captures A) two ``torch.cuda._sleep`` spins serially on one stream and B) the same two
spins forked onto two streams (event fork/join), then times graph replays.  If B takes
about half of A, independent branches (e.g. conv wgrad vs the dgrad chain) overlap.
"""
import torch


def timed(g, n=50):
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    g.replay(); torch.cuda.synchronize()
    s.record()
    for _ in range(n):
        g.replay()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def main():
    cyc = 200000
    main_s = torch.cuda.Stream()
    side = torch.cuda.Stream()
    x = torch.zeros(1 << 20, device="cuda")
    ga, gb, gc = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.stream(main_s):
        with torch.cuda.graph(ga, stream=main_s):
            torch.cuda._sleep(cyc); torch.cuda._sleep(cyc)
        with torch.cuda.graph(gb, stream=main_s):
            ev = torch.cuda.Event(); ev.record(main_s)
            side.wait_event(ev)
            with torch.cuda.stream(side):
                torch.cuda._sleep(cyc)
            torch.cuda._sleep(cyc)
            ev2 = torch.cuda.Event(); ev2.record(side)
            main_s.wait_event(ev2)
        # many small memory-bound kernels on two branches
        with torch.cuda.graph(gc, stream=main_s):
            ev = torch.cuda.Event(); ev.record(main_s)
            side.wait_event(ev)
            with torch.cuda.stream(side):
                for _ in range(20):
                    x.mul_(1.0001)
            y = x.clone()
            for _ in range(20):
                y.add_(1.0)
            ev2 = torch.cuda.Event(); ev2.record(side)
            main_s.wait_event(ev2)
    g1 = torch.cuda.CUDAGraph()
    with torch.cuda.stream(main_s):
        with torch.cuda.graph(g1, stream=main_s):
            torch.cuda._sleep(cyc)
    print(f"one sleep        {timed(g1):8.1f} us")
    print(f"serial 2 sleeps  {timed(ga):8.1f} us")
    print(f"forked 2 sleeps  {timed(gb):8.1f} us")
    print(f"forked 20+20 small kernels {timed(gc):8.1f} us")


if __name__ == "__main__":
    main()
