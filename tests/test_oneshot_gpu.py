"""One-shot peer-memory all-reduce (kubeml_amd.parallel.oneshot, csrc/kernels/comm.hip).

Two processes share the single GPU of the test box: each maps the other's IPC region, so
the flag protocol, the double-buffered slots and the rank-ordered sum run exactly as they
would across xGMI (only the link differs).  Checked: exact sums against the same-order fp32
sum for sizes around the float4/tail boundaries, averaging, many back-to-back calls (slot
reuse), graph capture with replays on fresh inputs, the TorchComm routing, and that no spin
ever gave up."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _rank_data(rank, n, salt):
    g = torch.Generator().manual_seed(1000 * salt + 7 * n + rank)
    return torch.randn(n, generator=g)


def _run(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from kubeml_amd.parallel.comm import TorchComm
        from kubeml_amd.parallel.oneshot import OneShotAllReduce
        os_ar = OneShotAllReduce(None, cap_bytes=1 << 20, device=torch.device("cuda", 0))
        bad = []

        def expect(n, salt, scale=1.0):
            acc = _rank_data(0, n, salt)
            for r in range(1, world):
                acc = acc + _rank_data(r, n, salt)
            return acc * scale

        # sizes: scalar, tails, a few float4 blocks, 1 MB - full capacity
        for salt, n in enumerate([1, 3, 4, 5, 1000, 1027, 65536, 262144]):
            t = _rank_data(rank, n, salt).cuda()
            os_ar.all_reduce_(t)
            if not torch.equal(t.cpu(), expect(n, salt)):
                bad.append(("sum", n, float((t.cpu() - expect(n, salt)).abs().max())))
        # average, and 50 back-to-back calls (double-buffered slot reuse)
        for it in range(50):
            n = 333 + it
            t = _rank_data(rank, n, 100 + it).cuda()
            os_ar.all_reduce_(t, scale=1.0 / world)
            if not torch.allclose(t.cpu(), expect(n, 100 + it, 1.0 / world), rtol=0, atol=1e-6):
                bad.append(("avg", it))
        torch.cuda.synchronize()
        # graph capture: three calls per replay, inputs refreshed between replays
        bufs = [torch.zeros(4096 + k, device="cuda") for k in range(3)]
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for b in bufs:
                os_ar.all_reduce_(b)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        dist.barrier()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for b in bufs:
                os_ar.all_reduce_(b)
        for rep in range(5):
            for k, b in enumerate(bufs):
                b.copy_(_rank_data(rank, b.numel(), 500 + 10 * rep + k))
            g.replay()
            torch.cuda.synchronize()
            for k, b in enumerate(bufs):
                if not torch.equal(b.cpu(), expect(b.numel(), 500 + 10 * rep + k)):
                    bad.append(("graph", rep, k))
        # TorchComm routing (avg) through the same mechanism
        comm = TorchComm()
        comm.oneshot = os_ar
        t = _rank_data(rank, 777, 900).cuda()
        comm.all_reduce_(t, op="avg")
        if not torch.allclose(t.cpu(), expect(777, 900, 1.0 / world), rtol=0, atol=1e-6):
            bad.append(("comm", 777))
        errs = os_ar.errors()
        os_ar.close()
        q.put((rank, bad, errs, None))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, None, None, repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_oneshot_allreduce_two_processes_one_gpu():
    import torch.multiprocessing as mp
    from kubeml_amd.runtime.pool import free_port
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_run, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=150) for _ in ps]
    for p in ps:
        p.join(30)
    for rank, bad, errs, exc in res:
        assert exc is None, (rank, exc)
        assert errs == 0, (rank, errs)
        assert not bad, (rank, bad[:5])
