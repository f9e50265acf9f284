"""Overlapped (staleness-1) K-AVG semantics — parallel/kavg.py AsyncModelAverager.

Two gloo ranks (real async collectives) and the in-process thread backend (sync fallback)
run scripted rounds: in round r rank i adds a known delta to every parameter and buffer,
then averages.  Expected, with A_r = mean_i x_i^(r) and the model corrected one round late:

    x_i <- A_(r-1) + (x_i - x_i^(r-1))     (then round r's average starts)

and after flush_() every rank holds the same model: the corrected model, averaged."""
import os

import numpy as np
import torch

ROUNDS = 4


def _delta(rank, r, n):
    g = torch.Generator().manual_seed(100 * r + rank)
    return torch.randn(n, generator=g, dtype=torch.float64).float()


def _expected(world, n0):
    """Reference recurrence for every rank (numpy, float64)."""
    x = [np.zeros(n0) for _ in range(world)]
    pending = None          # (avg, snaps)
    for r in range(ROUNDS):
        for i in range(world):
            x[i] = x[i] + _delta(i, r, n0).double().numpy()
        if pending is not None:
            avg, snaps = pending
            x = [avg + (x[i] - snaps[i]) for i in range(world)]
        pending = (sum(x) / world, [v.copy() for v in x])
    avg, snaps = pending
    x = [avg + (x[i] - snaps[i]) for i in range(world)]
    return sum(x) / world, x


class _Tiny(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.lin = torch.nn.Linear(3, 2)
        self.register_buffer("stat", torch.zeros(4))
        with torch.no_grad():
            self.lin.weight.zero_()
            self.lin.bias.zero_()


def _tensors(m):
    return [m.lin.weight, m.lin.bias, m.stat]


def _run_rank(rank, world, comm):
    from kubeml_amd.parallel.kavg import AsyncModelAverager
    m = _Tiny()
    av = AsyncModelAverager(m)
    n0 = sum(t.numel() for t in _tensors(m))
    for r in range(ROUNDS):
        d = _delta(rank, r, n0)
        off = 0
        with torch.no_grad():
            for t in _tensors(m):
                t.add_(d[off:off + t.numel()].view_as(t))
                off += t.numel()
        av.average_(comm)
    assert av.pending
    av.flush_(comm)
    assert not av.pending
    return torch.cat([t.detach().reshape(-1) for t in _tensors(m)]).double().numpy()


def _gloo_rank(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from kubeml_amd.parallel.comm import TorchComm
        q.put((rank, _run_rank(rank, world, TorchComm()), None))
    except Exception as e:
        q.put((rank, None, repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_async_kavg_gloo_two_ranks():
    import torch.multiprocessing as mp
    from kubeml_amd.runtime.pool import free_port
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_gloo_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=120) for _ in ps], key=lambda t: t[0])
    for p in ps:
        p.join(30)
    for _, _, err in res:
        assert err is None, err
    final, _ = _expected(2, len(res[0][1]))
    for _, x, _ in res:
        np.testing.assert_allclose(x, final, rtol=1e-5, atol=1e-5)


def test_async_kavg_thread_backend_matches_recurrence():
    import threading
    from kubeml_amd.parallel.comm import ThreadComm
    world = 3
    comms = ThreadComm.create(world)
    out = [None] * world

    def body(i):
        out[i] = _run_rank(i, world, comms[i])
    th = [threading.Thread(target=body, args=(i,)) for i in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(60)
    final, _ = _expected(world, len(out[0]))
    for x in out:
        np.testing.assert_allclose(x, final, rtol=1e-5, atol=1e-5)
