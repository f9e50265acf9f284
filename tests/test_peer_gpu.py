"""Peer-memory all-reduce (kubeml_amd.parallel.peer, csrc/kernels/comm.hip).

Two processes share the single GPU of the test box: each maps the other's IPC region, so
the barrier protocol, the double-buffered slots, the reduce-scatter / all-gather split and
the rank-ordered sums run exactly as they would across xGMI (only the link differs).

Checked, for one-shot and two-shot, fp32 and bf16 wire:
  * sums exact against the same-order fp32 sum (bf16 wire: against a torch emulation of the
    rounding), sizes from 1 element to 256 MB, aligned and unaligned views;
  * block caps (the CU-capped overlap configuration) and many back-to-back calls;
  * graph capture with replays on fresh inputs;
  * both ranks bit-identical;
  * a peer that stops calling: the waiting rank's call returns NaN (never a silent wrong sum),
    ``check()`` raises PeerCommError, and the group stays poisoned.
"""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _rank_data(rank, n, salt, dev):
    g = torch.Generator(device=dev).manual_seed(1000 * salt + 7 * n + rank)
    return torch.randn(n, generator=g, device=dev)


def _bf(x):
    return x.to(torch.bfloat16).float()


def _expect(world, n, salt, dev, wire, scale=1.0, algo="twoshot"):
    """Same-order fp32 sum; bf16 wire: inputs rounded, and the two-shot result rounded again
    (the reduced chunk travels as bf16), the one-shot result kept in fp32."""
    if wire == torch.bfloat16:
        acc = _bf(_rank_data(0, n, salt, dev))
        for r in range(1, world):
            acc = acc + _bf(_rank_data(r, n, salt, dev))
        return (_bf(acc) if algo == "twoshot" else acc) * scale
    acc = _rank_data(0, n, salt, dev)
    for r in range(1, world):
        acc = acc + _rank_data(r, n, salt, dev)
    return acc * scale


def _run(rank, world, port, q, late):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from kubeml_amd.parallel.comm import TorchComm
        from kubeml_amd.parallel.peer import PeerAllReduce, PeerCommError
        bad = []
        if late:
            ar = PeerAllReduce(None, cap_bytes=1 << 20, device=dev, timeout_s=1.0)
            t = torch.ones(1000, device=dev)
            ok = torch.ones(1000, device=dev)
            ar.all_reduce_(ok, algo="twoshot")          # a healthy call first
            torch.cuda.synchronize()
            if not torch.equal(ok, torch.full_like(ok, 2.0)):
                bad.append("healthy call")
            dist.barrier()
            if rank == 1:
                import time
                time.sleep(3.0)                          # rank 0's wait expires meanwhile
            for algo in ("twoshot", "oneshot"):
                t.fill_(1.0)
                ar.all_reduce_(t, algo=algo)
                torch.cuda.synchronize()
                if rank == 0 and not bool(torch.isnan(t).all()):
                    bad.append(f"rank 0 {algo}: expected NaN after the timeout, got {t[:4].tolist()}")
                if rank == 1 and not (bool(torch.isnan(t).any()) or torch.equal(t, torch.full_like(t, 2.0))):
                    bad.append(f"rank 1 {algo}: neither NaN nor the true sum: {t[:4].tolist()}")
            errs = ar.errors()
            raised = False
            try:
                ar.check()
            except PeerCommError:
                raised = True
            if rank == 0 and not (errs > 0 and raised):
                bad.append(f"rank 0: errors={errs} raised={raised}")
            dist.barrier()
            ar.close()
            q.put((rank, bad, 0, None))
            return

        cap = 2 * (64 << 20) * 4 // 2 + (1 << 20)      # 256 MB of fp32 per call, one slot
        ar = PeerAllReduce(None, cap_bytes=cap, device=dev)
        # sizes: scalar, tails, vectors, 1 MB .. 256 MB; both algorithms, both wires
        cases = [(n, algo, wire) for n in (1, 3, 5, 8, 1000, 1027, 65536, 262144 + 3)
                 for algo in ("oneshot", "twoshot") for wire in (torch.float32, torch.bfloat16)]
        cases += [(n, "twoshot", wire) for n in (4 << 20, (16 << 20) + 5, 64 << 20)
                  for wire in (torch.float32, torch.bfloat16)]
        for salt, (n, algo, wire) in enumerate(cases):
            t = _rank_data(rank, n, salt, dev)
            ar.all_reduce_(t, algo=algo, wire=wire)
            exp = _expect(world, n, salt, dev, wire, algo=algo)
            if not torch.equal(t, exp):
                bad.append(("sum", n, algo, str(wire), float((t - exp).abs().max())))
            # bit-identical on both ranks
            cs = torch.tensor([float(t.double().sum()), float(t.double().abs().sum())], dtype=torch.float64)
            lst = [None] * world
            dist.all_gather_object(lst, cs.tolist())
            if any(x != lst[0] for x in lst):
                bad.append(("ranks differ", n, algo, str(wire)))
            del t, exp
        # unaligned views, block caps, averaging, 60 back-to-back calls (slot reuse)
        big = _rank_data(rank, 1 << 20, 777, dev)
        for it in range(60):
            off = it % 5
            n = 40000 + 97 * it
            blocks = (1, 8, 32, 256)[it % 4]
            algo = ("oneshot", "twoshot")[it % 2]
            wire = (torch.float32, torch.bfloat16)[(it // 2) % 2]
            v = big[off:off + n]
            src = v.clone()
            ar.all_reduce_(v, scale=1.0 / world, algo=algo, wire=wire, max_blocks=blocks)
            # expected: every rank's slice of its own 'big' (same seeds per rank)
            exp = None
            for r in range(world):
                x = _rank_data(r, 1 << 20, 777, dev)[off:off + n] if r != rank else src
                x = _bf(x) if wire == torch.bfloat16 else x
                exp = x if exp is None else exp + x
            exp = (_bf(exp) if wire == torch.bfloat16 and algo == "twoshot" else exp) * (1.0 / world)
            if not torch.equal(v, exp):
                bad.append(("loop", it, algo, str(wire), blocks, float((v - exp).abs().max())))
            big = _rank_data(rank, 1 << 20, 777, dev)
        torch.cuda.synchronize()
        # graph capture: three calls per replay (mixed algorithms), inputs refreshed between replays
        specs = [(4096, "oneshot", torch.float32), (300001, "twoshot", torch.float32),
                 (200003, "twoshot", torch.bfloat16)]
        bufs = [torch.zeros(n, device=dev) for n, _, _ in specs]
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for b, (_, algo, wire) in zip(bufs, specs):
                ar.all_reduce_(b, algo=algo, wire=wire, max_blocks=64)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        dist.barrier()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for b, (_, algo, wire) in zip(bufs, specs):
                ar.all_reduce_(b, algo=algo, wire=wire, max_blocks=64)
        for rep in range(5):
            for k, (b, (n, _, wire)) in enumerate(zip(bufs, specs)):
                b.copy_(_rank_data(rank, n, 500 + 10 * rep + k, dev))
            g.replay()
            torch.cuda.synchronize()
            for k, (b, (n, _, wire)) in enumerate(zip(bufs, specs)):
                if not torch.equal(b, _expect(world, n, 500 + 10 * rep + k, dev, wire, algo=specs[k][1])):
                    bad.append(("graph", rep, k))
        # TorchComm routing (avg) through the same mechanism
        comm = TorchComm()
        comm.peer = ar
        t = _rank_data(rank, 777, 900, dev)
        comm.all_reduce_(t, op="avg")
        if not torch.allclose(t, _expect(world, 777, 900, dev, torch.float32, 1.0 / world), rtol=0, atol=1e-6):
            bad.append(("comm", 777))
        comm.check()
        if not ar.self_test(kavg=True):       # gradient transport + the fused K-AVG round
            bad.append(("self_test",))
        errs = ar.errors()
        ar.close()
        # the verified factory (what make_train_step uses) agrees on both ranks
        from kubeml_amd.parallel.peer import verified_peer
        vp = verified_peer(None, cap_bytes=64 << 20, device=dev)
        if vp is None:
            bad.append(("verified_peer", None))
        else:
            vp.close()
        q.put((rank, bad, errs, None))
    except Exception as e:  # report instead of hanging the parent
        import traceback
        q.put((rank, None, None, repr(e) + traceback.format_exc()[-1500:]))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _spawn(late):
    import torch.multiprocessing as mp
    from kubeml_amd.runtime.pool import free_port
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_run, args=(r, 2, port, q, late)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=150) for _ in ps]
    for p in ps:
        p.join(30)
    return res


def test_peer_allreduce_two_processes_one_gpu():
    for rank, bad, errs, exc in _spawn(False):
        assert exc is None, (rank, exc)
        assert errs == 0, (rank, errs)
        assert not bad, (rank, bad[:5])


def test_peer_allreduce_late_peer_fails_loudly():
    for rank, bad, errs, exc in _spawn(True):
        assert exc is None, (rank, exc)
        assert not bad, (rank, bad[:5])


def _run_kavg(rank, world, port, q, peer_data):
    """Fused K-AVG rounds (comm.hip kml_peer_kavg through ModelAverager) on a ResNet-18 flat
    state against the unfused reference computed from every rank's pre-round state: the SUM in
    rank order, times fp32 1/count below the count slot, the raw sum at and above it, bf16
    shadow of the parameters, int64 counters floored.  Round 2 leaves the last rank out."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from kubeml_amd.models.resnet import resnet18
        from kubeml_amd.nn import flatten_module
        from kubeml_amd.parallel.comm import TorchComm
        from kubeml_amd.parallel.kavg import ModelAverager
        torch.manual_seed(10 + rank)                      # different models per rank
        net = resnet18(10).to(dev)
        sp = flatten_module(net)
        arena = sp.i64_arena_now()
        comm = TorchComm(peer_data=peer_data)
        av = ModelAverager(net)
        bad = []
        for rnd in range(3):
            arena.copy_(torch.arange(sp.n_i64, device=dev) + 5 * rank + rnd)
            with torch.no_grad():
                sp.state[:sp.i64_off].add_(0.01 * (rank + rnd))
            part = not (rnd == 1 and rank == world - 1)
            # every rank's contribution as kavg_pack builds it, gathered on the host
            mine = sp.state.clone()
            if not part:
                mine.zero_()
            mine[sp.i64_off:sp.i64_off + sp.n_i64] = arena.float() if part else 0.0
            mine[sp.count_idx] = 1.0 if part else 0.0
            allc = [None] * world
            dist.all_gather_object(allc, mine.cpu())
            av.average_(comm, participate=part)
            torch.cuda.synchronize()
            tot = allc[0].clone()
            for r in range(1, world):
                tot = tot + allc[r]
            cnt = float(tot[sp.count_idx])
            inv = torch.tensor(1.0) / max(cnt, 1.0)
            want = tot.clone()
            want[:sp.count_idx] = tot[:sp.count_idx] * inv
            got = sp.state.cpu()
            if not torch.equal(got, want):
                bad.append(("state", rnd, float((got - want).abs().max())))
            if not torch.equal(sp.shadow.cpu(), want[:sp.numel].to(torch.bfloat16)):
                bad.append(("shadow", rnd))
            wi = torch.floor(want[sp.i64_off:sp.i64_off + sp.n_i64] + 1e-3).long()
            if not torch.equal(arena.cpu(), wi):
                bad.append(("counters", rnd))
        q.put((rank, bad, av.fused_rounds, None))
        comm.check()
    except Exception as e:  # report instead of hanging the parent
        import traceback
        q.put((rank, None, None, repr(e) + traceback.format_exc()[-1500:]))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("peer_data", [True, False])
def test_fused_kavg_round_three_ranks_one_gpu(peer_data):
    """peer_data=True: the packed workers' data-plane transport; False: the transport an RCCL
    group builds for K-AVG on first use (verified_peer, self-test with a fused round)."""
    import torch.multiprocessing as mp
    from kubeml_amd.runtime.pool import free_port
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    world = 3
    ps = [ctx.Process(target=_run_kavg, args=(r, world, port, q, peer_data)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=150) for _ in ps]
    for p in ps:
        p.join(30)
    for rank, bad, fused, exc in res:
        assert exc is None, (rank, exc)
        assert not bad, (rank, bad[:5])
        assert fused == 3, (rank, fused)
