"""Synchronous data-parallel train step builder (north-star config 2).

One function, :func:`make_train_step`, assembles the framework's hot loop for a
flattened model: the (optionally stage-split) forward/backward, the backward-overlapped
gradient all-reduce over the job's RCCL group, the fused optimizer with the 1/P average
folded in, and the hipGraph capture that never mutates training state.  It is what
``KubeModel.step`` runs on resident GPU workers (sdk/model.py) and what the headline
``bench.py`` runs — the benchmark measures the framework's own path.

Reference: the per-iteration HTTP fan-out + Redis weight round trip of K=1 training
(ml/pkg/train/job.go:295-334, python/kubeml/kubeml/network.py:252-310).
"""
from __future__ import annotations

import os
from typing import Callable, Optional, Sequence

import logging

import torch

from .step import GraphedTrainStep, train_state_tensors

_log = logging.getLogger("kubeml.dp")

# rider blocks per shard-rider slice (``shardride``): a slice alone runs fastest at 256 (1.05M
# elements: 9.7 us at 256, 11.6 at 512, 16.7 at 1024 blocks; tools/diag/zs_rider_micro.py).
# Ranks packed on one GPU (tests, packed workers) share PACKED_RIDE_BLOCKS: a rider block spins
# until every peer published, and the spinning blocks of P - 1 ranks must never fill the CUs the
# last rank's launch needs to publish (4 ranks x 256 did)
SHARD_RIDE_BLOCKS = 256
PACKED_RIDE_BLOCKS = 128


def make_train_step(model: torch.nn.Module, space, optimizer, loss_fn: Callable, x: torch.Tensor,
                    y: torch.Tensor, *, pre: Optional[Callable[[], None]] = None,
                    post: Optional[Callable[[], None]] = None, group=None, world: int = 1,
                    use_graph: bool = True, graph_comm: bool = True, overlap: bool = True,
                    bucket_mb: float = 0.0, force_comm: bool = False, warmup: int = 1,
                    extra_state: Sequence[torch.Tensor] = (), comm_dtype=None,
                    opt_overlap: Optional[bool] = None, advance=None, plan=None, peer=None,
                    ride: Optional[bool] = None,
                    comm_timing: int = 0, forward: Optional[Callable] = None) -> GraphedTrainStep:
    """Build (not capture) the train step on static input buffers ``x``/``y``.

    pre():  runs first inside the step (e.g. on-device augmentation into ``x``)
    post(): runs after the optimizer
    advance: (ctr, batch, n) -- advance the on-device data counter after the optimizer
            (``ops.kernels.advance_counter_``); folded into the fused SGD launch when the
            optimizer can (``fuse_advance``)
    world:  ranks in ``group``; > 1 adds the gradient all-reduce (SUM) and sets the
            optimizer's gradient scale to 1/world
    overlap: split backward at ``model.stages()`` (if the model has them) so each
            stage's gradients are all-reduced while the next stage's backward runs
    comm_dtype: torch.bfloat16 all-reduces bf16-rounded gradients (half the bytes; see
            :class:`GraphedTrainStep`); None = fp32
    opt_overlap: apply the optimizer per backward stage on a side stream as soon as the
            stage's gradients are final (after its all-reduce when world > 1), overlapping the
            bandwidth-bound update with the rest of the latency-bound backward; needs a model
            with stages, an optimizer with ``step_range`` and the whole step in one graph.
            None = off (on one MI355X the concurrent
            side-stream update slows the backward's latency-bound kernel stream, ResNet-34
            1.40 -> 1.73-1.81 ms/step whatever its grid; profiles/launch_fusion_r2.md)
    plan:   a :class:`kubeml_amd.parallel.plan.CommPlan` (transport, schedule, wire, block cap);
            it overrides ``overlap`` and ``comm_dtype``.  ``backend="peer"`` uses ``peer`` (a
            :class:`kubeml_amd.parallel.peer.PeerAllReduce` over ``group``) or, when None,
            creates one sized for the flat gradient — collective over ``group``.
    comm_timing: T > 0 stamps the collectives on the device every step and samples their time
            every T-th step (``step.comm_seconds()``; exported as kubeml_allreduce_seconds)
    ride:   apply the SGD update of the parameters ``model.ride_plan()`` names (ResNet: layer4 + fc)
            in extra blocks of the grouped conv-backward launches of its host convs (layer3), where
            the memory-bound update streams beside latency-bound conv tiles in the same launch (no
            second queue); the end-of-step launch then covers the rest.  One GPU, no collective,
            fused SGD.  None = ``KUBEML_RIDE`` (default on: ResNet-34 1.330 -> 1.320 ms/step over six
            alternating runs on two boxes, bit-identical weights; profiles/r5/sgd_rider.md).
    forward: ``forward(model, x, y) -> loss`` in place of ``loss_fn(model(x), y)`` (models whose
            call takes more than the batch, e.g. BERT MLM with its positions and labels, or a
            step that prepares its batch on the device first); the step is then not stage-split
    """
    comm = world > 1 or force_comm
    shard = None
    staged_shard = False
    ride_shard = False
    if plan is not None and plan.schedule == "shardride":
        # the sharded update of the stages whose gradients are final early (ResNet: layer4 + fc,
        # then layer3) rides in later backward launches of the same queue (_shard_ride)
        ride_shard = (forward is None and hasattr(model, "comm_ride_plan") and
                      getattr(optimizer, "kind", None) == "sgd" and optimizer.supports_ranges() and
                      bool(model.comm_ride_plan()))
        from ..parallel.plan import CommPlan
        plan = CommPlan("peer", "shard", plan.wire, plan.max_blocks,
                        source=plan.source + ("" if ride_shard else " (shardride -> shard: no ride plan / fused SGD)"))
    if plan is not None and plan.schedule == "shardov":
        # per-stage shard steps need stage-contiguous gradient ranges and the fused SGD
        staged_shard = (forward is None and hasattr(model, "stages") and hasattr(model, "stage_params") and
                        getattr(optimizer, "kind", None) == "sgd" and optimizer.supports_ranges())
        from ..parallel.plan import CommPlan
        plan = CommPlan("peer", "shard", plan.wire, plan.max_blocks,
                        source=plan.source + ("" if staged_shard else " (shardov -> shard: no stages / fused SGD)"))
    if plan is not None and plan.schedule == "shard":
        on_gpu = comm and torch.cuda.is_available() and space.grad.is_cuda
        # the optimizer's capability is checked BEFORE the collective setup (the same answer on
        # every rank), so an optimizer that cannot update one flat range falls back like a node
        # without IPC buffers instead of failing after the self-test
        can_shard = ((getattr(optimizer, "kind", None) == "sgd" and optimizer.supports_ranges())
                     or getattr(optimizer, "supports_shard_range", lambda: False)())
        if on_gpu and not can_shard:
            _log.warning("shard plan: the optimizer cannot update one flat range; using the all-reduce plan")
        if on_gpu and can_shard:
            from ..parallel.peer import PeerShard, verified_shard
            shard = peer if isinstance(peer, PeerShard) and peer.space is space and peer.region is not None else None
            if shard is None:
                shard = verified_shard(space, group, log=_log.warning)     # collective over group
        if shard is None:
            # no IPC buffers / self-test failed (every rank alike) / CPU group: exact all-reduce
            from ..parallel.plan import CommPlan
            plan = CommPlan("peer" if on_gpu else "rccl", "end" if on_gpu else "overlap", "fp32", plan.max_blocks,
                            source=f"{plan.source} (shard unavailable)")
        peer = shard
        if shard is not None:
            overlap = staged_shard            # one collective after the backward, or one per stage
        else:
            staged_shard = False
    if plan is not None and shard is None:
        overlap = plan.schedule == "overlap"
        comm_dtype = plan.wire_dtype
        if plan.backend == "peer" and comm and peer is None and torch.cuda.is_available() and space.grad.is_cuda:
            from ..parallel.peer import slot_bytes, verified_peer
            # collective; None (on every rank) when the node cannot map peers or the self-test
            # fails — the step then runs the same schedule over RCCL
            peer = verified_peer(group, cap_bytes=slot_bytes(space.grad.numel(), world, "twoshot", comm_dtype),
                                 device=space.grad.device, log=_log.warning)
        if plan.backend != "peer":
            peer = None
    if comm_dtype is None:
        comm_dtype = torch.float32
    from ..nn import backward_loss
    scale = 1.0 / max(world, 1)

    fold = None           # (ctr, batch, n) advanced inside the fused SGD launch (per call)

    def opt_step():
        optimizer.set_grad_scale(scale)
        if fold is not None:
            optimizer.step(advance=fold)
        else:
            optimizer.step()
        if post is not None:
            post()

    segs = seg_grads = seg_opt = opt_finish = None
    staged_ok = forward is None and hasattr(model, "stages") and hasattr(model, "stage_params")
    opt_overlap = bool(opt_overlap and staged_ok and use_graph and (graph_comm or not comm) and peer is None
                       and getattr(optimizer, "supports_ranges", lambda: False)())
    if advance is not None:
        fused = (not opt_overlap and getattr(optimizer, "fuse_advance", lambda *a: False)(*advance))
        if fused:
            fold = tuple(advance)
        else:
            user_post = post

            def post():
                if user_post is not None:
                    user_post()
                from ..ops import kernels as K
                K.advance_counter_(*advance)
    if (comm and overlap and staged_ok) or opt_overlap or staged_shard:
        from .staged import StagedForwardBackward

        def pre0():
            if pre is not None:
                pre()
            space.zero_grad()
        staged = StagedForwardBackward(model.stages(), lambda out: loss_fn(out, y), lambda: x, pre=pre0)
        sp = model.stage_params()
        stage_of_seg = [sp[len(sp) - 1 - k] for k in range(len(sp))]

        def _seg(k):
            run = staged.segment(k)

            def seg():
                out = run()
                space.finish_grads(stage_of_seg[k])   # this stage's gradients are final
                return out
            return seg
        segs = [_seg(k) for k in range(staged.n_segments)]
        seg_grads = [[space.grad_view(ps)] for ps in stage_of_seg]
        fwd_bwd = None
        if opt_overlap:
            ranges = [space.range_of(ps) for ps in stage_of_seg]
            tiles = sorted(ranges)
            if tiles[0][0] != 0 or tiles[-1][1] != space.numel or any(
                    a[1] != b[0] for a, b in zip(tiles, tiles[1:])):
                raise ValueError("stage ranges must tile the flat parameter space")
            def _seg_opt(k, s, e):
                def run():
                    if k == 0:
                        optimizer.begin_ranges()    # Adam: the bias-correction step advances once
                    optimizer.step_range(s, e, advance_step=False)
                return run
            seg_opt = [_seg_opt(k, s, e) for k, (s, e) in enumerate(ranges)]

            def opt_finish():
                optimizer.finish_ranges()
                if post is not None:
                    post()
    else:
        def fwd_bwd():
            if pre is not None:
                pre()
            space.zero_grad()
            loss = forward(model, x, y) if forward is not None else loss_fn(model(x), y)
            backward_loss(loss)
            space.finish_grads()
            return loss
    if ride is None:
        ride = os.environ.get("KUBEML_RIDE", "1") == "1"
    riding = bool(ride and fwd_bwd is not None and not comm and shard is None and seg_opt is None
                  and forward is None and hasattr(model, "ride_plan") and getattr(optimizer, "kind", None) == "sgd"
                  and optimizer.supports_ranges() and space.grad.is_cuda and bool(model.ride_plan()))
    if riding:
        fwd_bwd, opt_step = _ride(model, space, optimizer, fwd_bwd, post, lambda: fold, scale)
    shard_step = on_replay = seg_shard = None
    step_ref = {}                 # the GraphedTrainStep (its _comm_on gates the shard riders)
    shard_ride_info = None
    if shard is not None:
        blocks = plan.max_blocks
        fused_sgd = getattr(optimizer, "kind", None) == "sgd" and optimizer.supports_ranges()
        # the parameters the step reads from the fp32 master (BN / LN affine, biases) are re-read
        # from their owners after every step: the ZeRO-1 master is current only on own chunks
        shard.set_fresh([space.range_of([p]) for p in model.parameters() if p.requires_grad and p.dim() == 1])
        if staged_shard:
            # ownership cut per backward stage (every rank the same ranges): stage k's
            # reduce-scatter + SGD + all-gather run on a side stream once its gradients are final
            space.sync_master()
            ranges = [space.range_of(ps) for ps in stage_of_seg]
            order = sorted(range(len(ranges)), key=lambda k: ranges[k][0])
            shard.set_stages([ranges[k] for k in order])
            seg_of = {k: order.index(k) for k in range(len(ranges))}
            nseg = len(ranges)

            def _stage(k, stamps=None):
                s0, s1 = stamps if stamps is not None else (None, None)
                shard.stage_step(seg_of[k], optimizer, advance=fold, max_blocks=blocks, first_stage=k == 0,
                                 last_stage=k == nseg - 1, stamps=None if stamps is None else (s0, s1))
                if k == nseg - 1:
                    shard.gather_fresh()
            seg_shard = [(lambda st=None, k=k: _stage(k, st)) for k in range(nseg)]

        def shard_step(stamps=None):
            """stamps: int64[2] device buffer (timing) — start / end of the collective."""
            s0 = s1 = None
            if stamps is not None:
                s0, s1 = stamps.data_ptr(), stamps.data_ptr() + 8
            space.finish_grads()
            if fused_sgd:           # reduce-scatter + SGD + shadow chunk in one pass
                shard.reduce_scatter(optimizer, advance=fold, max_blocks=blocks, stamp=s0)
            else:
                shard.reduce_scatter(None, max_blocks=blocks, stamp=s0)
                optimizer.set_grad_scale(scale)
                optimizer.step_range(shard.lo, shard.hi, max_blocks=blocks)
                if fold is not None:
                    from ..ops import kernels as K
                    K.advance_counter_(*fold)
            shard.all_gather_shadow(max_blocks=blocks, stamp=s1)
            shard.gather_fresh()
            if post is not None:
                post()

        if seg_shard is not None:
            def shard_step(stamps=None):
                """Staged layout: the per-stage collectives ran beside the backward."""
                if post is not None:
                    post()

        if ride_shard and fused_sgd and fwd_bwd is not None and seg_shard is None:
            got = _shard_ride(model, space, optimizer, shard, fwd_bwd, post, lambda: fold,
                              _ride_blocks(shard, blocks), step_ref)
            if got is not None:
                fwd_bwd, shard_step, shard_ride_info = got

        def on_replay():
            space._master_stale = True

    optimizer.set_grad_scale(scale)
    step = step_ref["step"] = GraphedTrainStep(fwd_bwd, opt_step, [space.grad], group=group, use_graph=use_graph, warmup=warmup,
                            bucket_mb=bucket_mb, segments=segs, segment_grads=seg_grads, force_comm=force_comm,
                            graph_comm=graph_comm, comm_dtype=comm_dtype,
                            state_tensors=train_state_tensors(model, space, optimizer, extra_state),
                            segment_opt=seg_opt, opt_finish=opt_finish, peer=peer,
                            schedule=plan.schedule if plan is not None else "overlap",
                            peer_blocks=plan.max_blocks if plan is not None else 256, comm_timing=comm_timing,
                            shard_step=shard_step, on_replay=on_replay, world=max(int(world), 1),
                            segment_shard=seg_shard)
    step.ride_plan = (os.environ.get("KUBEML_RIDE_PLAN") or "4f:321;123:s") if riding else None
    step.shard_ride = shard_ride_info   # {"slices": n, "taken": set of the last step's carried slices}
    return step


def _ride_blocks(shard, blocks):
    per = max(1, int(getattr(shard, "ranks_per_device", 1)))
    cap = SHARD_RIDE_BLOCKS if per == 1 else max(16, PACKED_RIDE_BLOCKS // per)
    return max(1, min(int(blocks), cap))


def _shard_ride(model, space, optimizer, shard, fwd_bwd, post, get_fold, blocks, step_ref):
    """make_train_step's ``shardride`` plan: ``model.comm_ride_plan()`` = [(parameters, RS hosts,
    AG hosts)] for two early-final stages that must lead the flat layout (ResNet: layer4 + fc, then
    layer3).  The shard is cut per stage (rank r owns chunk r of each); each stage's reduce-scatter
    + fused SGD runs as :class:`~kubeml_amd.parallel.peer.ShardRider` slices in its RS hosts'
    backward launches and its shadow all-gather in its AG hosts' launches (same queue, no side
    stream; cross-rank progress counters, csrc/include/kml_sgd.h), so only the last stage (the rest
    of the space: ResNet's layer2 + layer1 + stem, ~7 % of the bytes) remains after the backward.
    The riders run only while the step's collectives are on (never in the local warm-up)."""
    from ..parallel.peer import PeerShard
    groups = model.comm_ride_plan()
    if len(groups) != PeerShard.RIDER_STAGES:
        raise ValueError(f"comm ride plan: {PeerShard.RIDER_STAGES} groups (parameters, RS hosts, AG hosts)")
    ranges = [space.range_of(ps) for ps, _, _ in groups]
    if ranges[0][0] != 0 or ranges[0][1] != ranges[1][0] or not ranges[1][1] < space.numel:
        raise ValueError("comm ride plan: the riding stages must lead the flat layout, in backward order")
    space.sync_master()                # collective: the master is complete before the ownership switch
    shard.set_stages([ranges[0], ranges[1], (ranges[1][1], space.numel)])
    riders, seen = [], set()           # (group, kind, ShardRider), in phase order
    holder = {}

    def take_for(j):
        return lambda: holder["take"](j)
    for gi, (ps, rs_hosts, ag_hosts) in enumerate(groups):
        for kind, hosts in (("rs", rs_hosts), ("ag", ag_hosts)):
            if not hosts or any(id(h) in seen for h in hosts):
                raise ValueError("comm ride plan: every phase needs host convs of its own")
            seen.update(id(h) for h in hosts)
            for h, r in zip(hosts, shard.rider_slices(gi, kind, len(hosts), optimizer, blocks)):
                riders.append((gi, kind, r))
                object.__setattr__(h, "_kml_rider", take_for(len(riders) - 1))
    if not shard.rider_self_test([r for _, _, r in riders], optimizer):   # collective
        # every rank alike: no riders, the whole space back to one end-of-backward shard step
        _log.warning("shard riders failed their self-test; using the end-of-backward shard step")
        for _, rs_hosts, ag_hosts in groups:
            for h in list(rs_hosts) + list(ag_hosts):
                object.__setattr__(h, "_kml_rider", None)
        shard.set_stages([(0, space.numel)])
        return None
    state = {"active": False, "taken": set(), "fired": set()}

    def _take(j):
        gi, kind, r = riders[j]
        if not state["active"] or j in state["taken"]:
            return None
        if kind == "rs" and gi not in state["fired"]:
            space.finish_grads(groups[gi][0])   # e.g. layer3's deferred unrolled-weight folds, here
            state["fired"].add(gi)
        state["taken"].add(j)
        return r
    holder["take"] = _take

    def ride_fwd_bwd():
        st = step_ref.get("step")
        state["active"] = st is not None and st.comm and st._comm_on
        state["taken"], state["fired"] = set(), set()
        try:
            return fwd_bwd()
        finally:
            state["active"] = False

    def shard_step(stamps=None):
        """The rest of the space after the backward (stage 2), plus any slice whose host did not
        carry it (in phase order; on ResNet every host conv runs a rider-capable launch)."""
        left = [j for j in range(len(riders)) if j not in state["taken"]]
        if left:
            _log.warning("shard riders: %d slice(s) ran on their own launch", len(left))
            for j in left:
                riders[j][2].run_alone()
        space.finish_grads()
        st = None if stamps is None else (stamps.data_ptr(), stamps.data_ptr() + 8)
        shard.stage_step(2, optimizer, advance=get_fold(), max_blocks=blocks, first_stage=True, last_stage=True,
                         stamps=st)
        shard.gather_fresh()
        if post is not None:
            post()
    return ride_fwd_bwd, shard_step, {"slices": len(riders), "state": state}


def ride_rest(covered, numel):
    """The flat ranges of [0, numel) no ride group covers (the end-of-step update's ranges), in
    order; ``covered``: the groups' [lo, hi) ranges, which must not overlap."""
    covered = sorted(covered)
    if any(a[1] > b[0] for a, b in zip(covered, covered[1:])):
        raise ValueError("ride plan: groups overlap in the flat layout")
    rest, pos = [], 0
    for a, b in covered:
        if a > pos:
            rest.append((pos, a))
        pos = max(pos, b)
    if pos < numel:
        rest.append((pos, numel))
    return rest


def _ride(model, space, optimizer, fwd_bwd, post, get_fold, scale):
    """make_train_step's ``ride``: SgdRider slices of each ride group armed on its host convs for
    the duration of the step's backward; the end-of-step SGD covers the remaining ranges."""
    from ..ops import kernels as K
    g = optimizer.param_groups[0]
    dev = space.grad.device
    mom = optimizer._bufs(space, ["momentum"])["momentum"] if g["momentum"] != 0 else None
    first = optimizer.first_tensor(dev) if mom is not None else None
    lr = optimizer.lr_tensor(dev)
    blocks = 512   # rider blocks per launch: measured, 32 / 64 lose, 512-1024 best
    riders, covered, seen = [], [], set()       # riders: (group, SgdRider)
    groups = model.ride_plan()
    holder = {}                                 # this step's take(): set below

    def take_for(j):
        return lambda: holder["take"](j)
    for gi, (params, hosts) in enumerate(groups):
        lo, hi = space.range_of(params)
        if hi <= lo or not hosts or any(id(h) in seen for h in hosts):
            raise ValueError("ride plan: each group needs parameters and host convs of its own")
        seen.update(id(h) for h in hosts)
        covered.append((lo, hi))
        n = len(hosts)
        cuts = [lo + ((hi - lo) * i // n) // 64 * 64 for i in range(n)] + [hi]
        for i, (conv, a, b) in enumerate(zip(hosts, cuts, cuts[1:])):
            r = None if b <= a else K.SgdRider(
                space.master[a:b], space.grad[a:b], None if mom is None else mom[a:b],
                None if space.shadow is None else space.shadow[a:b], lr, first, g["weight_decay"], g["momentum"],
                g["dampening"], g["nesterov"], scale, blocks)
            riders.append((gi, r))
            object.__setattr__(conv, "_kml_rider", take_for(len(riders) - 1))
    rest = ride_rest(covered, space.numel)
    state = {"active": False, "fired": set(), "taken": set()}

    def _rider_take_impl(j):
        gi, r = riders[j]
        if not state["active"] or r is None or j in state["taken"]:
            return None
        if gi not in state["fired"]:
            space.finish_grads(groups[gi][0])   # e.g. layer3's deferred folds, one launch, here
            state["fired"].add(gi)
        state["taken"].add(j)
        return r
    holder["take"] = _rider_take_impl

    def ride_fwd_bwd():
        state["active"], state["fired"], state["taken"] = True, set(), set()
        try:
            return fwd_bwd()
        finally:
            state["active"] = False

    def ride_opt_step():
        optimizer.set_grad_scale(scale)
        # a host conv whose backward did not run (or took another path) leaves its slice to here
        for j, (gi, r) in enumerate(riders):
            if r is not None and j not in state["taken"]:
                r.run_alone()
        for k, (a, b) in enumerate(rest):
            optimizer.step_range(a, b, max_blocks=2048, advance=get_fold() if k == len(rest) - 1 else None)
        if not rest and get_fold() is not None:
            K.advance_counter_(*get_fold())
        optimizer.finish_ranges()
        if post is not None:
            post()
    return ride_fwd_bwd, ride_opt_step

