"""ResNet family on the MI355X-native layers (torchvision-compatible names/shapes).

``resnet34()`` is the reference's headline workload: torchvision ``resnet34()`` with
the ImageNet stem (7x7/2 conv + 3x3/2 max-pool) and the 1000-class head, trained on
32x32 CIFAR-10 images (ml/experiments/kubeml/function_resnet34.py:101).  With that
stem the spatial size is 16 -> 8 -> 8 -> 4 -> 2 -> 1, so layer4 runs at 1x1 and the
implicit-GEMM kernels collapse its 3x3 convolutions to their centre tap.

GPU training runs every residual block as ONE autograd node (:class:`BlockFn`):
conv(+BN-stats) -> BN(+residual)+ReLU forward, fused BN-backward / split-K wgrad /
dgrad(+residual-gradient) backward.  ``state_dict()`` is key-for-key and
shape-for-shape torchvision's, so reference checkpoints load unchanged.
Also: ``resnet50`` (Bottleneck, north-star config 3) and CIFAR ResNet-20/32/44/56
(option-A shortcut, reference ml/experiments/kubeml/resnet32.py:44-146).
"""
from __future__ import annotations

import torch
import torch.nn as tnn
import torch.nn.functional as F

from ..nn import modules as M
from ..nn.fused import BlockFn, BNRegistry, ConvBNUnit, block_params, refresh_transposed


def _gpu_train(x):
    return x.is_cuda and torch.is_grad_enabled()


class BasicBlock(tnn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = M.Conv2d(inplanes, planes, 3, stride, 1, bias=False)
        self.bn1 = M.BatchNorm2d(planes)
        self.relu = M.ReLU(inplace=True)
        self.conv2 = M.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = M.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride
        plan = [(self.conv1, self.bn1, True, "main")]
        if downsample is not None:
            plan.append((downsample[0], downsample[1], False, "short"))
        plan.append((self.conv2, self.bn2, True, "last"))
        self._kml_plan = plan

    def forward(self, x):
        if x.is_cuda:
            if _gpu_train(x) and self.training:
                return BlockFn.apply(x, self, *block_params(self))
            return _block_eval(self, x)
        idt = x if self.downsample is None else self.downsample(x)
        out = self.bn1(self.conv1(x), relu=True)
        return self.bn2(self.conv2(out), relu=True, residual=idt)


class Bottleneck(tnn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = M.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = M.BatchNorm2d(planes)
        self.conv2 = M.Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.bn2 = M.BatchNorm2d(planes)
        self.conv3 = M.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = M.BatchNorm2d(planes * 4)
        self.relu = M.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride
        plan = [(self.conv1, self.bn1, True, "main"), (self.conv2, self.bn2, True, "main")]
        if downsample is not None:
            plan.append((downsample[0], downsample[1], False, "short"))
        plan.append((self.conv3, self.bn3, True, "last"))
        self._kml_plan = plan

    def forward(self, x):
        if x.is_cuda:
            if _gpu_train(x) and self.training:
                return BlockFn.apply(x, self, *block_params(self))
            return _block_eval(self, x)
        idt = x if self.downsample is None else self.downsample(x)
        out = self.bn1(self.conv1(x), relu=True)
        out = self.bn2(self.conv2(out), relu=True)
        return self.bn3(self.conv3(out), relu=True, residual=idt)


def _block_eval(block, x):
    """Inference / no-grad forward (running or batch statistics, no saved tensors)."""
    training = block.training
    short = None
    h = x
    for conv, bn, relu, role in block._kml_plan:
        if role == "short":
            short, _ = ConvBNUnit.forward(x, conv, bn, relu, None, training)
        elif role == "last":
            h, _ = ConvBNUnit.forward(h, conv, bn, relu, short if short is not None else x, training)
        else:
            h, _ = ConvBNUnit.forward(h, conv, bn, relu, None, training)
    return h


class _Stem(tnn.Module):
    """Holds nothing; ResNet.forward drives conv1/bn1/maxpool (names stay top-level)."""


class ResNet(tnn.Module):
    def __init__(self, block, layers, num_classes=1000, in_channels=3):
        super().__init__()
        self.inplanes = 64
        self.conv1 = M.Conv2d(in_channels, 64, 7, 2, 3, bias=False)
        self.bn1 = M.BatchNorm2d(64)
        self.relu = M.ReLU(inplace=True)
        self.maxpool = M.MaxPool2d(3, 2, 1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], 2)
        self.layer3 = self._make_layer(block, 256, layers[2], 2)
        self.layer4 = self._make_layer(block, 512, layers[3], 2)
        self.avgpool = M.AdaptiveAvgPool2d((1, 1))
        self.fc = M.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, M.Conv2d):
                tnn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, M.BatchNorm2d):
                tnn.init.constant_(m.weight, 1)
                tnn.init.constant_(m.bias, 0)
        self._arena = BNRegistry([m for m in self.modules() if isinstance(m, M.BatchNorm2d)])
        # backward fusion chain: each block's first dgrad emits the previous block's last-BN
        # dgamma/dbeta partials (nn/fused.py); weak links, not submodules
        import weakref
        blocks = [b for layer in (self.layer1, self.layer2, self.layer3, self.layer4) for b in layer]
        for prev, b in zip([None] + blocks[:-1], blocks):
            object.__setattr__(b, "_kml_prev_ref", weakref.ref(prev) if prev is not None else None)
        # forward fusion chain: a block may leave its output BN to the next block's first conv
        for b, nxt in zip(blocks, blocks[1:] + [None]):
            object.__setattr__(b, "_kml_next_ref", weakref.ref(nxt) if nxt is not None else None)
        object.__setattr__(self, "_kml_blocks", blocks)

    def _make_layer(self, block, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = tnn.Sequential(M.Conv2d(self.inplanes, planes * block.expansion, 1, stride, bias=False),
                                        M.BatchNorm2d(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * block.expansion
        layers += [block(self.inplanes, planes) for _ in range(1, blocks)]
        return tnn.Sequential(*layers)

    def forward(self, x):
        """x: NHWC bf16 (channels padded to 8) on GPU, or NCHW float (converted)."""
        with self._chain(x):
            x = self._head(x)
            x = self.layer4(self.layer3(x))
        return self._classify(x)

    def _classify(self, x):
        """avgpool + fc of layer4's output, on every forward path (plain and staged): at 1x1 maps
        the classifier reads the last block's output as is, so its dgrad can hand that block's
        output-BN partial rows over (nn/modules.py _LinearFn); the hand-off flag is decided here
        for each forward, never left over from another path's forward."""
        last = self.layer4[-1]
        object.__setattr__(self.fc, "_kml_bnf_block",
                           last if (self.training and x.is_cuda and x.dim() == 4 and x.shape[1] * x.shape[2] == 1
                                    and getattr(last, "_kml_plan", None) is not None) else None)
        return self.fc(self.avgpool(x))

    def _chain(self, x):
        """Training forward on the GPU: blocks may hand their output BN to the next block's
        first conv (nn/fused.py cross-block fold); every deferred output is applied by the end."""
        import contextlib
        if x.is_cuda and self.training and torch.is_grad_enabled():
            from ..nn.fused import chain
            return chain(self._kml_blocks)
        return contextlib.nullcontext()

    def _chained(self, layer):
        def run(h):
            with self._chain(h):
                return layer(h)
        return run

    def _head(self, x):
        return self.layer2(self._stem_l1(x))

    def _stem_l1(self, x):
        if x.dim() == 4 and (x.shape[-1] not in (self.conv1.in_channels, self.conv1.cin_pad)
                             or x.dtype != torch.bfloat16 and x.is_cuda):
            x = M.to_nhwc(x, self.conv1.cin_pad)
        if x.is_cuda:
            if self.training:
                if not (torch.is_grad_enabled() and _STEM_FUSE):
                    self._bump_counters()      # else the fused stem kernel bumps them
                if torch.is_grad_enabled():
                    convs = getattr(self, "_kml_convs", None)
                    if convs is None:
                        convs = [m for m in self.modules() if isinstance(m, M.Conv2d)]
                        object.__setattr__(self, "_kml_convs", convs)
                    refresh_transposed(convs)
            x = self._stem_gpu(x)
        else:
            x = self.maxpool(self.bn1(self.conv1(x), relu=True))
        return self.layer1(x)

    def stages(self):
        """Forward split for overlapped gradient all-reduce (engine/staged.py):
        [stem+layer1, layer2, layer3, layer4+head].  Parameters of later stages sit first in
        the flat buffer, so each stage's gradients are one contiguous range.  Backward runs
        the stages in reverse, so the all-reduce that nothing can hide (the first stage's)
        carries only the stem + layer1 gradients (~1 % of ResNet-34's 87 MB)."""
        return [self._chained(self._stem_l1), self._chained(self.layer2), self._chained(self.layer3),
                lambda h: self._classify(self._chained(self.layer4)(h))]

    def ride_plan(self):
        """[(parameters, host convs), ...] for engine/dp.py ``ride``: each group's SGD update runs
        in extra blocks of its host convs' grouped backward launches, which all run after the
        group's gradients are final (backward order: fc, layer4, layer3, layer2, layer1).
        ``KUBEML_RIDE_PLAN`` = groups separated by ``;``, each ``<layers>:<host layers>`` with
        ``f`` for fc and host ``s`` for the stem conv: "4f:3;3:21" rides layer4 + fc on layer3's convs
        and layer3 on layer2's and layer1's; "123:s" rides layers 1-3 on the stem's weight-gradient
        launch (the last of the backward: 416 latency-bound tiles, kernels.conv_wgrad's rider
        z-slices).  Layer3's 3x3 convs run unrolled; their deferred gradient fold runs when the
        first host of a group holding layer3 takes its slice (the same single fold launch, earlier)."""
        import os
        spec = os.environ.get("KUBEML_RIDE_PLAN")
        if spec is None:
            # measured on ResNet-34 / CIFAR (BasicBlock); other depths ride only when asked
            if not isinstance(self.layer1[0], BasicBlock):
                return []
            spec = "4f:321;123:s"
        groups = []
        for part in filter(None, spec.split(";")):
            own, host = part.split(":")
            ps = [p for d in own for p in (self.fc if d == "f" else getattr(self, f"layer{d}")).parameters()]
            # the riders sit on the hosts' conv-backward pairs (BN-backward hosts measured no better)
            hosts = [m for d in host for m in
                     ([self.conv1] if d == "s" else getattr(self, f"layer{d}").modules()) if isinstance(m, M.Conv2d)]
            groups.append((ps, hosts))
        return groups

    def comm_ride_plan(self):
        """[(parameters, RS host convs, AG host convs)] of the peer-shard riders (engine/dp.py
        ``shardride``, N > 1): layer4 + fc (62 % of ResNet-34's gradient bytes) reduce-scatter + SGD
        in layer3's 13 backward launches and all-gather in the last 4 of layer2's; layer3 (31 %)
        reduce-scatters + SGD in the first 5 of layer2's and all-gathers in layer1's 6.  Only
        layer2 + layer1 + stem (7 %) remain after the backward.  Measured against spreading
        layer3's reduce-scatter over all 9 layer2 launches (both gathers in layer1): 1.405 vs
        1.448 ms per 1-rank rehearsal step; riding every 2nd / 3rd launch only (thicker slices):
        1.408 / 1.414 vs 1.392 ms; adding the BN-backward launches as hosts (56 slices): 1.50 ms
        (profiles/r6/shardride.md).  BasicBlock nets only, [] otherwise."""
        if not isinstance(self.layer1[0], BasicBlock):
            return []

        def convs(layer):
            return [m for m in layer.modules() if isinstance(m, M.Conv2d)]
        l2 = convs(self.layer2)
        half = len(l2) // 2
        # backward runs layer2's convs in reverse module order: l2[half:] (the second stage's
        # reduce-scatter) first, then l2[:half] (the first stage's gather)
        return [(list(self.layer4.parameters()) + list(self.fc.parameters()), convs(self.layer3), l2[:half]),
                (list(self.layer3.parameters()), l2[half:], convs(self.layer1))]

    def stage_params(self):
        """Parameters owned by each stage of :meth:`stages`."""
        later = ("layer2.", "layer3.", "layer4.", "fc.")
        head = [p for n, p in self.named_parameters() if not n.startswith(later)]
        return [head, list(self.layer2.parameters()), list(self.layer3.parameters()),
                list(self.layer4.parameters()) + list(self.fc.parameters())]

    def _bump_counters(self):
        from ..ops import kernels as K
        K.add_i64_(self._counter_arena())

    def _counter_arena(self):
        # num_batches_tracked of every BN: one tiny kernel each is avoided by keeping
        # the counters in one int64 arena (allocated on first use)
        arena = getattr(self, "_nbt_arena", None)
        bns = self._arena.bns
        if arena is None or arena.device != bns[0].running_mean.device:
            dev = bns[0].running_mean.device
            ts = [bn.num_batches_tracked for bn in bns]
            if ts[0].device == dev and all(t.data_ptr() == ts[0].data_ptr() + 8 * i for i, t in enumerate(ts)):
                arena = ts[0].as_strided((len(bns),), (1,))   # already packed (nn/flat.py)
            else:
                arena = torch.zeros(len(bns), dtype=torch.int64, device=dev)
                for i, bn in enumerate(bns):
                    arena[i] = bn.num_batches_tracked.to(dev)
                    bn.num_batches_tracked = arena[i]
            self._nbt_arena = arena
        return arena

    def _stem_gpu(self, x):
        if torch.is_grad_enabled() and self.training:
            return _StemFn.apply(x, self, self.conv1.weight, self.bn1.weight, self.bn1.bias)
        y, _ = ConvBNUnit.forward(x, self.conv1, self.bn1, True, None, self.training)
        from ..ops import kernels as K
        y, _ = K.maxpool_fwd(y, 3, 2, 1)
        return y


class _StemFn(torch.autograd.Function):
    """conv1 -> bn1 -> ReLU -> max-pool of the training forward.  BN-apply, ReLU and the pool
    run as ONE pass (``bn_relu_maxpool``: the full-resolution normalised map is never
    written); backward folds the ReLU mask into the gather max-pool backward, so the BN
    backward reads dz and the conv output only.  ``_STEM_FUSE = False``: unfused path (tests)."""

    @staticmethod
    def forward(ctx, x, net, *params):
        from ..ops import kernels as K
        if not _STEM_FUSE:
            y, s = ConvBNUnit.forward(x, net.conv1, net.bn1, True, None, True)
            p, idx = K.maxpool_fwd(y, 3, 2, 1)
            ctx.net, ctx.s, ctx.idx, ctx.yshape, ctx.p = net, s, idx, y.shape, None
            return p
        conv, bn = net.conv1, net.bn1
        from ..nn.flat import master_of, shadow_of
        w = shadow_of(conv.weight)
        kh, kw = conv.kernel_size
        G = K.conv_fwd_stats_rows(x.shape, w.shape[0], kh, kw, conv.stride, conv.padding)
        stats = torch.empty(G * 2 * w.shape[0], dtype=torch.float32, device=x.device)
        c = K.conv_fwd(x, w, kh, kw, conv.stride, conv.padding, stats=stats, stats_part=True)
        C = c.shape[-1]
        mean = torch.empty(C, dtype=torch.float32, device=x.device)
        rstd = torch.empty_like(mean)
        # the model's BN num_batches_tracked counters are bumped by this kernel's block 0 (one
        # launch less per step; _stem_l1 skips its own bump on this path)
        p, idx = K.bn_relu_maxpool(c, stats, master_of(bn.weight), master_of(bn.bias), 3, 2, 1, save_mean=mean,
                                   save_rstd=rstd, run_mean=bn.running_mean, run_var=bn.running_var, eps=bn.eps,
                                   momentum=bn.momentum if bn.momentum is not None else 0.1, stats_rows=G,
                                   counters=net._counter_arena())
        # saved like a ConvBNUnit without ReLU: the mask travels in the pooled output
        ctx.net, ctx.s, ctx.idx, ctx.yshape, ctx.p = net, (x, c, None, mean, rstd), idx, c.shape, p
        return p

    @staticmethod
    def backward(ctx, dp):
        from ..ops import kernels as K
        net = ctx.net
        dy = K.maxpool_bwd(dp.contiguous(), ctx.idx, ctx.yshape, 3, 2, 1, relu_out=ctx.p)
        dx, _, _ = ConvBNUnit.backward(dy, ctx.s, net.conv1, net.bn1, False, ctx.needs_input_grad[0])
        ctx.s = ctx.idx = ctx.p = None
        return (dx, None) + (None,) * (len(ctx.needs_input_grad) - 2)


_STEM_FUSE = True


def resnet18(num_classes=1000, **kw):
    return ResNet(BasicBlock, [2, 2, 2, 2], num_classes, **kw)


def resnet34(num_classes=1000, **kw):
    return ResNet(BasicBlock, [3, 4, 6, 3], num_classes, **kw)


def resnet50(num_classes=1000, **kw):
    return ResNet(Bottleneck, [3, 4, 6, 3], num_classes, **kw)


# ---------------------------------------------------------------------------------------
# CIFAR ResNet (He et al. 2016, option-A identity shortcut) — reference resnet32.py
# ---------------------------------------------------------------------------------------

class _ShortcutAFn(torch.autograd.Function):
    """Option-A shortcut on the GPU: one gather launch each way (pool.hip k_shortcut_a_*)."""

    @staticmethod
    def forward(ctx, x, pad):
        from ..ops import kernels as K
        ctx.shape, ctx.pad = tuple(x.shape), pad
        return K.shortcut_a_fwd(x.contiguous(), pad)

    @staticmethod
    def backward(ctx, dy):
        from ..ops import kernels as K
        return K.shortcut_a_bwd(dy.contiguous(), ctx.shape, ctx.pad), None


class _LambdaShortcut(tnn.Module):
    """Option A: stride-2 subsample + zero-pad channels (parameter-free) — reference
    ml/experiments/kubeml/resnet32.py LambdaLayer.  bf16 CUDA tensors take the in-tree HIP
    gather; CPU keeps the stock slice + ``F.pad`` it is checked against."""

    def __init__(self, planes):
        super().__init__()
        self.pad = planes // 4

    def forward(self, x):  # NHWC
        if x.is_cuda and x.dtype == torch.bfloat16:
            return _ShortcutAFn.apply(x, self.pad)
        y = x[:, ::2, ::2, :]
        return F.pad(y, (self.pad, self.pad)).contiguous()


class CifarBasicBlock(tnn.Module):
    def __init__(self, in_planes, planes, stride=1):
        super().__init__()
        self.conv1 = M.Conv2d(in_planes, planes, 3, stride, 1, bias=False)
        self.bn1 = M.BatchNorm2d(planes)
        self.conv2 = M.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = M.BatchNorm2d(planes)
        self.shortcut = _LambdaShortcut(planes) if (stride != 1 or in_planes != planes) else None

    def forward(self, x):
        idt = x if self.shortcut is None else self.shortcut(x)
        out = self.bn1(self.conv1(x), relu=True)
        return self.bn2(self.conv2(out), relu=True, residual=idt)


class CifarResNet(tnn.Module):
    def __init__(self, num_blocks, num_classes=10):
        super().__init__()
        self.in_planes = 16
        self.conv1 = M.Conv2d(3, 16, 3, 1, 1, bias=False)
        self.bn1 = M.BatchNorm2d(16)
        self.layer1 = self._make(16, num_blocks, 1)
        self.layer2 = self._make(32, num_blocks, 2)
        self.layer3 = self._make(64, num_blocks, 2)
        self.linear = M.Linear(64, num_classes)
        for m in self.modules():
            if isinstance(m, (M.Conv2d, M.Linear)):
                tnn.init.kaiming_normal_(m.weight)

    def _make(self, planes, n, stride):
        layers = []
        for s in [stride] + [1] * (n - 1):
            layers.append(CifarBasicBlock(self.in_planes, planes, s))
            self.in_planes = planes
        return tnn.Sequential(*layers)

    def forward(self, x):
        if x.dim() == 4 and x.shape[1] == 3 and x.shape[-1] != 3:
            x = M.to_nhwc(x, self.conv1.cin_pad)
        out = self.bn1(self.conv1(x), relu=True)
        out = self.layer3(self.layer2(self.layer1(out)))
        B, H, W, C = out.shape
        out = out.reshape(B, H * W, C).float().mean(1) if not out.is_cuda else M.AdaptiveAvgPool2d()(out)
        return self.linear(out)


def resnet20(num_classes=10):
    return CifarResNet(3, num_classes)


def resnet32(num_classes=10):
    return CifarResNet(5, num_classes)


def resnet44(num_classes=10):
    return CifarResNet(7, num_classes)


def resnet56(num_classes=10):
    return CifarResNet(9, num_classes)
