"""Training-dynamics parity: the bf16 HIP path against stock fp32 PyTorch.

The reference's headline results are time-to-accuracy and final accuracy of ResNet-34 on
CIFAR-10, trained in fp32 (torch 1.7.1, no AMP).  There is no CIFAR-10 in the
container, so this trains on a LEARNABLE synthetic CIFAR-shaped task instead: 10 classes,
each a fixed random low-frequency colour template; a sample is its class template at a
random contrast, shifted by up to 3 pixels, plus per-pixel noise.  Both runs see the same
init (the torchvision-named state_dict is copied), the same batches in the same order and
the same augmentation (our on-device crop/flip/normalise kernel produces each batch once;
the fp32 model gets it as NCHW fp32 — identical inputs up to the bf16 rounding of the
normalised pixels):

  * ours:  kubeml_amd ResNet-34 (NHWC bf16, hand-written HIP kernels, fp32 master weights,
           graph-captured step via engine/dp.py make_train_step, fused SGD)
  * stock: models/torch_reference.resnet34 in fp32 NCHW (MIOpen / hipBLASLt), torch.optim.SGD

Both: SGD(lr, momentum, wd 1e-4), batch 256, ImageNet stem + 1000-class head (as the
reference's function_resnet34.py).  Writes the loss curves and final accuracies as JSON.

    python tools/convergence_check.py [--steps 1200] [--out profiles/convergence_r3.json]
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def make_task(n, g, dev, templates, noise=40.0, label_noise=0.0):
    import torch
    cls = torch.randint(0, 10, (n,), device=dev, generator=g)
    contrast = 0.6 + 0.8 * torch.rand(n, 1, 1, 1, device=dev, generator=g)
    img = templates[cls] * contrast                                  # [n, 38, 38, 3] float
    sy = torch.randint(0, 7, (n,), device=dev, generator=g)
    sx = torch.randint(0, 7, (n,), device=dev, generator=g)
    rows = (sy.view(n, 1) + torch.arange(32, device=dev).view(1, 32))  # [n, 32]
    cols = (sx.view(n, 1) + torch.arange(32, device=dev).view(1, 32))
    img = img[torch.arange(n, device=dev).view(n, 1, 1), rows.view(n, 32, 1), cols.view(n, 1, 32)]
    img = img + noise * torch.randn(img.shape, device=dev, generator=g)
    labels = cls.clone()
    if label_noise > 0:   # training labels only: a fraction replaced by uniform random classes
        flip = torch.rand(n, device=dev, generator=g) < label_noise
        labels[flip] = torch.randint(0, 10, (int(flip.sum()),), device=dev, generator=g)
    return img.clamp(0, 255).round().to(torch.uint8).contiguous(), labels


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=1200)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--lr", type=float, default=0.05)
    ap.add_argument("--momentum", type=float, default=0.9)
    ap.add_argument("--n-train", type=int, default=25600)
    ap.add_argument("--n-test", type=int, default=5120)
    ap.add_argument("--log-every", type=int, default=25)
    ap.add_argument("--eval-every", type=int, default=200, help="validation accuracy of both paths every N steps")
    ap.add_argument("--noise", type=float, default=70.0, help="per-pixel Gaussian noise (uint8 units)")
    ap.add_argument("--mix", type=float, default=0.75,
                    help="share of a template common to every class (higher: classes overlap more)")
    ap.add_argument("--label-noise", type=float, default=0.2, help="fraction of random training labels")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "convergence.json"))
    a = ap.parse_args()

    import torch
    import torch.nn.functional as F
    from kubeml_amd.engine.dp import make_train_step
    from kubeml_amd.models import torch_reference as TR
    from kubeml_amd.models.resnet import resnet34
    from kubeml_amd.nn import cross_entropy, flatten_module
    from kubeml_amd.ops import kernels as K
    from kubeml_amd.optim import SGD

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(2024)
    # low-frequency colour templates (8x8 random field upsampled to 38x38)
    common = torch.rand(1, 3, 8, 8, device=dev, generator=g) * 255.0
    base = a.mix * common + (1.0 - a.mix) * torch.rand(10, 3, 8, 8, device=dev, generator=g) * 255.0
    templates = F.interpolate(base, size=(38, 38), mode="bilinear", align_corners=False).permute(0, 2, 3, 1)
    xtr, ytr = make_task(a.n_train, g, dev, templates, a.noise, a.label_noise)
    xte, yte = make_task(a.n_test, g, dev, templates, a.noise, 0.0)
    B = a.batch

    torch.manual_seed(7)
    ours = resnet34(num_classes=1000).to(dev)
    ref = TR.resnet34(num_classes=1000).to(dev)
    ref.load_state_dict({k: v.detach().float().cpu() for k, v in ours.state_dict().items()})
    space = flatten_module(ours)
    ours.train()
    ref.train()
    opt = SGD(ours.parameters(), lr=a.lr, momentum=a.momentum, weight_decay=1e-4)
    ropt = torch.optim.SGD(ref.parameters(), lr=a.lr, momentum=a.momentum, weight_decay=1e-4)

    # every batch augmented ONCE (our kernel), consumed by both models
    ctr = torch.tensor([11.0, 0.0, 0.0], dtype=torch.float32, device=dev)
    xb = torch.empty((B, 32, 32, 8), dtype=torch.bfloat16, device=dev)
    yb = torch.empty((B,), dtype=torch.int64, device=dev)
    xin = torch.empty_like(xb)
    yin = torch.empty_like(yb)
    step = make_train_step(ours, space, opt, cross_entropy, xin, yin, extra_state=[])
    step.capture()

    def evaluate(model, fp32):
        model.eval()
        vctr = torch.zeros(3, dtype=torch.float32, device=dev)
        correct, tot, loss_sum = 0, 0, 0.0
        with torch.no_grad():
            for _ in range(a.n_test // B):
                K.augment(xte, yte, vctr, B, out=xb, labels_out=yb, pad=0, flip=False, train=False)
                K.advance_counter_(vctr, B, a.n_test)
                if fp32:
                    out = model(xb[..., :3].float().permute(0, 3, 1, 2).contiguous())
                else:
                    out = model(xb).float()
                loss_sum += float(F.cross_entropy(out, yb, reduction="sum"))
                correct += int((out.argmax(1) == yb).sum())
                tot += B
        model.train()
        return 100.0 * correct / tot, loss_sum / tot

    curve, val_curve = [], []
    t0 = time.time()
    for s in range(a.steps):
        K.augment(xtr, ytr, ctr, B, out=xb, labels_out=yb, train=True)
        K.advance_counter_(ctr, B, a.n_train)
        xin.copy_(xb)
        yin.copy_(yb)
        lo = step()
        # stock fp32 on the same batch
        ropt.zero_grad(set_to_none=True)
        lr_ = F.cross_entropy(ref(xb[..., :3].float().permute(0, 3, 1, 2).contiguous()), yb)
        lr_.backward()
        ropt.step()
        if s % a.log_every == 0 or s == a.steps - 1:
            curve.append({"step": s, "ours": round(float(lo), 4), "stock_fp32": round(float(lr_), 4)})
            print(json.dumps(curve[-1]), flush=True)
        if a.eval_every and (s + 1) % a.eval_every == 0 and s + 1 < a.steps:
            ao, _ = evaluate(ours, False)
            ar, _ = evaluate(ref, True)
            val_curve.append({"step": s + 1, "ours_acc": round(ao, 2), "stock_fp32_acc": round(ar, 2)})
            print(json.dumps(val_curve[-1]), flush=True)
    acc_o, vl_o = evaluate(ours, False)
    acc_r, vl_r = evaluate(ref, True)
    epochs = a.steps * B / a.n_train
    val_curve.append({"step": a.steps, "ours_acc": round(acc_o, 2), "stock_fp32_acc": round(acc_r, 2)})
    res = {"task": (f"synthetic learnable CIFAR-shaped (10 overlapping class templates, mix {a.mix}, shift, "
                    f"contrast, noise {a.noise}, {100 * a.label_noise:.0f}% random training labels)"),
           "model": "resnet34 (ImageNet stem, 1000-class head)", "batch": B, "steps": a.steps,
           "epochs": round(epochs, 2), "optimizer": f"SGD lr={a.lr} momentum={a.momentum} wd=1e-4",
           "ours": {"path": "kubeml_amd bf16 HIP kernels, fp32 master, graphed step",
                    "final_val_acc": round(acc_o, 2), "final_val_loss": round(vl_o, 4)},
           "stock_fp32": {"path": "torch fp32 NCHW (MIOpen/hipBLASLt), torch.optim.SGD",
                          "final_val_acc": round(acc_r, 2), "final_val_loss": round(vl_r, 4)},
           "acc_gap_points": round(acc_o - acc_r, 2), "wall_s": round(time.time() - t0, 1),
           "val_curve": val_curve, "curve": curve}
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k not in ("curve", "val_curve")}), flush=True)
    if not all(math.isfinite(c["ours"]) for c in curve):
        sys.exit(1)


if __name__ == "__main__":
    main()
