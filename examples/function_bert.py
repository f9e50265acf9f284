"""BERT-base masked-LM pre-training function (north-star config 5; the reference has no
transformer workload, so this follows its function shape, ml/experiments/kubeml/
function_resnet34.py:47-104, on the BERT model).

Dataset: token ids uploaded through the storage API like any other dataset —
``kubeml dataset create --traindata ids.npy --trainlabels seg.npy ...`` with ``ids.npy``
an int64 ``[N, L]`` array of WordPiece ids and ``seg.npy`` an int64 ``[N]`` array (unused by
MLM; the storage format needs a label per sample).  Masking happens on the device per
batch (Google BERT's recipe): 15 % of the positions, at most 76 per 512-token sequence, are
predicted; of those 80 % become [MASK], 10 % a random token, 10 % stay.

Model: HuggingFace-layout BertForMaskedLM (kubeml_amd/models/bert.py) on the hand-written
MFMA GEMM / flash-attention kernels; optimizer AdamW (fused single launch on the GPU).
Validation reports masked-token accuracy (%) and MLM loss.

GPU path: masking (one HIP kernel, ``kernels.mlm_mask``: a fresh mask per replay from a device
counter), forward, loss, backward and AdamW of a batch are ONE hipGraph replay
(``self.step(..., forward=...)``); validation is a captured eval forward with a fixed mask.
Train with ``kubeml train -f bert --K 1 --grad-sync`` for synchronous data parallelism with
persistent Adam moments (the reference semantics — an optimizer rebuilt every round — would
make every AdamW step a first step).  CPU workers run the same recipe with stock torch ops.
"""
from typing import Tuple

import numpy as np
import torch
from torch.optim import AdamW

from kubeml import KubeDataset, KubeModel
from kubeml_amd.models.bert import BertForMaskedLM

MASK_ID, VOCAB = 103, 30522
MASK_FRAC, MAX_PREDS = 0.15, 76


class TokenDataset(KubeDataset):
    def __init__(self, name="wiki_tokens"):
        super().__init__(name)

    def collate_batch(self, data: np.ndarray, labels: np.ndarray):
        return (torch.from_numpy(np.ascontiguousarray(data).astype(np.int64)),
                torch.from_numpy(np.ascontiguousarray(labels).reshape(-1).astype(np.int64)))

    def __getitem__(self, i):
        return self.data[i], int(self.labels[i])

    def __len__(self):
        return len(self.data) if self.data is not None else 0


def mask_tokens(ids: torch.Tensor, gen: torch.Generator):
    """(masked input ids, positions [B, P], labels [B, P]) — BERT's 80/10/10 recipe."""
    B, L = ids.shape
    P = min(MAX_PREDS, max(1, int(round(L * MASK_FRAC))))
    score = torch.rand(B, L, device=ids.device, generator=gen)
    pos = score.topk(P, dim=1).indices.sort(dim=1).values
    lab = ids.gather(1, pos)
    r = torch.rand(B, P, device=ids.device, generator=gen)
    rnd = torch.randint(0, VOCAB, (B, P), device=ids.device, generator=gen)
    repl = torch.where(r < 0.8, torch.full_like(lab, MASK_ID), torch.where(r < 0.9, rnd, lab))
    x = ids.clone()
    x.scatter_(1, pos, repl)
    return x, pos.contiguous(), lab.contiguous()


def _preds(L):
    return min(MAX_PREDS, max(1, int(round(L * MASK_FRAC))))


class KubeBert(KubeModel):
    def __init__(self, network, dataset):
        super().__init__(network, dataset, gpu=True)
        self._gen = None
        self._ctr = {}     # "train" / "val" -> device [seed, step] of the masking kernel

        # captured with the step / eval graphs, so created once (their identity keys the graphs)
        def fwd_train(net, ids, seg):
            from kubeml_amd.ops import kernels as K
            x, pos, lab = K.mlm_mask(ids, self._counter("train"), _preds(ids.shape[1]), MASK_ID, VOCAB)
            return net(x, mlm_positions=pos, labels=lab)

        def fwd_val(net, ids, seg):
            from kubeml_amd.ops import kernels as K
            x, pos, lab = K.mlm_mask(ids, self._counter("val"), _preds(ids.shape[1]), MASK_ID, VOCAB, advance=False)
            loss, correct = net(x, mlm_positions=pos, labels=lab, return_correct=True)
            return correct, loss
        self._fwd_train, self._fwd_val = fwd_train, fwd_val

    def _counter(self, split):
        t = self._ctr.get(split)
        if t is None or t.device != self.device:
            seed = 1 + self.args._func_id + (7919 if split == "val" else 0)
            t = self._ctr[split] = torch.tensor([float(seed), 0.0], dtype=torch.float32, device=self.device)
        return t

    def _generator(self):
        if self._gen is None or self._gen.device != self.device:
            self._gen = torch.Generator(device=self.device).manual_seed(1 + self.args._func_id)
        return self._gen

    def configure_optimizers(self) -> torch.optim.Optimizer:
        return AdamW(self.parameters(), lr=self.lr, weight_decay=0.01)

    def train(self, batch, batch_index) -> float:
        ids, seg = batch
        if ids.is_cuda:
            return self.step(ids, seg, forward=self._fwd_train)   # device loss: read back once per task
        x, pos, lab = mask_tokens(ids, self._generator())
        self.optimizer.zero_grad()
        loss = self(x, mlm_positions=pos, labels=lab)
        loss.backward()
        self.optimizer.step()
        return loss.detach()

    def validate(self, batch, batch_index) -> Tuple[float, float]:
        ids, seg = batch
        if ids.is_cuda:
            correct, loss = self.evaluate(ids, seg, forward=self._fwd_val)
            return correct * 100 / (ids.shape[0] * _preds(ids.shape[1])), loss
        x, pos, lab = mask_tokens(ids, self._generator())
        loss, correct = self(x, mlm_positions=pos, labels=lab, return_correct=True)
        return correct * 100 / lab.numel(), loss

    def infer(self, data):
        ids = torch.tensor(data, dtype=torch.int64, device=self.device)
        return self(ids).float().argmax(-1)


def main():
    return KubeBert(BertForMaskedLM(), TokenDataset()).start()
