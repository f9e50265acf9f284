"""BERT-base masked-LM (north-star config 5 — absent from the reference).

HuggingFace ``BertForMaskedLM`` architecture and ``state_dict`` names
(``bert.embeddings.*``, ``bert.encoder.layer.{i}.attention.self.query.weight``, ...,
``cls.predictions.transform.*``, ``cls.predictions.decoder.weight`` tied to the word
embeddings) on the MI355X layers:

* token-major bf16 activations ``[B*L, 768]``; fused QKV projection (one ``[T, 2304]`` GEMM
  per layer); the weight gradients (deterministic fp32 slab split-K) and FFN2's dgrad (FFN1's
  GELU backward in its epilogue) on the hand-written LDS-DMA MFMA kernel (csrc/kernels/gemm.hip);
  the plain forward / dgrad GEMMs there too, on the tile ops/gemm_tuning.json measured best per
  shape (no library GEMM in the step);
* attention is the fused flash-attention kernel (scores stay in LDS/registers);
* LayerNorm with fused residual add, erf GELU, counter-based dropout (hidden dropout
  0.1, and attention-probability dropout 0.1 applied inside the fused attention kernels
  from the same counter-based mask in forward and backward);
* the MLM head runs only on the masked positions (``mlm_positions``, Google BERT's
  ``masked_lm_positions``), saving ~85 % of the 30522-way decoder GEMM.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as tnn

from ..nn.modules import Linear, cross_entropy
from ..nn.transformer import GELU, Dropout, Embeddings, LayerNorm, RNGState, SelfAttention, gather_rows


class _Dense(tnn.Module):
    """Container so parameter names read ``<name>.dense.weight`` like HF."""

    def __init__(self, fin, fout, ln_eps=None):
        super().__init__()
        self.dense = Linear(fin, fout)
        if ln_eps is not None:
            self.LayerNorm = LayerNorm(fout, eps=ln_eps)


class BertLayer(tnn.Module):
    def __init__(self, hidden=768, heads=12, inter=3072, eps=1e-12, dropout=0.1, rng=None):
        super().__init__()
        self.attention = SelfAttention(hidden, heads, post_ln_eps=eps, attn_dropout=dropout, rng=rng)
        self.intermediate = _Dense(hidden, inter)
        self.output = _Dense(inter, hidden, ln_eps=eps)
        self.act = GELU()
        self.drop1 = Dropout(dropout, rng)
        self.drop2 = Dropout(dropout, rng)
        # each LayerNorm's residual input also feeds a Linear (h -> qkv, h1 -> FFN1): its
        # residual gradient is summed in that Linear's dgrad epilogue (nn/transformer.py)
        object.__setattr__(self.attention.ln, "_kml_res_linear", self.attention.qkv)
        object.__setattr__(self.output.LayerNorm, "_kml_res_linear", self.intermediate.dense)
        # ... and its input is the (dropped-out) output of the out-projection / FFN2 Linear
        # alone: that Linear's bias gradient is summed inside the LayerNorm backward
        object.__setattr__(self.attention.ln, "_kml_in_linear", self.attention.out)
        object.__setattr__(self.output.LayerNorm, "_kml_in_linear", self.output.dense)
        # FFN2 is the only consumer of FFN1's GELU output: FFN2's dgrad applies the GELU
        # backward (and sums FFN1's bias gradient) in its epilogue (nn/modules.py)
        object.__setattr__(self.output.dense, "_kml_gelu_producer", self.intermediate.dense)

    def forward(self, h, B: int, L: int, bias=None):
        # hidden dropout runs inside the LayerNorm kernels (LN(dropout(a) + h))
        h1 = self.attention.ln(self.attention(h, B, L, bias), residual=h, dropout=self.drop1)
        i = self.intermediate.dense(h1, act="gelu")   # erf-GELU in the GEMM epilogue
        return self.output.LayerNorm(self.output.dense(i), residual=h1, dropout=self.drop2)


class BertEncoder(tnn.Module):
    def __init__(self, n_layers, **kw):
        super().__init__()
        self.layer = tnn.ModuleList([BertLayer(**kw) for _ in range(n_layers)])


class BertModel(tnn.Module):
    def __init__(self, vocab=30522, hidden=768, layers=12, heads=12, inter=3072, max_pos=512, type_vocab=2,
                 eps=1e-12, dropout=0.1, rng=None):
        super().__init__()
        self.embeddings = Embeddings(vocab, hidden, max_pos, type_vocab, eps, dropout, rng)
        self.encoder = BertEncoder(layers, hidden=hidden, heads=heads, inter=inter, eps=eps, dropout=dropout, rng=rng)

    def forward(self, ids, token_type_ids=None, attention_mask=None):
        B, L = ids.shape
        bias = None
        if attention_mask is not None:
            bias = ((1.0 - attention_mask.float()) * -10000.0).reshape(B, L).contiguous()
        h = self.embeddings(ids, token_type_ids)
        for layer in self.encoder.layer:
            h = layer(h, B, L, bias)
        return h


class _Predictions(tnn.Module):
    def __init__(self, hidden, vocab, eps):
        super().__init__()
        self.transform = _Dense(hidden, hidden, ln_eps=eps)
        self.decoder = Linear(hidden, vocab)


class _Cls(tnn.Module):
    def __init__(self, hidden, vocab, eps):
        super().__init__()
        self.predictions = _Predictions(hidden, vocab, eps)


class BertForMaskedLM(tnn.Module):
    def __init__(self, vocab=30522, hidden=768, layers=12, heads=12, inter=3072, max_pos=512, type_vocab=2,
                 eps=1e-12, dropout=0.1, seed: int = 0):
        super().__init__()
        self.rng = RNGState(seed)
        self.vocab = vocab
        self.bert = BertModel(vocab, hidden, layers, heads, inter, max_pos, type_vocab, eps, dropout, self.rng)
        self.cls = _Cls(hidden, vocab, eps)
        self.act = GELU()
        # weight tying (HF tie_word_embeddings): decoder.weight IS the word table
        self.cls.predictions.decoder.weight = self.bert.embeddings.word_embeddings.weight
        self._init_weights()
        self._register_state_dict_hook(BertForMaskedLM._sd_hook)
        self._register_load_state_dict_pre_hook(BertForMaskedLM._load_hook, with_module=True)

    def _init_weights(self):
        for m in self.modules():
            if isinstance(m, (Linear, tnn.Embedding)):
                if m is self.cls.predictions.decoder:
                    continue
                tnn.init.normal_(m.weight, 0.0, 0.02)
                if isinstance(m, Linear) and m.bias is not None:
                    tnn.init.zeros_(m.bias)
            elif isinstance(m, LayerNorm):
                tnn.init.ones_(m.weight)
                tnn.init.zeros_(m.bias)
        tnn.init.zeros_(self.cls.predictions.decoder.bias)

    @staticmethod
    def _sd_hook(mod, sd, prefix, local_metadata):
        # HF stores the decoder bias twice (cls.predictions.bias is the canonical one)
        b = sd.get(prefix + "cls.predictions.decoder.bias")
        if b is not None:
            sd[prefix + "cls.predictions.bias"] = b
        return sd

    @staticmethod
    def _load_hook(mod, sd, prefix, local_metadata, strict, missing, unexpected, errors):
        b = sd.pop(prefix + "cls.predictions.bias", None)
        if b is not None and prefix + "cls.predictions.decoder.bias" not in sd:
            sd[prefix + "cls.predictions.decoder.bias"] = b
        if prefix + "cls.predictions.decoder.weight" not in sd and \
                prefix + "bert.embeddings.word_embeddings.weight" in sd:
            sd[prefix + "cls.predictions.decoder.weight"] = sd[prefix + "bert.embeddings.word_embeddings.weight"]

    def forward(self, ids, token_type_ids=None, attention_mask=None, mlm_positions=None, labels=None,
                return_correct=False):
        """ids [B, L]; mlm_positions [B, P] (positions to predict) or None (all);
        labels [B, P] (or [B, L]) with -100 = ignore.  Returns logits, or the mean MLM
        loss (and the correct count) when labels are given."""
        B, L = ids.shape
        if self.training and ids.is_cuda:
            self.rng.advance(ids.device)
        h = self.bert(ids, token_type_ids, attention_mask)
        if mlm_positions is not None:
            if ids.is_cuda:
                from ..ops import kernels as K
                idx = K.row_index(mlm_positions, L)      # one kernel (no arange / mul / add)
            else:
                idx = (mlm_positions + (torch.arange(B, device=ids.device) * L).view(B, 1)).reshape(-1)
            h = gather_rows(h, idx)
        t = self.cls.predictions.transform
        z = t.LayerNorm(t.dense(h, act="gelu"))
        if labels is None:
            return self.cls.predictions.decoder(z)
        # vocab-padded logits used in place (no slice copy / gradient re-pad of [T, 30528])
        logits = self.cls.predictions.decoder(z, keep_pad=True)
        return cross_entropy(logits, labels.reshape(-1), ignore_index=-100, return_correct=return_correct,
                             classes=self.vocab)


    def stages(self, ids, token_type_ids=None, attention_mask=None, mlm_positions=None, labels=None, n: int = 3):
        """Forward split into ``n`` stages for backward-overlapped gradient all-reduce
        (engine/staged.py): stage 0 = embeddings + the first encoder layers, the last stage
        ends with the MLM head and returns the loss.  Each stage's parameters are one
        contiguous range of the flat gradient buffer (reverse registration order; the tied
        word embedding belongs to stage 0, whose backward finishes its gradient last).
        Returns (stage callables h -> h, per-stage parameter lists)."""
        B, L = ids.shape
        layers = list(self.bert.encoder.layer)
        per = -(-len(layers) // n)
        groups = [layers[i * per:(i + 1) * per] for i in range(n)]
        bias = None
        if attention_mask is not None:
            bias = ((1.0 - attention_mask.float()) * -10000.0).reshape(B, L).contiguous()

        def first(_x):
            if self.training and ids.is_cuda:
                self.rng.advance(ids.device)
            h = self.bert.embeddings(ids, token_type_ids)
            for lay in groups[0]:
                h = lay(h, B, L, bias)
            return h

        def mid(g):
            def f(h):
                for lay in g:
                    h = lay(h, B, L, bias)
                return h
            return f

        def last(h):
            for lay in groups[-1]:
                h = lay(h, B, L, bias)
            if mlm_positions is not None:
                from ..ops import kernels as K
                h = gather_rows(h, K.row_index(mlm_positions, L))
            t = self.cls.predictions.transform
            z = t.LayerNorm(t.dense(h, act="gelu"))
            return cross_entropy(self.cls.predictions.decoder(z, keep_pad=True), labels.reshape(-1),
                                 ignore_index=-100, classes=self.vocab)
        fns = [first] + [mid(g) for g in groups[1:-1]] + [last]
        params = [list(self.bert.embeddings.parameters()) + [p for l in groups[0] for p in l.parameters()]]
        params += [[p for l in g for p in l.parameters()] for g in groups[1:-1]]
        tied = {id(p) for p in params[0]}
        params.append([p for l in groups[-1] for p in l.parameters()] +
                      [p for p in self.cls.parameters() if id(p) not in tied])
        return fns, params


def bert_base_mlm(**kw) -> BertForMaskedLM:
    return BertForMaskedLM(**kw)


def bert_tiny_mlm(**kw) -> BertForMaskedLM:
    """2-layer, 128-hidden variant for tests."""
    cfg = dict(vocab=1000, hidden=128, layers=2, heads=2, inter=512, max_pos=128)
    cfg.update(kw)
    return BertForMaskedLM(**cfg)
