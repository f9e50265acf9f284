"""Pinned streaming loader on the MI355X (sdk/loader.py + csrc/runtime/loader.cpp):
every planned minibatch arrives in HBM byte-exact against ``ShardStore.load_docs``,
in order, across rounds with ragged tails, while the compute stream keeps consuming
earlier batches (device ring reuse is ordered by events)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = torch.device("cuda", 0)


def _store(tmp_path, n=64 * 15 + 37):
    from kubeml_amd.store.shards import ShardStore
    rng = np.random.default_rng(3)
    st = ShardStore(str(tmp_path))
    x = rng.integers(0, 256, (n, 32, 32, 3), dtype=np.uint8)
    y = rng.integers(0, 10, n).astype(np.int64)
    st.create("ds", x, y, x[:300], y[:300])
    return st, x, y


def test_stream_matches_load_docs(tmp_path):
    from kubeml_amd.sdk.loader import SplitStreamer
    st, x, y = _store(tmp_path)
    s = SplitStreamer(st, "ds", "train", dev)
    rounds = [(0, 4), (4, 9), (9, 16)]           # last round has a ragged doc
    bs = 100
    s.plan(rounds, bs)
    acc = torch.zeros((), dtype=torch.float64, device=dev)
    seen = []
    for d0, d1 in rounds:
        ref_x, ref_y = st.load_docs("ds", "train", d0, d1)
        for b0 in range(0, len(ref_x), bs):
            xb, yb = s.next()
            # consume on the compute stream (keeps the ring busy while later copies run)
            acc += xb.double().sum()
            seen.append((xb.clone(), yb.clone(), ref_x[b0:b0 + bs], ref_y[b0:b0 + bs]))
    torch.cuda.synchronize()
    assert s.stream.pending() == 0
    total = 0
    for xb, yb, rx, ry in seen:
        assert xb.shape == rx.shape
        assert np.array_equal(xb.cpu().numpy(), rx)
        assert np.array_equal(yb.cpu().numpy(), ry)
        total += float(rx.astype(np.float64).sum())
    assert float(acc) == total
    # re-plan (new task) with a different batch size while nothing is pending
    s.plan([(2, 3)], 64)
    xb, yb = s.next()
    assert np.array_equal(xb.cpu().numpy(), x[128:192])
