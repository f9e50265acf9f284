"""Host side of the paired launches (ops/kernels.py conv_fwd_pair / bn_apply_pair / bn_bwd_pair),
on the CPU with a recording stand-in for the HIP library: calls made inside a pair block launch
nothing until the block ends; then the pair entry point gets both argument lists packed as 64-bit
values (floats as their bit patterns), or — when it reports the plans unpairable — each call
launches on its own, in order; a record keeps its operands alive until the launch (the bug the
multi-rank trajectory test caught: a dropped workspace went back to the allocator first)."""
import ctypes
import gc
import struct
import weakref

import pytest
import torch

from kubeml_amd.ops import kernels as K

SIZES = {"kml_conv_fwd_pair": 30, "kml_bn_apply_pair": 18, "kml_bn_bwd_pair": 17}


class FakeHIP:
    def __init__(self, pair_rc=0):
        self.calls, self.packed, self.pair_rc = [], [], pair_rc

    def call(self, name, sig, *args):
        self.calls.append((name, args))
        if name in SIZES:
            n = SIZES[name]
            self.packed = [list((ctypes.c_longlong * n).from_address(a)) for a in args[:2]]
        return 0

    def raw(self, name, *args):
        return 64

    def fn(self, name, sig=None):
        def f(*args):
            if name == "kml_bn_fold_rows":
                return 0
            self.calls.append((name, args))
            if name in SIZES:
                n = SIZES[name]
                self.packed = [list((ctypes.c_longlong * n).from_address(a)) for a in args[:2]]
                return self.pair_rc
            return 0
        return f


@pytest.fixture
def hip(monkeypatch):
    def make(rc=0):
        h = FakeHIP(rc)
        monkeypatch.setattr(K, "HIP", h)
        monkeypatch.setattr(K, "_s", lambda: 0)
        monkeypatch.setattr(K, "_chk", lambda *a, **k: None)   # CPU stand-in tensors
        return h
    return make


def _args(base):
    return tuple(base + i for i in range(30))


def test_conv_pair_launches_once_with_both_argument_lists(hip):
    h = hip(0)
    n0 = K.FWD_PAIRS_LAUNCHED[0]
    with K.conv_fwd_pair():
        K._conv_fwd_launch("sig", _args(100))
        K._conv_fwd_launch("sig", _args(1000))
        assert h.calls == []
    assert [c[0] for c in h.calls] == ["kml_conv_fwd_pair"]
    assert h.packed == [list(_args(100)), list(_args(1000))]
    assert K.FWD_PAIRS_LAUNCHED[0] == n0 + 1


def test_conv_pair_unpairable_plans_launch_separately_in_order(hip):
    h = hip(1)
    with K.conv_fwd_pair():
        K._conv_fwd_launch("sig", _args(100))
        K._conv_fwd_launch("sig", _args(1000))
    assert [c[0] for c in h.calls] == ["kml_conv_fwd_pair", "kml_conv_fwd", "kml_conv_fwd"]
    assert h.calls[1][1][:30] == _args(100) and h.calls[2][1][:30] == _args(1000)


def test_conv_pair_single_call_and_third_call(hip):
    h = hip(0)
    with K.conv_fwd_pair():
        K._conv_fwd_launch("sig", _args(100))
    assert [c[0] for c in h.calls] == ["kml_conv_fwd"]
    h.calls.clear()
    with K.conv_fwd_pair():
        K._conv_fwd_launch("sig", _args(1))
        K._conv_fwd_launch("sig", _args(2))
        K._conv_fwd_launch("sig", _args(3))        # a third call is not recorded: launches at once
        assert [c[0] for c in h.calls] == ["kml_conv_fwd"]
    assert [c[0] for c in h.calls] == ["kml_conv_fwd", "kml_conv_fwd_pair"]


def test_record_keeps_operands_alive_until_the_launch(hip):
    hip(1)
    t = torch.empty(16)
    ref = weakref.ref(t)
    with K.conv_fwd_pair():
        K._conv_fwd_launch("sig", _args(100), keep=(t,))
        del t
        gc.collect()
        assert ref() is not None
        K._conv_fwd_launch("sig", _args(1000))
    gc.collect()
    assert ref() is None


def _bn_operands(M=64, C=32):
    x = torch.zeros(M, C, dtype=torch.bfloat16)
    st = torch.zeros(4 * 2 * C)
    g, b = torch.ones(C), torch.zeros(C)
    return x, st, g, b


def test_bn_apply_pair_packs_floats_as_bits(hip):
    h = hip(0)
    n0 = K.BN_PAIRS_LAUNCHED[0]
    x1, s1, g1, b1 = _bn_operands()
    x2, s2, g2, b2 = _bn_operands(C=64)
    with K.bn_apply_pair():
        y1 = K.bn_apply(x1, s1, g1, b1, eps=1e-5, momentum=0.1, relu=True, stats_rows=4)
        y2 = K.bn_apply(x2, s2, g2, b2, eps=2e-5, momentum=0.25, stats_rows=4)
        assert h.calls == []
    assert [c[0] for c in h.calls] == ["kml_bn_apply_pair"]
    bits = lambda f: struct.unpack("<I", struct.pack("<f", f))[0]
    q1, q2 = h.packed
    assert q1[0] == x1.data_ptr() and q1[6] == y1.data_ptr() and q1[11] == 64 and q1[12] == 32
    assert q1[13] == bits(1e-5) and q1[14] == bits(0.1) and q1[15] == 1 and q1[16] == 0
    assert q2[12] == 64 and q2[13] == bits(2e-5) and q2[14] == bits(0.25) and q2[15] == 0
    assert K.BN_PAIRS_LAUNCHED[0] == n0 + 1


def test_bn_apply_pair_fallback(hip):
    h = hip(1)
    ops = [_bn_operands(), _bn_operands()]
    with K.bn_apply_pair():
        for x, s, g, b in ops:
            K.bn_apply(x, s, g, b, stats_rows=4)
    assert [c[0] for c in h.calls] == ["kml_bn_apply_pair", "kml_bn_apply", "kml_bn_apply"]
    assert h.calls[1][1][0] == ops[0][0].data_ptr() and h.calls[2][1][0] == ops[1][0].data_ptr()


class _Rider:
    def arm(self):
        pass


def test_bn_bwd_pair_kinds_and_riders(hip):
    h = hip(0)
    n0 = K.BNB_PAIRS[0]
    C = 32
    dy, x = torch.zeros(64, C, dtype=torch.bfloat16), torch.zeros(64, C, dtype=torch.bfloat16)
    mean, rstd, g = torch.zeros(C), torch.ones(C), torch.ones(C)
    dg, db = torch.zeros(C), torch.zeros(C)
    part = torch.zeros(4, 2 * C)
    with K.bn_bwd_pair():
        K.bn_bwd(dy, None, x, mean, rstd, g, dg, db)                      # full: reduction + apply
        K.bn_bwd(dy, None, x, mean, rstd, g, dg, db, partial=(part, 4))   # partial rows given
        assert h.calls == []
    assert [c[0] for c in h.calls] == ["kml_bn_bwd_pair"]
    assert h.packed[0][0] == 0 and h.packed[1][0] == 1
    assert h.packed[1][7] == part.data_ptr() and h.packed[1][8] == 4
    assert K.BNB_PAIRS[0] == n0 + 1
    # a call carrying a rider launches at once (the rider is armed around that call only)
    h.calls.clear()
    with K.bn_bwd_pair():
        K.bn_bwd(dy, None, x, mean, rstd, g, dg, db, rider=None)
        K.bn_bwd(dy, None, x, mean, rstd, g, dg, db, partial=(part, 4), rider=_Rider())
        assert [c[0] for c in h.calls] == ["kml_bn_bwd_apply_partial", "kml_rider_flush"]
    assert [c[0] for c in h.calls][-1] == "kml_bn_bwd"
