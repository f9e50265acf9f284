"""LDS layouts the round-6 bank-conflict fixes rely on, checked on the CPU with the CDNA4 banking
rules of tools/lds_banks.py (MI355X_MICROARCH.md §LDS) and the constants parsed from the HIP
sources, so a later edit of a stride cannot silently bring the conflicts back:

* bn.hip ``bn_tstride``: the per-channel coefficient stores (lane = channel, ds_write_b32, banks
  (a / 4) mod 32 per 32-lane half) conflict-free, the 8-channel reads contiguous;
* gemm.hip / conv_igemm.hip epilogue partial-sum rows (``RED_STR``): per-thread ds_write_b32
  stores conflict-free;
* conv_igemm.hip ``PADK``: the 16x16x32 fragment reads (ds_read_b128) of K-contiguous operand
  rows conflict-free for BK = 32 and 64."""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

from lds_banks import G128, cycles  # noqa: E402

HALVES = [list(range(0, 32)), list(range(32, 64))]


def _src(name):
    return open(os.path.join(ROOT, "csrc", "kernels", name)).read()


def _cycles32(addrs, groups=HALVES):
    """ds_write_b32 / ds_read_b32: banks (a / 4) mod 32 per 32-lane half."""
    worst = 0
    for g in groups:
        banks = {}
        for lane in g:
            if addrs[lane] is None:
                continue
            banks.setdefault((addrs[lane] // 4) % 32, set()).add(addrs[lane] // 4)
        worst = max(worst, max((len(v) for v in banks.values()), default=1))
    return worst


def _bn_tstride(ch8):
    # the C++ expression, evaluated with C's truncating %
    src = _src("bn.hip")
    m = re.search(r"constexpr int bn_tstride\(int ch8\) \{ return ch8 \+ \(\(\((\d+) - ch8\) % (\d+)\) \+ (\d+)\) % (\d+); \}",
                  src)
    assert m, "bn_tstride changed shape: update this test"
    a, b, c, d = (int(v) for v in m.groups())
    t = a - ch8
    r = abs(t) % b * (1 if t >= 0 else -1)
    return ch8 + ((r + c) % d)


def test_bn_coefficient_slots_conflict_free():
    for C in (64, 128, 256, 512, 1024, 2048):
        ch8 = C // 8
        s = _bn_tstride(ch8)
        assert s >= ch8
        for base in range(0, C, 64):      # the per-channel store loop: lane = channel c
            addrs = [((c & 7) * s + (c >> 3)) * 4 if c < C else None for c in range(base, base + 64)]
            assert _cycles32(addrs) == 1, (C, s, base)
        # the streaming loop's reads: lane j8 = i0 % (C / 8), slot k * s + j8
        for k in range(8):
            addrs = [(k * s + (lane % ch8)) * 4 for lane in range(64)]
            assert _cycles32(addrs) == 1, (C, k)


def test_epilogue_partial_rows_conflict_free():
    g = _src("gemm.hip")
    m = re.search(r"constexpr int RED_STR = (\d+), RED_STR8 = (\d+);", g)
    assert m
    for stride in (int(m.group(1)), int(m.group(2))):
        for k in range(8):
            assert _cycles32([(tid * stride + k) * 4 for tid in range(64)]) == 1, (stride, k)
    c = _src("conv_igemm.hip")
    assert "sF[(wave * CPR + lane) * 17 + k]" in c
    for k in range(16):
        assert _cycles32([((0 * 16 + lane) * 17 + k) * 4 if lane < 16 else None for lane in range(64)]) == 1


def test_implicit_gemm_operand_rows_conflict_free():
    m = re.search(r"constexpr int PADK = (\d+);", _src("conv_igemm.hip"))
    assert m
    pad = int(m.group(1))
    for bk in (32, 64):
        row = (bk + pad) * 2                      # bytes per K-contiguous row
        assert row % 16 == 0                      # 16-byte operand stores stay aligned
        for ks in range(bk // 32):
            addrs = [(lane & 15) * row + 64 * ks + 16 * (lane >> 4) for lane in range(64)]
            assert cycles(addrs, 16, G128) == 1, (bk, pad, ks)


def test_halo_4x4_patch_reads_conflict_free():
    """conv_igemm.hip HaloBody::swz on 4x4 maps at pitch 8 (ResNet-34 layer2's 3x3 convs, C = 128,
    4 images per block): every A-fragment read of the main loop (ds_read_b128 lane groups, all taps,
    K-steps and wave rows) hits 16 distinct 16-byte chunks."""
    src = _src("conv_igemm.hip")
    m = re.search(r"if constexpr \(HW == 4 && PITCH == 8\) return \(2 \* \(pix & 7\) \+ \(pix & 8\)\) & SWZ;", src)
    assert m, "the 4x4 halo swizzle changed shape: update this test"
    HW, C, IMG = 4, 128, 4
    HP, CH, PITCH = HW + 2, C // 8, 8
    IMGPIX, WM = HP * PITCH, IMG * HW * HW // 2
    h = lambda p: (2 * (p & 7) + (p & 8)) & 15
    for wm in range(2):
        for i in range(WM // 16):
            for ks in range(9 * C // 32):
                tap = ks // (C // 32)
                toff = (tap // 3) * PITCH + tap % 3
                addrs = []
                for lane in range(64):
                    r = wm * WM + i * 16 + (lane & 15)
                    im, p = divmod(r, HW * HW)
                    pix = im * IMGPIX + (p // HW) * PITCH + (p % HW) + toff
                    chunk = (ks % (C // 32)) * 4 + (lane >> 4)
                    addrs.append((pix * CH + (chunk ^ h(pix))) * 16)
                assert cycles(addrs, 16, G128) == 1, (wm, i, ks)
