"""Measured-table routing (no GPU needed): which GEMM runs a linear / 1x1-conv product.

ops/gemm_tuning.json picks a hand-written MFMA tile per shape (no library route is left);
ops/wgrad_gemm.json sends a 1x1 / stride-1 conv weight gradient to gemm.hip's slab split-K.
Everything not in a table stays on the hand-written kernels' default plans."""
import json
import os

from kubeml_amd.ops import gemm as G
from kubeml_amd.ops import kernels as K

OPS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "kubeml_amd", "ops")


def test_every_gemm_route_is_a_hand_written_tile():
    d = json.load(open(os.path.join(OPS, "gemm_tuning.json")))
    assert d["entries"]
    for e in d["entries"]:
        key = (e["layout"], e["M"], e["N"], e["K"])
        tile, splits = G.plan(*key)
        base = tuple(t for t in tile if t != "slab")
        assert base in G.TILES, (key, tile)    # a gemm.hip tile, never a library route
        assert splits >= 1
    for e in json.load(open(os.path.join(OPS, "wgrad_gemm.json")))["entries"]:
        assert e["route"][0] in ("slab", "gather")
    assert G.plan(0, 4096, 3072, 768)[0] in G.TILES    # shapes outside the table: default tile
    import inspect
    assert "torch.mm" not in inspect.getsource(G) and "addmm" not in inspect.getsource(G)


def test_wgrad_gemm_route_only_for_plain_1x1():
    d = json.load(open(os.path.join(OPS, "wgrad_gemm.json")))
    assert d["entries"]
    e = d["entries"][0]
    B = 128
    hw = int(round((e["P"] // B) ** 0.5))
    shape = (B, hw, hw, e["C"])
    assert K.wgrad_gemm_route(shape, e["K"], 1, 1, (1, 1), (0, 0)) == tuple(e["route"])
    assert K.wgrad_gemm_route(shape, e["K"], 3, 3, (1, 1), (1, 1)) is None       # not a GEMM
    assert K.wgrad_gemm_route(shape, e["K"], 1, 1, (2, 2), (0, 0)) is None       # strided
    assert K.wgrad_gemm_route(shape, e["K"], 1, 1, (1, 1), (0, 0), dbias=object()) is None
    assert K.wgrad_gemm_route((B, hw, hw, e["C"] + 8), e["K"], 1, 1, (1, 1), (0, 0)) is None
    for r in d["entries"]:
        if r.get("KH", 1) == 1:
            assert r["route"][0] == "slab"
        else:   # implicit-GEMM weight gradients on the GEMM tiles: only their exact geometry
            assert r["route"][0] == "gather"
            kh, st = r["KH"], r["S"]
            hw2 = int(round((r["P"] // B) ** 0.5))
            xs = (B, hw2, hw2, r["C"])
            p = (kh - 1) // 2
            assert K.wgrad_gemm_route(xs, r["K"], kh, kh, (st, st), (p, p)) == tuple(r["route"])
            assert K.wgrad_gemm_route(xs, r["K"], kh, kh, (st, st), (0, 0)) is None          # other padding
            assert K.wgrad_gemm_route(xs, r["K"], kh, kh, (3 - st, 3 - st), (p, p)) is None  # other stride
            assert K.wgrad_gemm_route(xs, r["K"], 1, 1, (1, 1), (0, 0)) is None              # other kernel


def test_conv_gemm_route_plans_only_for_eligible_geometry():
    """conv_tuning.json entries with variant GEMM1X1 (the conv GEMM routes) are planned only for
    geometries the route runs: a plain GEMM for 1x1 / stride 1, an implicit GEMM (C % 64) otherwise;
    any other conv with the same GEMM dimensions falls back to an implicit-GEMM tile."""
    d = json.load(open(os.path.join(OPS, "conv_tuning.json")))
    routed = [e for e in d["entries"] if e["mode"] == "fwd" and len(e["cfg"]) == 5 and e["cfg"][4] == K.GEMM1X1]
    assert routed
    for e in routed:
        M, N, Kd = e["M"], e["N"], e["Kd"]
        if Kd % 64 == 0 and Kd // 9 % 64 == 0 and Kd % 9 == 0:     # a 3x3 conv over C = Kd / 9
            C, geom = Kd // 9, (14, 14, 3, 3, (1, 1), (1, 1))
        else:
            C, geom = Kd, (7, 7, 1, 1, (1, 1), (0, 0))
        assert K.conv_fwd_plan(C, M, N, Kd, geom=geom)[4] == K.GEMM1X1
        # C not a multiple of 64 and not a 1x1 conv: never the GEMM route
        assert K.conv_fwd_plan(C + 8, M, N, Kd, cfg=tuple(e["cfg"]),
                               geom=(14, 14, 3, 3, (1, 1), (1, 1)))[4] != K.GEMM1X1
