"""Tile / kernel-selection policy of the native GEMM and conv kernels (CPU: the policy is host code in
the extension). Pins the per-layer A/B decisions recorded in profiles/r5a, r5c, r5d, r5e, r5h at the
ResNet-50 shapes."""
import pytest

from distributed_learning_amd.ops import _ext

pytestmark = pytest.mark.skipif(not _ext.available(), reason="native extension not built")

T128, T128x64, T256 = 1, 2, 8


@pytest.mark.parametrize("M,N,K,want", [
    (100352, 256, 2304, T256),   # s14 3x3 fwd (bs512): compute-bound -> 256x256
    (25088, 512, 4608, T256),    # s7 3x3 fwd: 98 x 2 = 196 tiles >= 192
    (100352, 256, 1024, T256),   # s14 conv1 fwd, K = 1024
    (100352, 1024, 256, T128),   # s14 conv3 fwd: short K stays on 128x128
    (401408, 128, 1152, T128),   # s28 3x3: N = 128 (256-wide tiles measured slower)
    (1605632, 64, 576, T128x64),  # s56 3x3: narrow N
    (6272, 384, 1728, T128),     # GoogLeNet-size M: too few 256x256 tiles for the chip
    (100352, 320, 2880, T128),   # N not a multiple of 256
])
def test_pick_tile(M, N, K, want):
    C = _ext.require()
    assert C.pick_tile(M, N, K, True) == want


def test_pick_tile_wide_gate():
    C = _ext.require()
    # 3x3 kernels whose loaded channel count is not % 64 have no 8-wave path
    assert C.pick_tile(100352, 256, 2304, False) == T128


def test_conv_tile_512x128():
    C = _ext.require()
    # Cout = 128 3x3 passes with >= 1024 row tiles of 512 (ResNet-50 stage 2 at bs1280): the 512x128 8-wave tile
    assert C.pick_conv_tile(1003520, 128, 1152, True) == 9
    assert C.pick_conv_tile(401408, 128, 1152, True) == T128   # 784 tiles (bs512): stays on 128x128
    assert C.pick_conv_tile(1003520, 128, 1152, False) == T128  # no 8-wave path
    assert C.pick_conv_tile(1003520, 256, 2304, True) == T256
    assert C.pick_tile(1003520, 128, 1152, True) == T128  # the 1x1 GEMMs never get it


def test_gemm_tn_splits_targets():
    C = _ext.require()
    # 256x256 weight-gradient tiles (both dims % 256): ~256 blocks, >= 16 k-steps per split
    assert C.gemm_tn_splits(1024, 256, 100352) == 64
    assert C.gemm_tn_splits(2048, 512, 25088) == 16
    # 128-wide tiles elsewhere: ~512 blocks
    assert C.gemm_tn_splits(128, 512, 401408) == 128
    assert C.gemm_tn_splits(64, 64, 8192) == 8  # capped by K / (16 * 64)


def test_halo_default_policy():
    C = _ext.require()
    # default mode (DLA_HALO unset in the test process): forward and data gradient, 64 -> 64, stride 1,
    # W <= 63
    assert C.halo_conv_eligible(64, 64, 56, 1, False)
    assert C.halo_conv_eligible(64, 64, 56, 1, True)
    assert not C.halo_conv_eligible(128, 128, 28, 1, False)
    assert not C.halo_conv_eligible(64, 64, 56, 2, False)
    assert not C.halo_conv_eligible(64, 64, 64, 1, False)
