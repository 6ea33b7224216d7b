"""Host-side launch geometry of the GEMM / conv paths (kernels.py): which form a conv pass takes and how deep its
split-K runs.  Pure arithmetic, no GPU: these choices decide which kernel the GPU tests and the bench exercise,
so a change that silently moves a production shape to another path shows up here first."""

import pytest

from spine_vision_amd import kernels as K


def _shape(B, H, W, Cs, Cout, k, stride, pad):
    return K.conv_shape(B, H, W, Cs, Cout, k, stride, pad)


# ResNet-50 @256 bs32 strided convs: the three 3x3 conv2s and the four 1x1 shortcuts that stride
RESNET50_S2 = [(32, 64, 64, 128, 128, 3, 1), (32, 32, 32, 256, 256, 3, 1), (32, 16, 16, 512, 512, 3, 1),
               (32, 64, 64, 256, 512, 1, 0), (32, 32, 32, 512, 1024, 1, 0), (32, 16, 16, 1024, 2048, 1, 0)]


@pytest.mark.parametrize("case", RESNET50_S2, ids=lambda c: "x".join(map(str, c)))
def test_resnet50_strided_dgrads_go_straight_into_dx(case):
    """every strided data gradient of ResNet-50 @256 takes the one-launch parity-class GEMM with no split-K
    (csrc/gemm3.hip mode 5 with remapped epilogue rows): no f32 slabs, no scatter pass"""
    B, H, W, Cs, Cout, k, pad = case
    s = _shape(B, H, W, Cs, Cout, k, 2, pad)
    assert K._s2_direct(s)
    assert K._s2_split(s, B * H * W, k * k) == 1


def test_odd_grids_keep_the_slab_form(monkeypatch):
    s = _shape(2, 15, 13, 64, 64, 3, 2, 1)  # classes of different sizes: no shared grid
    assert not K._s2_direct(s)
    monkeypatch.setattr(K, "_S2_DIRECT", False)
    assert not K._s2_direct(_shape(2, 16, 16, 64, 64, 3, 2, 1))


def test_s2_split_restorable(monkeypatch):
    """SV_S2_NOSPLIT=0 restores _conv_split's choice on the direct path (A/B runs)"""
    s = _shape(32, 16, 16, 512, 512, 3, 2, 1)
    monkeypatch.setattr(K, "_S2_NOSPLIT", False)
    assert K._s2_split(s, 32 * 16 * 16, 9) == K._conv_split(32 * 16 * 16 // 4, 512, max(32, 9 * 512 // 4))


@pytest.mark.parametrize("M,N,Kd", [(131072, 64, 576), (8192, 512, 4608), (2048, 2048, 1024), (524288, 128, 128)])
def test_conv_split_bounds(M, N, Kd):
    """split-K depth: 1 for grids of >= 192 tiles or short K, else <= 16 slices of >= 16 k-steps each within
    32 MiB of f32 slabs"""
    s = K._conv_split(M, N, Kd)
    tiles = -(-M // 256) * -(-N // 128)
    assert 1 <= s <= 16
    if tiles >= 192 or Kd // 32 < 32:
        assert s == 1
    else:
        assert (Kd // 32) // s >= 16 and s * M * N * 4 <= 32 << 20


# ConvNeXt-base bs32 @512 weight gradients: (N, K, M) of fc1 / fc2 at every stage
CONVNEXT_WGRADS = [(512, 128, 524288), (128, 512, 524288), (1024, 256, 131072), (256, 1024, 131072),
                   (2048, 512, 32768), (512, 2048, 32768), (4096, 1024, 8192), (1024, 4096, 8192)]


@pytest.mark.parametrize("N,Kd,M", CONVNEXT_WGRADS)
def test_wgrad_split_fills_half_the_chip(N, Kd, M):
    """the persistent 256x256 wgrads: slices cut M into whole 64-row K-tiles, one workgroup per CU at most,
    and the grid lands near the 128-workgroup target (the side stream's half of the chip)"""
    s = K._wgrad_split_for(N, Kd, M)
    tiles9 = -(-N // 256) * -(-Kd // 256)
    assert M % (s * 64) == 0
    assert tiles9 * s <= 256
    assert abs(tiles9 * s - K._WGRAD9_TARGET) <= max(tiles9, K._WGRAD9_TARGET // 2)


@pytest.mark.parametrize("N,Kd,M", CONVNEXT_WGRADS)
def test_wgrad_split_whole_chip_target(N, Kd, M):
    """the ConvNeXt backward's target (256: the whole chip, with bf16 slabs): whole 64-row K-tiles per slice, at most
    one workgroup per CU, never fewer workgroups than the 128 target gives"""
    s = K._wgrad_split_for(N, Kd, M, 256)
    tiles9 = -(-N // 256) * -(-Kd // 256)
    assert M % (s * 64) == 0 and tiles9 * s <= 256
    assert tiles9 * s >= tiles9 * K._wgrad_split_for(N, Kd, M)
