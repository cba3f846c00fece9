"""CPU checks of the round-5 CNN host plans (no GPU, no kernel launches):
  * C3's trunk (AC_CNN_Atari 4x84x84, [32, 64, 64], fc 512) takes the split fc path for the update's minibatches and
    not for the rollout's 1024 frames, with the last conv's activation backward fused (6400 = 25 x 256 columns);
  * a trunk whose flattened width is not a multiple of 256 keeps the split but not the fused epilogue, and its last
    data-gradient column block is aligned to the row's end (overlapping its neighbour, never padded);
  * the grouped split GEMM entries refuse host tensors (no CPU path);
  * the conv forms' defaults: K25B / K26B / K27B on, K28B off."""
import pytest
import torch

from xuanpolicy_amd import fused_cnn, ops
from xuanpolicy_amd.policies import AC_CNN_Atari


def _trunk(hw):
    rep = AC_CNN_Atari((hw, hw, 4), [8, 4, 3], [4, 2, 1], [32, 64, 64], None, torch.nn.init.orthogonal_,
                       torch.nn.ReLU, "cpu", [512])
    return fused_cnn._Trunk(rep, fused_cnn._Part())


def test_c3_trunk_plans_the_split_fc_and_the_fused_act():
    t = _trunk(84)
    assert t.tail == "flatten" and t.fc[0][0].in_features == 6400
    assert ops.S3_GEMMS and t._fc_split_ok(16384) and t._fc_fuse_ok(16384)
    assert not t._fc_split_ok(1024) and not t._fc_fuse_ok(1024)        # the rollout's forwards stay on hipBLASLt
    c0s = [min(c, 6400 - 256) for c in range(0, 6400, 256)]
    assert len(c0s) == 25 and c0s[-1] == 6144 and all(c % 64 == 0 for c in c0s)


def test_ragged_fc_width_keeps_split_without_fused_act():
    t = _trunk(76)   # 19 -> 9 -> 9: 9 x 9 x 64 = 5184 columns
    in_f = t.fc[0][0].in_features
    assert in_f == 5184 and in_f % 256 == 64
    assert t._fc_split_ok(16384) and not t._fc_fuse_ok(16384)
    c0s = [min(c, in_f - 256) for c in range(0, in_f, 256)]
    assert c0s[-1] == in_f - 256 and c0s[-2] + 256 > c0s[-1]   # the overlap, no padded block


def test_fc_split_switches():
    t = _trunk(84)
    old = fused_cnn._Trunk.fc_split, fused_cnn._Trunk.fc_fuse_act
    try:
        fused_cnn._Trunk.fc_fuse_act = False
        assert t._fc_split_ok(16384) and not t._fc_fuse_ok(16384)
        fused_cnn._Trunk.fc_split = False
        assert not t._fc_split_ok(16384) and not t._fc_fuse_ok(16384)
    finally:
        fused_cnn._Trunk.fc_split, fused_cnn._Trunk.fc_fuse_act = old


def test_grouped_split_gemm_refuses_host_tensors():
    a = torch.zeros(512, 64)
    b = torch.zeros(16, dtype=torch.uint8)
    c = torch.zeros(512, 256)
    with pytest.raises(ValueError):
        ops.s3_gemm_group([(a, b, c)], 64)
    with pytest.raises(ValueError):
        ops.s3_gemm_group_act([(a, b, c)], 64, [c], 1, 0.0, 64, torch.zeros(2, 64))


def test_conv_form_defaults():
    L = ops.lib()
    assert L.xpa_conv1_form(-1) == 7
    assert L.xpa_conv_igemm_form(-1) == 0
