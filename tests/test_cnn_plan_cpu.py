"""CPU checks of the explicit CNN path's construction-time plan (fused_cnn._Trunk): a small-channel conv that K28 / K29
cannot take must be refused at construction (ValueError -> the learner's generic autograd path), not mid-update."""
import pytest
import torch.nn as nn

from xuanpolicy_amd import _lib
from xuanpolicy_amd.policies import AC_CNN_Atari, Basic_CNN


def _lib_or_skip():
    try:
        _lib.load()
    except Exception as e:  # noqa: BLE001 - no built library in this checkout
        pytest.skip("libxuanpolicy_amd.so not built: %s" % e)


def test_rgb_first_conv_is_refused_at_construction():
    """configs/perdqn/box2d/CarRacing-v2.yaml: Basic_CNN filters [16, 16, 32] on 3-channel frames (3 -> 16)."""
    _lib_or_skip()
    from xuanpolicy_amd.fused_cnn import _Trunk
    rep = Basic_CNN((96, 96, 3), kernels=[8, 4, 3], strides=[4, 2, 1], filters=[16, 16, 32], activation=nn.ReLU)
    with pytest.raises(ValueError, match="no K28 / K29 form"):
        _Trunk(rep, parts=None)


def test_k28_capable_small_channel_nets_keep_the_explicit_path():
    """The 4 -> 8 -> 8 test nets and the production Nature CNN construct (K25 / K28 / K29 take every conv)."""
    _lib_or_skip()
    from xuanpolicy_amd.fused_cnn import _Trunk
    small = Basic_CNN((84, 84, 4), kernels=[8, 4], strides=[4, 2], filters=[8, 8], activation=nn.ReLU)
    _Trunk(small, parts=None)
    prod = AC_CNN_Atari((84, 84, 4), kernels=[8, 4, 3], strides=[4, 2, 1], filters=[32, 64, 64], activation=nn.ReLU,
                        fc_hidden_sizes=[512])
    t = _Trunk(prod, parts=None)
    assert t.u8_conv1
