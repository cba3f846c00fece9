"""pytest plugin for A/B runs of the GPU tests (tools only): XPA_AB_CONV_FORM=<xpa_conv1_form mask>,
XPA_AB_FC_SPLIT=0|1 set for every test.   PYTHONPATH=tools python -m pytest -p ab_plugin ..."""
import os

import pytest


@pytest.fixture(autouse=True)
def _xpa_ab(monkeypatch):
    form = os.environ.get("XPA_AB_CONV_FORM")
    prev = None
    if form is not None:
        from xuanpolicy_amd import ops
        prev = ops.lib().xpa_conv1_form(int(form))
    fc = os.environ.get("XPA_AB_FC_SPLIT")
    if fc is not None:
        from xuanpolicy_amd import fused_cnn
        monkeypatch.setattr(fused_cnn._Trunk, "fc_split", bool(int(fc)))
    yield
    if prev is not None:
        from xuanpolicy_amd import ops
        ops.lib().xpa_conv1_form(prev)
