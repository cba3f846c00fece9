"""Diagnostic: per-update drift of the production CNN replays (G8P / G9P) against the reference fixtures."""
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tests.test_gpu_atari as ta  # noqa: E402
import tests.test_gpu_perdqn as tp  # noqa: E402

GOLD = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")


def golden(name):
    return dict(np.load(os.path.join(GOLD, name), allow_pickle=False))


orig = np.testing.assert_allclose
log = []


def rec(actual, desired, rtol=1e-7, atol=0, err_msg="", **k):
    a, d = np.asarray(actual, np.float64), np.asarray(desired, np.float64)
    with np.errstate(invalid="ignore", divide="ignore"):
        rel = np.nanmax(np.abs(a - d) / np.maximum(np.abs(d), 1e-30)) if a.size else 0
    log.append((err_msg[:30], a.shape, float(np.nanmax(np.abs(a - d))) if a.size else 0, float(rel)))


np.testing.assert_allclose = rec
for name, fn, arg in (("G8P", ta.test_a2c_atari_replays_reference_agent, "atari_a2c_prod.npz"),
                      ("G9P", tp.test_perdqn_learner_replays_reference, "perdqn_prod.npz")):
    log.clear()
    fn(golden, arg)
    print(name)
    for e in log:
        print("   %-30s %-14s abs %.3e rel %.3e" % (e[0], str(e[1]), e[2], e[3]))
