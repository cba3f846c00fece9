"""Deterministic starting weights for the large golden fixtures (test infrastructure, no reference import).

The production CNN nets (AC_CNN_Atari [32, 64, 64] + fc 512: 3.4 M parameters) are too large to commit twice per
fixture, so make_golden.py overwrites the reference policy's freshly initialised parameters with these values before
recording, and the GPU replay regenerates them the same way.  Uniform draws from numpy's PCG64 (`Generator.random`,
integer-based and platform independent) cast to float32: bit-identical on the build container and the GPU box.
Scale: weights U(-a, a) with a = sqrt(3 / fan_in) (variance 1 / fan_in), biases U(-0.05, 0.05)."""
import numpy as np


def uniform_state(named_shapes, seed):
    """{name: float32 array} for [(name, shape), ...] in the given order (a state_dict's order)."""
    rng = np.random.default_rng(seed)
    out = {}
    for name, shape in named_shapes:
        shape = tuple(int(s) for s in shape)
        u = rng.random(shape) * 2.0 - 1.0
        if len(shape) >= 2:
            fan_in = int(np.prod(shape[1:]))
            out[name] = (u * np.sqrt(3.0 / fan_in)).astype(np.float32)
        else:
            out[name] = (u * 0.05).astype(np.float32)
    return out


def checksum(arr):
    """(sum, sum of squares) in float64: pins a regenerated tensor to the one the fixture was recorded with."""
    a = np.asarray(arr, np.float64)
    return np.asarray([a.sum(), (a * a).sum()], np.float64)


BIG = 1 << 20   # tensors with more elements are recorded as every 16th row (+ per-row sums), not whole
