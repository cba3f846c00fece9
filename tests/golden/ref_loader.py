"""Import the read-only reference (XuanCe 1.0.5 fork at /root/reference) in THIS container only.

Test infrastructure for golden-vector capture.  The reference needs gym,
gymnasium, mpi4py, wandb, cv2 and torch.utils.tensorboard, none of which are installed; this module
writes throw-away stub packages into a temp dir, puts it first on sys.path and imports `xuance`.
Never imported by the product path, never run on the GPU box (the reference does not travel).
"""
import os
import sys
import tempfile
import types

REF_ROOT = "/root/reference"

_SPACES = '''
import numpy as np
class Space:
    def __init__(self, shape=None, dtype=None, seed=None):
        self.shape = None if shape is None else tuple(shape)
        self.dtype = dtype
class Box(Space):
    def __init__(self, low=0.0, high=1.0, shape=None, dtype=np.float32, seed=None):
        if shape is None:
            shape = np.shape(low)
        super().__init__(shape, dtype)
        self.low = np.broadcast_to(np.asarray(low, np.float32), self.shape)
        self.high = np.broadcast_to(np.asarray(high, np.float32), self.shape)
class Discrete(Space):
    def __init__(self, n, seed=None, start=0):
        super().__init__((), np.int64)
        self.n = int(n)
class Dict(dict, Space):
    def __init__(self, spaces=None, **kw):
        dict.__init__(self, spaces or kw)
        self.spaces = dict(self)
        self.shape = None
class Tuple(tuple, Space):
    def __new__(cls, spaces):
        return tuple.__new__(cls, spaces)
    def __init__(self, spaces):
        self.spaces = tuple(spaces)
        self.shape = None
class MultiDiscrete(Space):
    def __init__(self, nvec, seed=None):
        super().__init__(np.shape(nvec), np.int64)
        self.nvec = np.asarray(nvec)
'''

_GYM_INIT = '''
from . import spaces
from .spaces import Space
class Wrapper:
    def __init__(self, env):
        self.env = env
class Env:
    pass
def make(*a, **k):
    raise RuntimeError("gym stub: real environments are unavailable offline")
'''


def _write_stubs(root):
    for pkg in ("gym", "gymnasium"):
        sp = os.path.join(root, pkg, "spaces")
        os.makedirs(sp, exist_ok=True)
        with open(os.path.join(root, pkg, "__init__.py"), "w") as f:
            f.write(_GYM_INIT)
        with open(os.path.join(sp, "__init__.py"), "w") as f:
            f.write(_SPACES)
        for sub, names in (("box", "Box"), ("discrete", "Discrete"), ("dict", "Dict"),
                           ("tuple", "Tuple"), ("multi_discrete", "MultiDiscrete"), ("space", "Space")):
            with open(os.path.join(sp, sub + ".py"), "w") as f:
                f.write("from . import %s\n" % names)
    os.makedirs(os.path.join(root, "mpi4py"), exist_ok=True)
    with open(os.path.join(root, "mpi4py", "__init__.py"), "w") as f:
        f.write('''
class _Comm:
    def Allreduce(self, a, b, op=None):
        b[...] = a
    def Get_rank(self):
        return 0
    def Get_size(self):
        return 1
class MPI:
    COMM_WORLD = _Comm()
    SUM = "sum"
''')
    with open(os.path.join(root, "wandb.py"), "w") as f:
        f.write("def init(*a, **k): pass\ndef log(*a, **k): pass\ndef finish(*a, **k): pass\n"
                "class Video:\n    def __init__(self, *a, **k): pass\n")
    with open(os.path.join(root, "cv2.py"), "w") as f:
        f.write("INTER_AREA = 3\ndef resize(*a, **k):\n    raise RuntimeError('cv2 stub')\n")


def import_reference():
    """Return the imported `xuance` reference package (stubs installed on first call)."""
    if "xuance" in sys.modules and getattr(sys.modules["xuance"], "__file__", "").startswith(REF_ROOT):
        return sys.modules["xuance"]
    if not os.path.isdir(REF_ROOT):
        raise RuntimeError("reference not present (golden capture runs only in the build container)")
    sys.dont_write_bytecode = True
    root = tempfile.mkdtemp(prefix="xref_stubs_")
    _write_stubs(root)
    sys.path.insert(0, root)
    tb = types.ModuleType("torch.utils.tensorboard")

    class SummaryWriter:
        def __init__(self, *a, **k): pass
        def add_scalar(self, *a, **k): pass
        def add_scalars(self, *a, **k): pass
        def add_video(self, *a, **k): pass
        def close(self): pass
    tb.SummaryWriter = SummaryWriter
    sys.modules["torch.utils.tensorboard"] = tb
    import numpy as np
    if not hasattr(np, "int"):
        np.int = int
    if not hasattr(np, "float"):
        np.float = float
    if not hasattr(np, "bool"):
        np.bool = bool
    sys.path.insert(1, REF_ROOT)
    import xuance  # noqa: F401
    return xuance
