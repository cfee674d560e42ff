"""Debug: the n == 5 solve_pnp case vs the EPnP debug hook and the host (round 5)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in ("tests", "oracle", "visual-slam-pipeline_amd/python"):
    sys.path.insert(0, os.path.join(ROOT, p))
import oracle_py as oracle  # noqa: E402
import vslam_abi  # noqa: E402
from test_oracle_pnp import pnp_problem  # noqa: E402

lib = vslam_abi.load_library()
lib.vs_debug_epnp.restype = ctypes.c_int
lib.vs_debug_epnp.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] + [ctypes.c_void_p] * 2
obj, img, _, _, _ = pnp_problem(5, 3)
X = obj.astype(np.float64).reshape(1, 15).copy()
uv = img.astype(np.float64).reshape(1, 10).copy()
m = np.array([5], np.int32)
K = np.array([525.0, 525.0, 319.5, 239.5])
dev = np.zeros((1, 137))
lib.vs_debug_epnp(X.ctypes.data, uv.ctypes.data, m.ctypes.data, 1, K.ctypes.data, dev.ctypes.data)
host = oracle.epnp_debug(X, uv, m, tuple(K))
print('noinline small_eig v diff', np.abs(dev[0, 80:128] - host[0, :48]).max(), 'noinline epnp R diff', np.abs(dev[0, 128:137] - host[0, 48:57]).max())
dev = dev[:, :80]
print("debug hook v diff", np.abs(dev[0, :48] - host[0, :48]).max(), "R diff", np.abs(dev[0, 48:57] - host[0, 48:57]).max())
ctx = vslam_abi.Context(0)
g = ctx.solve_pnp(obj, img, 100, 5)
so = oracle.solve_pnp(obj, img, 100, 5)
print("rv dev", dev[0, 61:64], "host", host[0, 61:64], "R2 diff", np.abs(dev[0, 64:73] - host[0, 64:73]).max())
print("epnp_subset rv", dev[0, 73:76], "tv", dev[0, 76:79], "ok", dev[0, 79], "inline t", dev[0, 57:60])
print("solve_pnp Rw diff", np.abs(g[1] - so[1]).max())
print("host R^T", host[0, 48:57].reshape(3, 3).T.ravel())
print("dev  R^T", dev[0, 48:57].reshape(3, 3).T.ravel())
print("solve Rw", g[1].ravel())
print("orc   Rw", so[1].ravel())
ctx.close()
