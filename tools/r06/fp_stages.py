"""five_point_wave stage latencies (wall_clock64 stamps, 100 MHz) on random 5-point problems, one wave each,
problems launched alone (count=1, repeated) and as a full grid.  Prints per-stage medians in microseconds."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "visual-slam-pipeline_amd", "python"))
import vslam_abi  # noqa: E402

lib = vslam_abi.load_library()
f = lib.vs_debug_five_point_ck
f.restype = ctypes.c_int
f.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_int] + [ctypes.c_void_p] * 3
rng = np.random.default_rng(5)
names = ["basis", "columns", "gauss-jordan", "(stage 3 tail)", "roots", "models"]
for count in (1, 1, 64, 2048):
    q1 = rng.uniform(-0.6, 0.6, (count, 10))
    q2 = rng.uniform(-0.6, 0.6, (count, 10))
    E = np.zeros((count, 10, 9))
    nm = np.zeros(count, np.int32)
    ck = np.zeros((count, 8), np.int64)
    assert f(q1.ctypes.data, q2.ctypes.data, count, E.ctypes.data, nm.ctypes.data, ck.ctypes.data) == 0
    d = np.diff(ck[:, :7], axis=1) / 100.0  # us at 100 MHz
    print("count", count, "total med %.1f us max %.1f" % (np.median(d.sum(1)), d.sum(1).max()),
          " ".join("%s %.1f" % (n, v) for n, v in zip(names, np.median(d, 0))), flush=True)
