"""F4 dense voxel fusion (reference main.cpp:1081-1139) — CPU checks of the oracle restatement
(oracle/orc_dense.cpp) against a pure-Python statement of the same loop: points in the order of
their first voxel insertion, rejected depths (<= 0, >= DENSE_MAX_DEPTH), repeated frames adding
nothing, negative coordinates flooring away from zero."""
import math

import numpy as np


def _py_dense(frames, step=8, max_depth=5.0, voxel=0.02, K=(525.0, 525.0, 319.5, 239.5)):
    fx, fy, cx, cy = K
    inv = 1.0 / voxel
    seen, cloud = set(), []
    for depth, R, t in frames:
        rows, cols = depth.shape
        for v in range(0, rows, step):
            for u in range(0, cols, step):
                z = float(depth[v, u])
                if z <= 0 or z >= max_depth:
                    continue
                x = (u - cx) * z / fx
                y = (v - cy) * z / fy
                p = [R[i][0] * x + R[i][1] * y + R[i][2] * z + t[i] - 0.0 for i in range(3)]
                key = tuple(math.floor(c * inv) for c in p)
                if key not in seen:
                    seen.add(key)
                    cloud.append(p)
    return np.array(cloud, np.float64).reshape(-1, 3)


def _frames(n, h, w, seed):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        d = rng.uniform(0.3, 6.0, (h, w)).astype(np.float32)
        d[rng.random((h, w)) < 0.1] = 0.0
        d[rng.random((h, w)) < 0.02] = -1.0
        a = rng.normal(0, 0.3, 3)
        th = np.linalg.norm(a)
        k = a / th
        Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
        R = np.eye(3) + math.sin(th) * Kx + (1 - math.cos(th)) * Kx @ Kx
        t = rng.normal(0, 0.5, 3)
        out.append((d, R, t))
    return out


def test_oracle_equals_python_loop(oracle):
    frames = _frames(4, 48, 64, 1)
    frames.append(frames[1])  # a repeated frame adds nothing
    D = oracle.Dense()
    for d, R, t in frames:
        D.integrate(d, R, t)
    got = D.points()
    ref = _py_dense(frames)
    assert got.shape == ref.shape and got.shape[0] > 0
    assert np.array_equal(got.view(np.uint64), ref.view(np.uint64))
    D.close()


def test_coarse_voxels_keep_the_first_point(oracle):
    # a flat wall 1 m away seen twice with a 1 cm shift: with 0.5 m voxels the second frame's points
    # fall in voxels the first already holds, so only its new voxels (if any) add points
    d = np.full((480, 640), 1.0, np.float32)
    D = oracle.Dense(voxel_size=0.5)
    D.integrate(d, np.eye(3), np.zeros(3))
    n1 = D.points().shape[0]
    D.integrate(d, np.eye(3), np.array([0.01, 0.0, 0.0]))
    pts = D.points()
    ref = _py_dense([(d, np.eye(3), np.zeros(3)), (d, np.eye(3), np.array([0.01, 0.0, 0.0]))], voxel=0.5)
    assert np.array_equal(pts, ref) and n1 <= pts.shape[0] < 2 * n1
    D.close()
