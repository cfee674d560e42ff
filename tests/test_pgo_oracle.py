"""F4 pose graph optimisation (Optimizer::pose_graph_optimize, reference src/Optimizer.cpp:654-863)
— CPU checks: the oracle's dense restatement (oracle/orc_pgo.cpp) equals the independent numpy
restatement (tests/pgo_ref.py) to 1e-8 on chains with loop constraints and a height prior; the
first keyframe stays fixed and the loops pull the drifted chain toward its ground truth.  g2o is
not available offline: agreement with g2o itself is "parity unpinned"."""
import numpy as np
import pytest

import pgo_ref


@pytest.mark.parametrize("N,seed,every,prior", [(12, 1, 4, False), (25, 2, 8, True), (40, 3, 13, False)])
def test_oracle_equals_numpy(oracle, N, seed, every, prior):
    R, t, loops, gt = pgo_ref.chain_problem(N, seed, every)
    g = np.array([0.0, 1.0, 0.0]) if prior else None
    h = 0.4
    Ro, to, st, ch = oracle.pose_graph(R, t, loops, g, h)
    Rn, tn, chi = pgo_ref.optimize(R, t, loops, g, h)
    assert st[0] >= 1 and st[1] >= 1
    assert np.abs(Ro - Rn).max() < 1e-8 and np.abs(to - tn).max() < 1e-8
    assert abs(ch[1] - chi) <= 1e-6 * max(1.0, chi)
    assert np.array_equal(Ro[0], R[0]) and np.array_equal(to[0], t[0])  # the anchor
    err0 = np.linalg.norm(t - np.array([T[:3, 3] for T in gt]), axis=1).mean()
    err1 = np.linalg.norm(to - np.array([T[:3, 3] for T in gt]), axis=1).mean()
    assert err1 < err0
    assert ch[1] < ch[0]


def test_nothing_to_do(oracle):
    R, t, _, _ = pgo_ref.chain_problem(10, 4, 0)
    Ro, to, st, _ = oracle.pose_graph(R, t, [], None)
    assert st[0] == 0 and np.array_equal(Ro, R) and np.array_equal(to, t)
    R2, t2 = R[:2], t[:2]
    Ro, to, st, _ = oracle.pose_graph(R2, t2, [(0, 1, np.eye(3), np.zeros(3), 0.03, 0.01)], None)
    assert st[0] == 0 and np.array_equal(Ro, R2)
