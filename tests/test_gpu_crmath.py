"""The device's correctly rounded fp64 functions (csrc/cr_math.h, double-double) equal the
oracle's (libquadmath binary128 rounded to double) bit for bit — the property that makes the
Rodrigues-based stages (PnP LM, pose LM, local BA) and the 7-point cubic bit-identical between the
GPU and the CPU restatement."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_device_crmath_equals_quadmath(vsctx, oracle):
    rng = np.random.default_rng(11)
    n = 200000
    x = np.concatenate([(rng.random(n) * 2 - 1) * 8, np.ldexp(rng.random(n), -rng.integers(0, 60, n))])
    c = np.concatenate([rng.random(n) * 2 - 1, 1 - np.ldexp(rng.random(n), -rng.integers(1, 50, n)),
                        -1 + np.ldexp(rng.random(n), -rng.integers(1, 50, n)), [1.0, -1.0, 0.0, 0.5, -0.5]])
    y = np.exp((rng.random(n) * 2 - 1) * 40)
    p = rng.random(n) * 5 - 1.5
    u = rng.random(n)
    for op, a, b in (("sin", x, None), ("cos", x, None), ("acos", c, None), ("log", y, None), ("pow", y, p),
                     ("pow", u, np.full(n, 5.0)), ("pow", u, np.full(n, 1.0 / 3))):
        g = vsctx.crmath(op, a, b)
        o = oracle.crmath(op, a, b)
        bad = np.flatnonzero(g.view(np.uint64) != o.view(np.uint64))
        assert bad.size == 0, (op, bad[:5], a[bad[:5]], g[bad[:5]], o[bad[:5]])
