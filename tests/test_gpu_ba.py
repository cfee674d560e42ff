"""GPU parity for Optimizer::local_bundle_adjustment (A14, reference src/Optimizer.cpp:187-599).

Same algorithm and per-element accumulation order on both sides (ba_solvers.h; chunked global
sums); the remaining differences are last-ulp libm differences inside Rodrigues, so the LM
trajectory (iterations, accepted steps) must match exactly and poses / points / RMS errors to
1e-9 (relative for the errors and for points, to their distance)."""
import numpy as np
import pytest

import synth
from test_oracle_ba import ba_problem

pytestmark = pytest.mark.gpu


def windowed_problem(N, M, seed, span=5, noise=0.5, pert=0.03):
    """Points visible from `span` consecutive keyframes (the sliding-window structure; synth.ba_window)."""
    return synth.ba_window(N, M, seed, span=span, noise=noise, pert=pert)


def _compare(g, o):
    Rg, tg, Pg, ebg, eag, sg = g
    Ro, to, Po, ebo, eao, so = o
    assert np.array_equal(sg, so), (sg, so)
    assert abs(ebg - ebo) <= 1e-9 * max(1.0, ebo) and abs(eag - eao) <= 1e-9 * max(1.0, eao)
    # points: 1e-9 relative to their distance (the 50 KF / 10k window has weakly constrained
    # points 16 m out whose last-ulp Rodrigues differences grow to ~8e-9 m)
    tol = 1e-9 * np.maximum(1.0, np.linalg.norm(Po, axis=1))[:, None]
    assert np.all(np.abs(Pg - Po) <= tol), np.max(np.abs(Pg - Po))
    assert np.max(np.abs(tg - to)) <= 1e-9 and np.max(np.abs(Rg - Ro)) <= 1e-9


@pytest.mark.parametrize("args", [dict(N=5, M=120, seed=0), dict(N=4, M=60, seed=1, noise=0.3, pert=0.02, outliers=3),
                                  dict(N=8, M=300, seed=2, noise=1.0, pert=0.1, outliers=10)])
def test_local_ba_matches_oracle(vsctx, oracle, args):
    R, t, P, P0, kf, pt, uv = ba_problem(**args)
    _compare(vsctx.local_ba(R, t, P0, kf, pt, uv), oracle.local_ba(R, t, P0, kf, pt, uv))


# (50, 10000, span 3, 1 px, 5 cm): BASELINE config[2], the 50-keyframe / 10k-MapPoint stress
# window exactly as tools/bench_ba.py times it
@pytest.mark.parametrize("N,M,seed,kw", [(10, 2000, 3, {}), (30, 6000, 4, {}), (50, 10000, 5, {}),
                                         (50, 10000, 7, dict(span=3, noise=1.0, pert=0.05))])
def test_local_ba_window_matches_oracle(vsctx, oracle, N, M, seed, kw):
    R, t, P, P0, kf, pt, uv = windowed_problem(N, M, seed, **kw)
    g = vsctx.local_ba(R, t, P0, kf, pt, uv)
    _compare(g, oracle.local_ba(R, t, P0, kf, pt, uv))
    assert g[4] < g[3]


def test_local_ba_bailouts_and_single_step(vsctx, oracle):
    R, t, P, P0, kf, pt, uv = ba_problem(N=3, M=50, seed=3)
    g = vsctx.local_ba(R, t, P0, kf[:19], pt[:19], uv[:19])
    assert g[5][2] == 0 and g[3] == g[4] == 0 and np.array_equal(g[2], P0)
    _compare(vsctx.local_ba(R, t, P0, kf, pt, uv, max_iter=1), oracle.local_ba(R, t, P0, kf, pt, uv, max_iter=1))
    with pytest.raises(RuntimeError):
        vsctx.local_ba(R, t, P0, kf, pt + 1000, uv)  # point index out of range


_BAND_SCRIPT = r"""
import sys
import numpy as np
sys.path[:0] = sys.argv[2].split("|")
import synth, vslam_abi
ctx = vslam_abi.Context(0)
out = {}
for tag, (N, M, seed, kw) in {"c2": (50, 10000, 7, dict(span=3, noise=1.0, pert=0.05)),
                              "s5": (30, 6000, 4, {})}.items():
    R, t, P, P0, kf, pt, uv = synth.ba_window(N, M, seed, **kw)
    g = ctx.local_ba(R, t, P0, kf, pt, uv)
    for i, a in enumerate(g):
        out[f"{tag}_{i}"] = np.asarray(a)
ctx.close()
np.savez(sys.argv[1], **out)
"""


def test_local_ba_band_equals_dense(tmp_path):
    """k_ba_chol_band (the banded Cholesky, chosen for these windows: band 17 and 29) against the dense
    look-ahead kernel (VS_BA_BAND=0): every output bit for bit.  The band kernel skips only products
    with exact zeros outside S's band, in the dense kernel's per-element order."""
    import os
    import subprocess
    import sys
    paths = "|".join(p for p in sys.path if p)
    res = {}
    for band in ("1", "0"):
        f = tmp_path / f"band{band}.npz"
        subprocess.run([sys.executable, "-c", _BAND_SCRIPT, str(f), paths], check=True, timeout=240,
                       env={**os.environ, "VS_BA_BAND": band})
        res[band] = np.load(f)
    assert res["1"].files == res["0"].files
    for k in res["1"].files:
        assert np.array_equal(res["1"][k], res["0"][k]), k
