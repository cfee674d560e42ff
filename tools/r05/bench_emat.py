"""k_emat latency per call (round 5): Slam::estimate_motion through the C ABI on two-view problems of
the tracker's sizes, HIP-event stage time ("emat_motion"), with the registrator's iteration counts."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in ("visual-slam-pipeline_amd/python", "tests", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))


def main():
    import vslam_abi
    from test_oracle_emat import two_view
    ctx = vslam_abi.Context(0)
    for n, out in ((100, 0.2), (200, 0.4), (300, 0.3), (400, 0.5)):
        p1, p2, R, t, X, outl = two_view(n, 7, noise=0.4, outlier_frac=out)
        ctx.estimate_motion(p1, p2)
        ctx.profile(True)
        ctx.profile_reset()
        reps = 10
        for _ in range(reps):
            ok, Rg, tg, sc, diag = ctx.estimate_motion(p1, p2)
        pr = ctx.profile_read().get("emat_motion", (0.0, 1))
        ctx.profile(False)
        print(json.dumps({"n": n, "outliers": out, "ms_per_call": round(pr[0] / max(pr[1], 1), 4), "calls": pr[1],
                          "ok": bool(ok), "ransac_iterations": int(diag[1]), "inliers": int(diag[3])}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
