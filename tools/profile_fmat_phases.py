"""Per-phase cycle breakdown of the F-matrix kernel (profiling build libvslam_hip_prof.so, built by
`make -C visual-slam-pipeline_amd prof`).  Phases (lane-0 clock64 deltas summed over workgroups):
0 unused, 1 7-point solves, 2 scoring, 3 replay, 4 final inliers/compaction/errors,
5 RNG draws + modulo, 6 repeat rejection, 7 collinearity."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("visual-slam-pipeline_amd/python", "tests", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))


def main():
    import torch

    import vslam_abi as va
    lib = va.load_library(os.path.join(ROOT, "visual-slam-pipeline_amd", "libvslam_hip_prof.so"))
    lib.vs_debug_fm_cycles.argtypes = [ctypes.c_void_p, ctypes.c_int]
    from test_gpu_fmat import _pairs_inputs
    from test_oracle_fmat import two_view
    ctx = va.Context(0)
    P, n = 32, 300
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8)).cuda()  # noqa: E731
    names = ["-", "solve7", "score", "replay", "final", "rng+mod", "reject", "collinear"]
    for out in [float(x) for x in os.environ.get("FM_OUT", "0.1,0.3").split(",")]:
        probs = [two_view(n, 1000 + i, 0.7, out)[:2] for i in range(P)]
        cap, pairs, kp_tab, goods, ngood = _pairs_inputs(va, probs)
        bufs = [dev(pairs), dev(kp_tab), dev(goods), dev(ngood)]
        d_F = torch.zeros(P, 9, dtype=torch.float64, device="cuda")
        d_kept = torch.zeros(P * cap * 16, dtype=torch.uint8, device="cuda")
        d_nk = torch.zeros(P, dtype=torch.int32, device="cuda")
        d_err = torch.zeros(P, 2, dtype=torch.float64, device="cuda")
        d_diag = torch.zeros(P, 8, dtype=torch.int32, device="cuda")
        cyc = np.zeros(8, np.uint64)
        ctx.fmat_verify_pairs_dev(P, bufs[0].data_ptr(), bufs[1].data_ptr(), cap, bufs[2].data_ptr(),
                                  bufs[3].data_ptr(), d_F.data_ptr(), d_kept.data_ptr(), d_nk.data_ptr(),
                                  d_err.data_ptr(), d_diag.data_ptr())
        torch.cuda.synchronize()
        lib.vs_debug_fm_cycles(cyc.ctypes.data, 1)
        ctx.fmat_verify_pairs_dev(P, bufs[0].data_ptr(), bufs[1].data_ptr(), cap, bufs[2].data_ptr(),
                                  bufs[3].data_ptr(), d_F.data_ptr(), d_kept.data_ptr(), d_nk.data_ptr(),
                                  d_err.data_ptr(), d_diag.data_ptr())
        torch.cuda.synchronize()
        lib.vs_debug_fm_cycles(cyc.ctypes.data, 1)
        dg = d_diag.cpu().numpy()
        print(json.dumps({"outliers": out, "chunks_mean": float(dg[:, 7].mean()),
                          "iters_mean": float(dg[:, 1].mean()),
                          "kcycles_per_pair": {names[k]: round(float(cyc[k]) / P / 1e3, 1) for k in range(1, 8)}}))
    ctx.close()


if __name__ == "__main__":
    main()
