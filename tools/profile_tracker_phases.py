"""Phase breakdown of the F-matrix kernel inside the tracking loop (profiling build
libvslam_hip_prof.so: `make -C visual-slam-pipeline_amd prof`).  Runs the closed-loop synthetic
sequence through vs_slam like tools/bench_tracker.py and prints k_fmat's lane-0 clock64 phase
cycles per launch (phases as tools/profile_fmat_phases.py), and k_pnp_hyp's phase cycles summed
over a solve_pnp call's hypotheses (100 per call)."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visual-slam-pipeline_amd", "python"))


def main():
    import torch

    import synth
    import vslam_abi as va
    lib = va.load_library(os.environ.get("VS_PROF_LIB") or os.path.join(ROOT, "visual-slam-pipeline_amd", "libvslam_hip_prof.so"))
    lib.vs_debug_fm_cycles.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.vs_debug_pnp_cycles.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.vs_debug_r3_cycles.argtypes = [ctypes.c_void_p, ctypes.c_int]
    U, B, steps = 126, 32, 4
    L = synth.loop_sequence(U)
    dev = torch.device("cuda", 0)
    wrap = np.concatenate([np.arange(U), np.arange(B)])
    bgr = torch.from_numpy(L["bgr"][wrap]).to(dev)
    dep = torch.from_numpy(L["depth"][wrap]).to(dev)
    hdep = [L["depth"][i] for i in wrap]
    ctx = va.Context(0)
    S = va.Slam(ctx, max_batch=B)

    def step(k):
        g0 = k * B
        i0 = g0 % U
        return S.process_batch_dev(B, bgr[i0].data_ptr(), dep[i0].data_ptr(), hdep[i0:i0 + B],
                                   [1311868164.0 + 0.1 * (g0 + j) for j in range(B)], [3 * (g0 + j) for j in range(B)])

    step(0)
    torch.cuda.synchronize()
    cyc = np.zeros(8, np.uint64)
    pcyc = np.zeros(32, np.uint64)  # vs_debug_pnp_cycles copies 32 counters
    rcyc = np.zeros(8, np.uint64)
    lib.vs_debug_fm_cycles(cyc.ctypes.data, 1)
    lib.vs_debug_pnp_cycles(pcyc.ctypes.data, 1)
    lib.vs_debug_r3_cycles(rcyc.ctypes.data, 1)
    ctx.profile(True)
    ctx.profile_reset()
    for k in range(1, 1 + steps):
        step(k)
    torch.cuda.synchronize()
    lib.vs_debug_fm_cycles(cyc.ctypes.data, 1)
    lib.vs_debug_pnp_cycles(pcyc.ctypes.data, 1)
    lib.vs_debug_r3_cycles(rcyc.ctypes.data, 1)
    prof = ctx.profile_read()
    calls = max(1, prof.get("fmat_ransac", (0, 1))[1])
    names = ["-", "solve7", "score", "replay", "final", "rng+mod", "reject", "collinear"]
    print(json.dumps({"fmat_launches": calls, "fmat_ms_per_launch": prof.get("fmat_ransac", (0, 1))[0] / calls,
                      "kcycles_per_launch": {names[k]: round(float(cyc[k]) / calls / 1e3, 1) for k in range(1, 8)},
                      "pnp_hyp_kcycles_per_hypothesis_x100": {
                          n: round(float(pcyc[k]) / max(1, prof.get("solve_pnp", (0, 1))[1]) / 1e3, 1)
                          for k, n in ((21, "points to LDS + subset"), (22, "control: centroid + covariance"), (23, "control: sym_eig<3>"),
                                       (24, "control: axes, CC"), (25, "control: inverse + alphas"), (0, "control: rest"), (1, "eig: M^T QR + R R^T"), (2, "eig: tridiagonal"),
                                       (3, "eig: multisection"), (13, "eig: inverse iteration"),
                                       (14, "eig: Q back-transform"), (15, "variants: L, rho, initial betas"),
                                       (16, "variants: Gauss-Newton"), (17, "variants: control points, ABt"),
                                       (18, "variants: Kabsch"), (19, "variants: reprojection error"),
                                       (4, "variants: rest"), (20, "best + Rodrigues round trip"),
                                       (5, "count"))},
                      "pnp_ransac_kcycles_per_call": {
                          n: round(float(pcyc[k]) / max(1, prof.get("solve_pnp", (0, 1))[1]) / 1e3, 1)
                          for k, n in ((6, "replay"), (7, "lm tail"), (8, "inlier mask + lm rotations"), (9, "lm point terms"),
                                       (10, "lm reduction"), (11, "lm control+solve"))},
                      "pnp_lm_evaluations_per_call": round(float(pcyc[12]) / max(1, prof.get("solve_pnp", (0, 1))[1]), 2),
                      "ransac3d_kcycles_per_launch": {
                          n: round(float(rcyc[k]) / max(1, prof.get("ransac3d", (0, 1))[1]) / 1e3, 1)
                          for k, n in enumerate(["backproject", "mt_init", "twists", "sampling", "hypotheses",
                                                 "select", "refit"])},
                      "stats": S.stats_dict()}))
    S.close()
    ctx.close()


if __name__ == "__main__":
    main()
