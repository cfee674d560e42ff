"""Layer-by-layer comparison of the GPU MiDaS (csrc/midas.hip) with tests/midas_ref.py (torch fp64):
prints each step's max |diff| relative to its range and stops at the first step beyond 1e-4."""
import ctypes
import os
import sys

if "--reuse" not in sys.argv:
    os.environ["VS_MIDAS_KEEP_TENSORS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visual-slam-pipeline_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np
import torch

import midas_ref
import vslam_abi as va


def main():
    ctx = va.Context(0)
    lib = va.load_library()
    lib.vs_midas_debug_step.restype = ctypes.c_long
    lib.vs_midas_debug_step.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    m = va.Midas(ctx)
    rng = np.random.default_rng(0)
    x = (rng.standard_normal((1, 256, 256, 3)) * 1.0).astype(np.float32)
    if "--frame" in sys.argv:  # a synthetic HD frame through the reference pre-processing
        import synth
        L = synth.loop_sequence(1, workers=1, K=synth.K_HD, w=synth.W_HD, h=synth.H_HD)
        x = midas_ref.preprocess(L["bgr"][0])[None]
    elif "--const" in sys.argv:
        x = np.full((1, 256, 256, 3), 0.5, np.float32)
    d_in = torch.from_numpy(x).cuda()
    d_out = torch.zeros((1, 256, 256), dtype=torch.float32, device="cuda")
    m.forward_dev(1, d_in.data_ptr(), d_out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    trace = []
    ref_out = midas_ref.forward(m.weights(), torch.from_numpy(x).permute(0, 3, 1, 2), trace=trace).numpy()[0]
    o = d_out.cpu().numpy()[0]
    print("final output via forward_dev: max err", float(np.abs(o - ref_out).max()), "range", float(np.ptp(ref_out)))
    if "--reuse" in sys.argv:
        return
    for i, t in enumerate(trace):
        ref = t[0].permute(1, 2, 0).numpy()  # NHWC
        n = lib.vs_midas_debug_step(m.h, i, None)
        got = np.zeros(n, np.float32)
        lib.vs_midas_debug_step(m.h, i, got.ctypes.data)
        got = got.reshape(ref.shape)
        rg = float(ref.max() - ref.min()) or 1.0
        err = float(np.abs(got - ref).max())
        print(f"step {i:3d} shape {ref.shape} range {rg:10.4g} max err {err:10.4g} rel {err / rg:9.3g}", flush=True)
        if err > 1e-2 * rg:
            bad = np.unravel_index(np.argmax(np.abs(got - ref)), ref.shape)
            print("first bad step", i, "at", bad, "got", got[bad], "ref", ref[bad])
            badm = np.abs(got - ref) > 1e-2 * rg
            ys, xs, cs = np.nonzero(badm)
            print("bad elements", int(badm.sum()), "of", badm.size, "rows", ys.min(), ys.max(), "cols", xs.min(), xs.max(),
                  "channels", np.unique(cs)[:20], "nan in got", int(np.isnan(got).sum()))
            print("input finite", bool(np.isfinite(x).all()), "input range", float(x.min()), float(x.max()),
                  "contiguous", x.flags["C_CONTIGUOUS"])
            break
    m.close()
    ctx.close()


if __name__ == "__main__":
    main()
