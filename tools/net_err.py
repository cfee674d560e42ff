"""SuperPoint network error against the torch fp64 restatement (tests/test_oracle._torch_superpoint) at the
parity tests' geometries: prints max |semi - ref| / max(1, max|ref|) and max |desc - ref| per case, so that
Winograd variants can be compared against the tests' stated tolerances (2e-4 relative semi, 2e-5 desc).
Usage: python tools/net_err.py"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "visual-slam-pipeline_amd", "python"), os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests"), ROOT):
    sys.path.insert(0, p)

import oracle_py  # noqa: E402  (checker only: gray conversion)
import synth  # noqa: E402
import vslam_abi  # noqa: E402
from test_oracle import _torch_superpoint  # noqa: E402


def main():
    out = {}
    with vslam_abi.Context(0) as ctx:
        w = ctx.weights()
        seq = synth.sequence(2)
        cases = [("480x640", oracle_py.gray_to_f32(oracle_py.bgr_to_gray(seq[0]["bgr"])))]
        for h, wd in ((152, 200), (64, 96)):
            rng = np.random.default_rng(h * wd)
            cases.append((f"{h}x{wd}", rng.random((h, wd), dtype=np.float32)))
        for name, gray in cases:
            semi, desc = ctx.superpoint_forward(gray)
            ts, td = _torch_superpoint(w, gray)
            out[name] = {"semi_rel": float(np.max(np.abs(semi - ts)) / max(1.0, float(np.max(np.abs(ts))))),
                         "desc_abs": float(np.max(np.abs(desc - td))),
                         "semi_rms_rel": float(np.sqrt(np.mean((semi - ts) ** 2)) / max(1.0, float(np.max(np.abs(ts)))))}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
