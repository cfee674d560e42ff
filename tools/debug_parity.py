"""Diagnostics for GPU-vs-oracle mismatches (prints statistics; not a test)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "visual-slam-pipeline_amd", "python"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "tests")]
import oracle_py as oracle  # noqa: E402
import synth  # noqa: E402
import vslam_abi  # noqa: E402


def ulps(a, b):
    ai = a.view(np.int32).astype(np.int64)
    bi = b.view(np.int32).astype(np.int64)
    return np.abs(ai - bi)


def main():
    ctx = vslam_abi.Context(0)
    rng = np.random.default_rng(0)
    hc, wc = 60, 80
    semi = (rng.standard_normal((65, hc, wc)) * 2.0).astype(np.float32)
    dg = rng.standard_normal((256, hc, wc)).astype(np.float32)
    dg /= np.linalg.norm(dg, axis=0, keepdims=True)
    kg, dgpu = ctx.postprocess(semi, dg)
    ko, do = oracle.postprocess(semi, dg, order_mode=1)
    print("kps equal:", np.array_equal(kg.view(np.uint8), ko.view(np.uint8)), len(kg), len(ko))
    if len(kg) == len(ko):
        u = ulps(dgpu, do)
        print("desc: differing elems", int((u > 0).sum()), "of", u.size, "max ulp", int(u.max()),
              "rows", int((u.max(1) > 0).sum()))
    d1 = synth.random_descriptors(400, 1)
    d2 = synth.random_descriptors(400, 2)
    d2[:200] = d1[:200] + 0.1 * synth.random_descriptors(200, 5)
    rg, gg = ctx.match_ratio(d1, d2)
    ro, go = oracle.match_ratio(d1, d2)
    print("raw lens", len(rg), len(ro), "good lens", len(gg), len(go))
    if len(rg) == len(ro):
        print("train_idx diff", int((rg["train_idx"] != ro["train_idx"]).sum()),
              "dist ulp max", int(ulps(rg["distance"], ro["distance"]).max()),
              "dist differing", int((rg["distance"] != ro["distance"]).sum()))
    ctx.close()


if __name__ == "__main__":
    main()
