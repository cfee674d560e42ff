"""Runs the C++ façade program (tests/cpp/test_facade.cpp) on the GPU: FeatureExtractor with the
SPCF cache, match_features, F verification, estimate_motion_3d3d, solve_pnp, Optimizer::
optimize_pose and track_local_map through libvslam_hip.so, called the way the reference calls them."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

PKG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "visual-slam-pipeline_amd")


def test_cpp_facade_program():
    subprocess.run(["make", "-C", PKG, "-s", "facade_test"], check=True)
    r = subprocess.run([os.path.join(PKG, "facade_test")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "FACADE OK" in r.stdout, r.stdout
