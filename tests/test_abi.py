"""C-ABI boundary checks that need no GPU: the library loads and exports every declared symbol."""
import ctypes
import os

import pytest

import vslam_abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "vslam_abi.h")


def test_header_declares_expected_entry_points():
    names = vslam_abi.exported_symbols_from_header(HEADER)
    for must in ["vs_create", "vs_destroy", "vs_extract", "vs_extract_batch", "vs_extract_batch_dev",
                 "vs_superpoint_forward", "vs_postprocess", "vs_match_ratio", "vs_match_pairs_dev",
                 "vs_ransac_3d3d", "vs_ransac_3d3d_pairs_dev"]:
        assert must in names


@pytest.mark.skipif(not os.path.exists(vslam_abi.LIB_PATH), reason="libvslam_hip.so not built")
def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(vslam_abi.LIB_PATH)
    missing = [n for n in vslam_abi.exported_symbols_from_header(HEADER) if not hasattr(lib, n)]
    assert missing == []
    # every binding in the ctypes table corresponds to a declared symbol
    declared = set(vslam_abi.exported_symbols_from_header(HEADER))
    assert set(vslam_abi._SIG) <= declared


@pytest.mark.skipif(not os.path.exists(vslam_abi.LIB_PATH), reason="libvslam_hip.so not built")
def test_library_reports_abi_version_without_gpu():
    lib = vslam_abi.load_library()
    assert lib.vs_abi_version() == 1
    assert lib.vs_superpoint_num_params() == 1300865


def test_record_layouts_match_opencv():
    # cv::KeyPoint: Point2f pt, float size, angle, response, int octave, class_id
    assert vslam_abi.KEYPOINT_DTYPE.itemsize == 28
    # cv::DMatch: int queryIdx, trainIdx, imgIdx, float distance
    assert vslam_abi.MATCH_DTYPE.itemsize == 16


@pytest.mark.skipif(not os.path.exists(vslam_abi.LIB_PATH), reason="libvslam_hip.so not built")
def test_cpp_facade_builds_and_links():
    # the C++ host façade (host/vslam_amd.hpp) compiles against the C ABI and links the library;
    # running it needs the GPU (tests/test_gpu_facade.py)
    import subprocess
    pkg = os.path.dirname(vslam_abi.LIB_PATH)
    subprocess.run(["make", "-C", pkg, "-s", "facade_test"], check=True)
    assert os.path.exists(os.path.join(pkg, "facade_test"))
    lib = ctypes.CDLL(vslam_abi.LIB_PATH)
    # façade symbols live in the same library (namespace vslam_amd)
    out = subprocess.run(["nm", "-DC", vslam_abi.LIB_PATH], capture_output=True, text=True).stdout
    for sym in ["vslam_amd::FeatureExtractor::extract", "vslam_amd::match_features", "vslam_amd::solve_pnp",
                "vslam_amd::verify_fundamental", "vslam_amd::Optimizer::optimize_pose"]:
        assert sym in out, sym
    del lib


def test_vspw_weight_converter_roundtrip(tmp_path):
    import sys
    import numpy as np
    import torch
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import superpoint_to_vspw as cv
    assert cv.NUM_PARAMS == 1300865  # == vs_superpoint_num_params()
    g = torch.Generator().manual_seed(0)
    sd = {}
    for name, ci, co, k in cv.LAYERS:
        sd[name + ".weight"] = torch.randn(co, ci, k, k, generator=g)
        sd[name + ".bias"] = torch.randn(co, generator=g)
    torch.save(sd, tmp_path / "sp.pth")
    import subprocess
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "superpoint_to_vspw.py"), str(tmp_path / "sp.pth"),
                    str(tmp_path / "sp.vspw")], check=True, capture_output=True)
    blob = cv.read_vspw(tmp_path / "sp.vspw")
    want = np.concatenate([np.concatenate([sd[n + ".weight"].numpy().ravel(), sd[n + ".bias"].numpy()])
                           for n, *_ in cv.LAYERS])
    assert np.array_equal(blob, want)
