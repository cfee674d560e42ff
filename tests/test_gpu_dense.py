"""F4 dense voxel fusion on the GPU (csrc/dense.hip; reference main.cpp:1081-1146, dense_map.ply
:1463-1474) against the sequential oracle (oracle/orc_dense.cpp).  Bar: bit-exact points in the
same order (integer voxel keys and the reference's fp64 expressions, no contraction), across
integrate calls of 1, 5 and 40 frames (two launch groups), repeated frames, rejected depths; the
PLY text equals the reference's std::fixed / setprecision(6) output; overflow of the cloud, the
table is reported, never silent; voxels far outside the packed range join the cloud like any other; a tracker with a cloud attached fuses
every processed frame with its pose right after Slam::process_frame."""
import numpy as np
import pytest
import torch

import synth
import vslam_abi
from test_dense_oracle import _frames

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _s():
    return torch.cuda.current_stream().cuda_stream


def _gpu_integrate(D, frames):
    d = torch.from_numpy(np.stack([f[0] for f in frames])).to(DEV)
    h, w = d.shape[1:]
    ptrs = [d[i].data_ptr() for i in range(len(frames))]
    D.integrate_dev(ptrs, h, w, np.stack([f[1] for f in frames]), np.stack([f[2] for f in frames]), _s())
    torch.cuda.synchronize()
    return d  # keep alive until the enqueue completed


def test_dense_bit_exact_vs_oracle(vsctx, oracle):
    frames = _frames(46, 480, 640, 7)
    frames.insert(9, frames[3])  # a repeated frame
    D = vslam_abi.Dense(vsctx, table_log2=20, max_points=1 << 19)
    O = oracle.Dense()
    for a, b in ((0, 1), (1, 6), (6, 46), (46, 47)):
        _gpu_integrate(D, frames[a:b])
        for f in frames[a:b]:
            O.integrate(*f)
        got, ref = D.points(), O.points()
        assert got.shape == ref.shape and got.shape[0] > 0, (a, b, got.shape, ref.shape)
        assert np.array_equal(got.view(np.uint64), ref.view(np.uint64)), (a, b)
    D.reset()
    assert D.size() == 0
    _gpu_integrate(D, frames[:3])
    O2 = oracle.Dense()
    for f in frames[:3]:
        O2.integrate(*f)
    assert np.array_equal(D.points(), O2.points())
    D.close()


def test_dense_ply_text(vsctx, tmp_path):
    frames = _frames(2, 480, 640, 3)
    with vslam_abi.Dense(vsctx, table_log2=18, max_points=1 << 16) as D:
        _gpu_integrate(D, frames)
        p = tmp_path / "dense_map.ply"
        D.write_ply(p)
        pts = D.points()
    text = p.read_text()
    head = ("ply\nformat ascii 1.0\nelement vertex %d\nproperty float x\nproperty float y\nproperty float z\n"
            "end_header\n" % len(pts))
    assert text == head + "".join("%.6f %.6f %.6f\n" % tuple(q) for q in pts)


def test_dense_overflow_is_reported(vsctx):
    frames = _frames(2, 480, 640, 5)
    with vslam_abi.Dense(vsctx, table_log2=18, max_points=100) as D:
        _gpu_integrate(D, frames)
        with pytest.raises(vslam_abi.VSError, match="VS_ERR_CAPACITY"):
            D.size()
    with vslam_abi.Dense(vsctx, table_log2=10, max_points=1024) as D:
        _gpu_integrate(D, frames)
        with pytest.raises(vslam_abi.VSError, match="VS_ERR_CAPACITY"):
            D.size()



def test_dense_far_voxels_join_the_cloud(vsctx, oracle, tmp_path):
    """Voxels beyond the packed +-2^20 range (a diverged pose 100 km / 1e12 m out, and a NaN pose
    whose voxels are INT_MIN as x86 (int)floor gives) join the cloud in order like any other, as
    the reference's unordered_set inserts them: no global failure, the PLY is written;
    an empty cloud writes no PLY (main.cpp:1462)."""
    frames = _frames(3, 480, 640, 9)
    far = [(frames[0][0], np.eye(3), np.array([1e5, 0.0, 0.0])), frames[1],
           (frames[2][0], np.eye(3), np.array([1e12, -3e11, 7e10])),
           (frames[2][0], np.eye(3), np.array([np.nan, 0.0, 0.0]))]
    O = oracle.Dense()
    for f in far:
        O.integrate(*f)
    with vslam_abi.Dense(vsctx, table_log2=20, max_points=1 << 18) as D:
        _gpu_integrate(D, far)
        got, ref = D.points(), O.points()
        assert got.shape == ref.shape and got.shape[0] > 0
        assert np.array_equal(got.view(np.uint64), ref.view(np.uint64))
        D.write_ply(tmp_path / "far.ply")
        assert (tmp_path / "far.ply").exists()
    with vslam_abi.Dense(vsctx, table_log2=12, max_points=1024) as D:
        D.write_ply(tmp_path / "empty.ply")
    assert not (tmp_path / "empty.ply").exists()


def test_tracker_fuses_processed_frames(vsctx, oracle):
    seq = synth.sequence(24)
    feats = []
    for i in range(0, len(seq), 8):
        feats += vsctx.extract_batch([f["bgr"] for f in seq[i:i + 8]])
    O = oracle.Dense()
    with vslam_abi.Slam(vsctx, max_batch=8) as S, vslam_abi.Dense(vsctx, table_log2=20, max_points=1 << 19) as D:
        S.attach_dense(D)
        n_proc = 0
        for i, (f, (k, d)) in enumerate(zip(seq, feats)):
            if S.process_features(k, d, f["depth"], f["timestamp"], i):
                n_proc += 1
                ids, _, R, t = S.trajectory()
                assert ids[-1] == i
                O.integrate(f["depth"], R[-1], t[-1])  # the pose right after process_frame
        got = D.points()
        # the device batch path with the cloud attached gives the same cloud
        with vslam_abi.Slam(vsctx, max_batch=8) as S2, vslam_abi.Dense(vsctx, table_log2=20,
                                                                       max_points=1 << 19) as D2:
            S2.attach_dense(D2)
            bgr = torch.from_numpy(np.stack([f["bgr"] for f in seq])).to(DEV)
            dep = torch.from_numpy(np.stack([f["depth"] for f in seq])).to(DEV)
            torch.cuda.synchronize()
            for b0 in range(0, len(seq), 8):
                S2.process_batch_dev(8, bgr[b0].data_ptr(), dep[b0].data_ptr(),
                                     [f["depth"] for f in seq[b0:b0 + 8]],
                                     [f["timestamp"] for f in seq[b0:b0 + 8]], list(range(b0, b0 + 8)))
            got2 = D2.points()
    ref = O.points()
    assert n_proc > 10 and got.shape[0] > 1000
    assert np.array_equal(got.view(np.uint64), ref.view(np.uint64))
    assert np.array_equal(got2.view(np.uint64), ref.view(np.uint64))
