"""F2 on the GPU: the SPCF feature cache as the interchange between batch extraction and the
sequential tracker (reference src/FeatureExtractor.cpp:261-381 format, :52-61 sequential-index
lookup; main.cpp:1048-1050 load, :1323-1325 save).

* vs_extract_batch_dev output written with vs_spcf_write_dev reads back bit for bit;
* DevicePipeline(spcf_path=...) writes each step's records keyed by the processed-frame index;
* tracking replayed from the SPCF file through vs_slam_process_features equals the live
  vs_slam_process_batch_dev run over the same frames bit for bit (trajectory, map, counters)."""
import numpy as np
import pytest
import torch

import synth
import vslam_abi as va

pytestmark = pytest.mark.gpu

N = 64
B = 32
T0 = 1311868164.0


@pytest.fixture(scope="module")
def seq():
    return synth.loop_sequence(126, workers=8)


@pytest.fixture(scope="module")
def spcf_file(vsctx, seq, tmp_path_factory):
    """The first N frames extracted in B-frame device batches and appended to one SPCF file."""
    dev = torch.device("cuda", 0)
    path = tmp_path_factory.mktemp("spcf") / "feats.spcf"
    cap = va.SP_MAX_KEYPOINTS
    recs = []
    for i0 in range(0, N, B):
        bgr = torch.from_numpy(seq["bgr"][i0:i0 + B]).to(dev)
        kps = torch.zeros((B, cap * va.KEYPOINT_DTYPE.itemsize), dtype=torch.uint8, device=dev)
        desc = torch.zeros((B, cap, 256), dtype=torch.float32, device=dev)
        n = torch.zeros(B, dtype=torch.int32, device=dev)
        vsctx.extract_batch_dev(B, bgr.data_ptr(), 480, 640, kps.data_ptr(), desc.data_ptr(), n.data_ptr(), cap,
                                torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        vsctx.spcf_write_dev(path, np.arange(i0, i0 + B), B, kps.data_ptr(), desc.data_ptr(), n.data_ptr(), cap,
                             append=i0 > 0)
        recs.append((kps.cpu().numpy().view(va.KEYPOINT_DTYPE).reshape(B, cap), desc.cpu().numpy(),
                     n.cpu().numpy()))
    return path, recs


def test_extract_batch_dev_spcf_round_trip(spcf_file):
    path, recs = spcf_file
    idx, kps, desc, n = va.spcf_read(path)
    assert idx.tolist() == list(range(N))
    for b0, (k, d, m) in enumerate(recs):
        for j in range(B):
            f = b0 * B + j
            assert n[f] == m[j] > 0
            assert np.array_equal(kps[f, :m[j]].view(np.uint8), k[j, :m[j]].view(np.uint8))
            assert np.array_equal(desc[f, :m[j]].view(np.uint32), d[j, :m[j]].view(np.uint32))


def test_tracking_replayed_from_spcf_equals_live(vsctx, seq, spcf_file):
    path, _ = spcf_file
    dev = torch.device("cuda", 0)
    bgr = torch.from_numpy(seq["bgr"][:N]).to(dev)
    dep = torch.from_numpy(seq["depth"][:N]).to(dev)
    ts = [T0 + 0.1 * g for g in range(N)]
    ids = [3 * g for g in range(N)]
    with va.Slam(vsctx, max_batch=B) as live:
        for i0 in range(0, N, B):
            live.process_batch_dev(B, bgr[i0].data_ptr(), dep[i0].data_ptr(), list(seq["depth"][i0:i0 + B]),
                                   ts[i0:i0 + B], ids[i0:i0 + B])
        live.finish()
        L = (live.stats(), live.trajectory(), live.map_points())
    idx, kps, desc, n = va.spcf_read(path)
    with va.Slam(vsctx, max_batch=B) as rep:
        for g in range(N):  # the reference's sequential extract index g -> cache entry g
            assert idx[g] == g
            rep.process_features(kps[g, :n[g]], desc[g, :n[g]], seq["depth"][g], ts[g], ids[g])
        rep.finish()
        Rp = (rep.stats(), rep.trajectory(), rep.map_points())
    assert np.array_equal(L[0], Rp[0]), (L[0], Rp[0])
    assert L[0][0] == N
    for a, b in zip(L[1], Rp[1]):
        assert np.array_equal(a, b)
    for a, b in zip(L[2], Rp[2]):
        assert np.array_equal(a, b)


def test_device_pipeline_writes_spcf(vsctx, seq, tmp_path):
    from vslam_pipeline import DevicePipeline
    dev = torch.device("cuda", 0)
    Bp = 16
    path = tmp_path / "pipe.spcf"
    pipe = DevicePipeline(vsctx, Bp, spcf_path=str(path))
    outs = []
    for step in range(2):
        fr = torch.from_numpy(seq["bgr"][step * Bp:(step + 1) * Bp]).to(dev)
        de = torch.from_numpy(seq["depth"][step * Bp:(step + 1) * Bp]).to(dev)
        S = pipe.submit(fr, de, frame_count0=step * Bp)
        pipe.collect(S)
        o = DevicePipeline.outputs(S)
        outs.append((o["kps"].cpu().numpy().view(va.KEYPOINT_DTYPE).reshape(Bp, -1), o["desc"].cpu().numpy(),
                     o["n"].cpu().numpy()))
    idx, kps, desc, n = va.spcf_read(path)
    assert idx.tolist() == list(range(2 * Bp))
    for step, (k, d, m) in enumerate(outs):
        for j in range(Bp):
            f = step * Bp + j
            assert n[f] == m[j]
            assert np.array_equal(kps[f, :m[j]].view(np.uint8), k[j, :m[j]].view(np.uint8))
            assert np.array_equal(desc[f, :m[j]].view(np.uint32), d[j, :m[j]].view(np.uint32))
