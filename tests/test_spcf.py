"""F2: the SPCF feature cache (reference src/FeatureExtractor.cpp:261-381) through the C ABI
(vs_spcf_write / vs_spcf_read; host code, no GPU).  The expected bytes are packed here field by
field in the order of the reference's save_cache (:333-377) and parsed as its load_cache does
(:269-313): magic, version, count, then per entry frame_idx, num_kp, 7-field keypoints, rows, cols,
type and the raw CV_32F descriptor rows."""
import struct

import numpy as np
import pytest

import vslam_abi as va


def _pack(entries):
    """entries: [(frame_idx, kps (structured), desc (n,256) or None, mat=(rows, cols, type))]"""
    out = struct.pack("<III", 0x53504346, 1, len(entries))
    for idx, kps, desc, mat in entries:
        out += struct.pack("<ii", idx, len(kps))
        for k in kps:
            out += struct.pack("<fffffii", k["x"], k["y"], k["size"], k["angle"], k["response"], k["octave"],
                               k["class_id"])
        out += struct.pack("<iii", *mat)
        if desc is not None and mat[0] > 0 and mat[1] > 0:
            out += np.ascontiguousarray(desc, "<f4").tobytes()
    return out


def _frames(F, cap, ns, seed=0):
    rng = np.random.default_rng(seed)
    kps = np.zeros((F, cap), va.KEYPOINT_DTYPE)
    kps["x"] = rng.uniform(0, 640, (F, cap))
    kps["y"] = rng.uniform(0, 480, (F, cap))
    kps["size"] = 1.0
    kps["angle"] = -1.0
    kps["response"] = rng.uniform(0, 1, (F, cap))
    kps["class_id"] = -1
    desc = rng.standard_normal((F, cap, 256)).astype(np.float32)
    return kps, desc, np.asarray(ns, np.int32)


def test_write_is_the_reference_byte_layout(tmp_path):
    kps, desc, n = _frames(3, 8, [8, 0, 5])
    path = tmp_path / "a.spcf"
    va.spcf_write(path, [0, 1, 2], kps, desc, n)
    want = _pack([(0, kps[0, :8], desc[0, :8], (8, 256, 5)), (1, kps[1, :0], None, (0, 0, 0)),
                  (2, kps[2, :5], desc[2, :5], (5, 256, 5))])
    assert path.read_bytes() == want


def test_read_reference_file_round_trip_and_last_entry_wins(tmp_path):
    kps, desc, _ = _frames(3, 6, [6, 6, 6], seed=1)
    # out of order, a repeated index (the later entry wins, FeatureExtractor.cpp:310), an empty
    # cv::Mat() entry and a 0 x 256 CV_32F entry
    data = _pack([(7, kps[0, :6], desc[0, :6], (6, 256, 5)), (2, kps[1, :3], desc[1, :3], (3, 256, 5)),
                  (7, kps[2, :4], desc[2, :4], (4, 256, 5)), (4, kps[0, :0], None, (0, 0, 0)),
                  (5, kps[0, :0], None, (0, 256, 5))])
    path = tmp_path / "b.spcf"
    path.write_bytes(data)
    idx, k, d, n = va.spcf_read(path, cap=6)
    assert idx.tolist() == [2, 4, 5, 7] and n.tolist() == [3, 0, 0, 4]
    assert np.array_equal(k[0, :3].view(np.uint8), kps[1, :3].view(np.uint8))
    assert np.array_equal(k[3, :4].view(np.uint8), kps[2, :4].view(np.uint8))
    assert np.array_equal(d[3, :4].view(np.uint32), desc[2, :4].view(np.uint32))


def test_append_extends_the_file_and_updates_the_count(tmp_path):
    kps, desc, n = _frames(4, 5, [5, 4, 3, 2], seed=2)
    path = tmp_path / "c.spcf"
    va.spcf_write(path, [0, 1], kps[:2], desc[:2], n[:2], append=True)  # missing file: created
    va.spcf_write(path, [2, 3], kps[2:], desc[2:], n[2:], append=True)
    one = tmp_path / "d.spcf"
    va.spcf_write(one, [0, 1, 2, 3], kps, desc, n)
    assert path.read_bytes() == one.read_bytes()


def test_errors(tmp_path):
    kps, desc, n = _frames(1, 4, [4], seed=3)
    good = _pack([(0, kps[0], desc[0], (4, 256, 5))])
    cases = {
        "magic": b"XXXX" + good[4:],
        "version": good[:4] + struct.pack("<I", 2) + good[8:],
        "truncated": good[:-10],
        "type": good.replace(struct.pack("<iii", 4, 256, 5), struct.pack("<iii", 4, 256, 6)),
        "cols": good.replace(struct.pack("<iii", 4, 256, 5), struct.pack("<iii", 4, 128, 5))[:-4 * 128 * 4],
    }
    for name, data in cases.items():
        p = tmp_path / f"{name}.spcf"
        p.write_bytes(data)
        with pytest.raises(va.VSError, match="VS_ERR_IO"):
            va.spcf_read(p, cap=4)
    p = tmp_path / "ok.spcf"
    p.write_bytes(good)
    with pytest.raises(va.VSError, match="VS_ERR_CAPACITY"):
        va.spcf_read(p, cap=3)
    with pytest.raises(va.VSError, match="VS_ERR_ARG"):
        va.spcf_write(tmp_path / "e.spcf", [0], kps, desc, [5])
    with pytest.raises(va.VSError, match="VS_ERR_IO"):
        va.spcf_read(tmp_path / "missing.spcf")
