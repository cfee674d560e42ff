"""Convert SuperPoint weights to the VSPW file vs_create() loads (include/vslam_abi.h).

The reference runs `superpoint.onnx` under ONNX Runtime (FeatureExtractor.cpp:22-44); the same
network's PyTorch state_dict (magic-leap SuperPointNet layer names conv1a ... convDb) converts
directly.  VSPW: u32 magic 0x57505356 ("VSPW"), u32 version 1, u64 float count, then for each layer
in the order conv1a, conv1b, conv2a, conv2b, conv3a, conv3b, conv4a, conv4b, convPa, convPb,
convDa, convDb: weight [Cout][Cin][k][k] then bias [Cout], fp32 little-endian.

    python tools/superpoint_to_vspw.py superpoint_v1.pth superpoint.vspw

The state_dict is read with torch.load(weights_only=True) (no code from the file is executed).
"""
import struct
import sys

import numpy as np

LAYERS = [("conv1a", 1, 64, 3), ("conv1b", 64, 64, 3), ("conv2a", 64, 64, 3), ("conv2b", 64, 64, 3),
          ("conv3a", 64, 128, 3), ("conv3b", 128, 128, 3), ("conv4a", 128, 128, 3), ("conv4b", 128, 128, 3),
          ("convPa", 128, 256, 3), ("convPb", 256, 65, 1), ("convDa", 128, 256, 3), ("convDb", 256, 256, 1)]
NUM_PARAMS = sum(co * ci * k * k + co for _, ci, co, k in LAYERS)  # 1,300,865 == vs_superpoint_num_params()
MAGIC, VERSION = 0x57505356, 1


def blob_from_state_dict(sd):
    parts = []
    for name, ci, co, k in LAYERS:
        w = np.asarray(sd[name + ".weight"], dtype=np.float32)
        b = np.asarray(sd[name + ".bias"], dtype=np.float32)
        if w.shape != (co, ci, k, k) or b.shape != (co,):
            raise ValueError(f"{name}: expected weight {(co, ci, k, k)} / bias {(co,)}, got {w.shape} / {b.shape}")
        parts += [w.reshape(-1), b]
    blob = np.concatenate(parts)
    assert blob.size == NUM_PARAMS
    return blob


def write_vspw(path, blob):
    blob = np.ascontiguousarray(blob, dtype="<f4")
    with open(path, "wb") as f:
        f.write(struct.pack("<IIQ", MAGIC, VERSION, blob.size))
        f.write(blob.tobytes())


def read_vspw(path):
    with open(path, "rb") as f:
        magic, version, count = struct.unpack("<IIQ", f.read(16))
        if magic != MAGIC or version != VERSION or count != NUM_PARAMS:
            raise ValueError("not a VSPW v1 SuperPoint file")
        return np.frombuffer(f.read(4 * count), dtype="<f4")


def main():
    import torch
    src, dst = sys.argv[1], sys.argv[2]
    sd = torch.load(src, map_location="cpu", weights_only=True)
    if "state_dict" in sd:
        sd = sd["state_dict"]
    sd = {k.replace("module.", ""): v.numpy() for k, v in sd.items()}
    write_vspw(dst, blob_from_state_dict(sd))
    print(f"wrote {dst}: {NUM_PARAMS} floats")


if __name__ == "__main__":
    main()
