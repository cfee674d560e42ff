"""The SuperPoint network's outputs (semi, descriptor grid) for 4 fixed synthetic frames through the
library VS_LIB_PATH names (default the in-tree build), saved to an npz: A/B kernel changes that must
keep the network output bit-identical are checked by comparing two dumps (tools/r04/net_ab.sh)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visual-slam-pipeline_amd", "python"))

import torch  # noqa: E402

import vslam_abi  # noqa: E402


def main():
    rng = np.random.default_rng(5)
    nb, H, W = 4, 480, 640
    dev = torch.device("cuda", 0)
    bgr = torch.from_numpy(rng.integers(0, 256, (nb, H, W, 3), dtype=np.uint8)).to(dev)
    semi = torch.zeros((nb, 60, 80, vslam_abi.SEMI_CH), dtype=torch.float32, device=dev)
    dg = torch.zeros((nb, 60, 80, vslam_abi.DESC_DIM), dtype=torch.float32, device=dev)
    with vslam_abi.Context(0) as ctx:
        ctx.network_batch_dev(nb, bgr.data_ptr(), H, W, semi.data_ptr(), dg.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    np.savez(sys.argv[1], semi=semi.cpu().numpy(), dgrid=dg.cpu().numpy())


if __name__ == "__main__":
    main()
