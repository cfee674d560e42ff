"""World-size-2 CPU test (gloo) of the frame-sharded feature interchange:
the same FeatureExchange code the RCCL path runs in DevicePipeline / bench.py."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

B, CAP = 3, 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _frame_value(step, g):
    return float(1000 * step + g + 1)


def _worker(rank, world, port, errq, gather=True):
    try:
        import torch.distributed as dist

        from vslam_pipeline import KP_BYTES, FeatureExchange
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        x = FeatureExchange(B, CAP, rank, world, device="cpu", gather=gather)
        kps = torch.zeros((B + 1, CAP * KP_BYTES), dtype=torch.uint8)
        desc = torch.zeros((B + 1, CAP, 256), dtype=torch.float32)
        n = torch.zeros(B + 1, dtype=torch.int32)
        for step in range(3):
            for b in range(B):  # this rank's frames: global index rank*B + b
                g = rank * B + b
                v = _frame_value(step, g)
                desc[1 + b].fill_(v)
                kps[1 + b].fill_(int(v) % 251)
                n[1 + b] = int(v) % 400
            got = x.exchange(kps, desc, n)
            if gather:  # gathered tables: the whole step in global frame order
                g_kps, g_desc, g_n = got
                for g in range(world * B):
                    v = _frame_value(step, g)
                    assert float(g_desc[g, 0, 0]) == v and int(g_n[g]) == int(v) % 400
                    assert int(g_kps[g, 0]) == int(v) % 251
            else:
                assert got is None
            # slot 0 = frame rank*B - 1 (previous step's global last frame for rank 0)
            if rank > 0:
                want = _frame_value(step, rank * B - 1)
            elif step > 0:
                want = _frame_value(step - 1, world * B - 1)
            else:
                want = None
            if want is None:
                assert int(n[0]) == 0 and float(desc[0].abs().sum()) == 0.0
            else:
                assert float(desc[0, 0, 0]) == want and int(n[0]) == int(want) % 400
                assert int(kps[0, 0]) == int(want) % 251
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:  # report to the parent
        errq.put(f"rank {rank}: {type(e).__name__}: {e}")
        raise


@pytest.mark.parametrize("world,gather", [(2, True), (2, False), (3, False)])
def test_feature_exchange_gloo(world, gather):
    """All-gather (SPCF consumer) and the default halo ring (one record per rank per step)."""
    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, errq, gather)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, errs
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def test_bench_block_indexing_covers_every_pair_once():
    # bench.py: rank r owns [rB, (r+1)B) plus the halo frame rB-1; its pairs are (g-1, g) for g
    # in its block, so over the ranks every consecutive pair of the step appears exactly once
    for world in (1, 2, 4, 8):
        n_total, pairs = world * B, []
        for rank in range(world):
            idx = [(rank * B - 1) % n_total] + list(range(rank * B, (rank + 1) * B))
            pairs += [(idx[p], idx[p + 1]) for p in range(B)]
        assert sorted(pairs) == sorted(((g - 1) % n_total, g) for g in range(n_total))
