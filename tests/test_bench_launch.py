"""bench.py's own N-rank launch (`--gpus N` without an external launcher) and its roofline
bookkeeping — host logic only, no GPU.  The per-frame loop this shards is main.cpp:1096-1107."""
import json
import os
import subprocess
import sys

import pytest

import bench


def test_launch_plan_single_rank():
    assert bench.launch_plan(1, {}, []) == ("run", None)
    assert bench.launch_plan(1, {"WORLD_SIZE": "1"}, []) == ("run", None)


def test_launch_plan_under_a_launcher():
    assert bench.launch_plan(8, {"WORLD_SIZE": "8", "RANK": "3"}, []) == ("run", None)


def test_launch_plan_mismatch_and_bad_count_fail():
    mode, msg = bench.launch_plan(4, {"WORLD_SIZE": "2"}, [])
    assert mode == "error" and "WORLD_SIZE=2" in msg
    assert bench.launch_plan(0, {}, [])[0] == "error"


def test_launch_plan_spawns_n_ranks():
    mode, cmd = bench.launch_plan(4, {}, ["--gpus", "4", "--steps", "3"])
    assert mode == "spawn"
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd and "--nnodes=1" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"]
    assert os.path.samefile(cmd[-5], bench.__file__)


def test_spawned_launcher_runs_n_ranks_and_relays_rank0(tmp_path):
    """The command launch_plan builds really starts N ranks with RANK / WORLD_SIZE set (gloo, CPU)
    and returns the ranks' exit code; a stand-in script replaces bench.py."""
    stub = tmp_path / "rank.py"
    stub.write_text(
        "import os, json, torch.distributed as dist\n"
        "dist.init_process_group('gloo')\n"
        "r, w = dist.get_rank(), dist.get_world_size()\n"
        "dist.barrier()\n"
        "if r == 0: print(json.dumps({'n_gpus': w, 'env_world': int(os.environ['WORLD_SIZE'])}), flush=True)\n"
        "dist.destroy_process_group()\n")
    mode, cmd = bench.launch_plan(2, {}, [])
    cmd = cmd[:-1] + [str(stub)]  # the script path is the last element when no args are passed
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1 and json.loads(line[0]) == {"n_gpus": 2, "env_world": 2}


def test_bench_exits_nonzero_on_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="2")
    p = subprocess.run([sys.executable, bench.__file__, "--gpus", "3"], env=env, capture_output=True, text=True,
                       timeout=240)
    assert p.returncode == 2 and "WORLD_SIZE=2" in p.stderr


@pytest.mark.parametrize("name,ok", [("vs::k_conv3_db<true, 1, true, false, 4>", True),
                                     ("vs::k_conv3_db<true, 1, true, false>", True),
                                     ("vs::k_conv3_db<true, 1, true, false4>", False),
                                     ("vs::k_conv3_db<false, 6, false, true, 4>", False)])
def test_stage_kernel_prefix(name, ok):
    assert bench.kernel_matches(name, bench.STAGE_KERNEL_DIRECT["conv1_fused"]) == ok


@pytest.mark.parametrize("name,ok", [("vs::k_wino3<true, true>", True), ("vs::k_wino3<true, false>", False),
                                     ("vs::k_wino3<false, false>", False)])
def test_stage_kernel_prefix_winograd(name, ok):
    assert bench.kernel_matches(name, bench.STAGE_KERNEL_WINO["conv1_fused"]) == ok


def test_pmc_traffic_per_frame(tmp_path, monkeypatch):
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "pmc_traffic.json").write_text(json.dumps({
        "tag": "rX", "frames_per_launch": 8,
        "kernels": {"vs::k_conv3_db<true, 1, true, false, 4>": {"hbm_bytes_per_launch": 8 * 1000.0}}}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.pmc_traffic(bench.STAGE_KERNEL_DIRECT["conv1_fused"]) == (1000.0, "rX", 8)
    assert bench.pmc_traffic(bench.STAGE_KERNEL_DIRECT["conv2a"]) == (None, None, None)


def test_ba_bytes_formula():
    # 30k observations, 10k points, 50 keyframes: ~7 MB per LM iteration (SURVEY.md 8(d) quotes ~5 MB)
    b = bench.ba_bytes_per_iteration(50, 10000, 30000)
    assert 5e6 < b < 8e6


# ---- config[3] through the C ABI (bench.frontend_batch: vs_batch_submit_dev / vs_batch_collect) ----
def test_batch_schedule_keeps_two_steps_in_flight():
    events, live, peak = [], [0], [0]

    def submit(i):
        events.append(("s", i))
        live[0] += 1
        peak[0] = max(peak[0], live[0])

    def collect():
        live[0] -= 1
        done = [e[1] for e in events if e[0] == "s"][len([e for e in events if e[0] == "c"])]
        events.append(("c", done))
        return done

    out = bench.batch_schedule(submit, collect, 3, 5)
    assert out == [3, 4, 5, 6, 7] and peak[0] == 2 and live[0] == 0
    # the next step is submitted before the previous one is collected (the overlap), in order
    assert events[:4] == [("s", 3), ("s", 4), ("c", 3), ("s", 5)]
    assert bench.batch_schedule(submit, collect, 0, 1) == [0]


@pytest.mark.parametrize("world", [1, 2, 8])
def test_frontend_frames_are_distinct(world):
    """config[3]'s ranks take disjoint, consecutive blocks of one world * B-frame drive
    (no frame repeats), and each halo frame is the frame before the rank's block."""
    B = 318
    seen = []
    for r in range(world):
        own, halo = bench.frontend_frame_indices(B, r, world)
        assert own == list(range(r * B, (r + 1) * B))
        assert halo == (own[0] - 1) % (world * B)
        seen += own
    assert sorted(seen) == list(range(world * B))


def test_batch_halo_rule():
    assert not bench.batch_halo_needed(0, 0, 1) and not bench.batch_halo_needed(5, 0, 1)  # no communicator
    assert not bench.batch_halo_needed(0, 0, 4)                                          # rank 0, first step
    assert bench.batch_halo_needed(0, 1, 4) and bench.batch_halo_needed(1, 0, 4)


def _share_id_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    uid = bench.share_batch_id(rank, world, lambda: bytes(range(7, 135)), "cpu", 128)
    q.put((rank, uid))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_share_batch_id_reaches_every_rank(world):
    """rank 0's vs_batch communicator id arrives byte for byte on every rank over the process group
    (gloo here; the GPU box's RCCL group carries the same broadcast)."""
    import socket

    import torch.multiprocessing as mp
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_share_id_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(60)
    assert all(got[r] == bytes(range(7, 135)) for r in range(world))
    assert bench.share_batch_id(0, 1, lambda: b"x") is None
