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
