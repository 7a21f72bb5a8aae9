"""bench.py's launcher and aggregation logic on the CPU (no GPU call).

The driver runs `bench.py --gpus N` under torch.distributed.run; run bare,
`--gpus N` must start N ranks itself or fail clearly, and `value` must be the
whole-job rate over the slowest rank (gloo, world size 2)."""
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_modes_and_default_workloads():
    a = bench.parse_args([])
    assert a.mode == "pose" and a.workload == "c2_meshrir_1024x256x512" and a.gpus is None
    assert bench.parse_args(["--mode", "ray-shard"]).workload == "c5_simu_4096x512x2048"
    assert bench.parse_args(["--mode", "ddp-train"]).workload == "c4_raf_empty_b4_per_gpu"
    assert bench.parse_args(["--mode", "ray-shard", "--workload", "c1_meshrir_plumbing"]).workload == \
        "c1_meshrir_plumbing"


def test_resolve_world_under_torchrun():
    assert bench.resolve_world(bench.parse_args([]), env={"WORLD_SIZE": "4"}) == ("run", 4)
    assert bench.resolve_world(bench.parse_args(["--gpus", "4"]), env={"WORLD_SIZE": "4"}) == ("run", 4)
    with pytest.raises(SystemExit, match="WORLD_SIZE=2"):
        bench.resolve_world(bench.parse_args(["--gpus", "8"]), env={"WORLD_SIZE": "2"})


def test_resolve_world_bare():
    assert bench.resolve_world(bench.parse_args([]), env={}, device_count=0) == ("run", 1)
    assert bench.resolve_world(bench.parse_args(["--gpus", "1"]), env={}, device_count=0) == ("run", 1)
    assert bench.resolve_world(bench.parse_args(["--gpus", "8"]), env={}, device_count=8) == ("launch", 8)
    with pytest.raises(SystemExit, match="only 1 GPU"):
        bench.resolve_world(bench.parse_args(["--gpus", "2"]), env={}, device_count=1)


def test_launch_command_is_one_process_per_gpu():
    cmd = bench.launch_command(8, ["--gpus", "8", "--steps", "5"], 29500, script="/x/bench.py")
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29500" in cmd
    assert cmd[-4:] == ["--gpus", "8", "--steps", "5"] and cmd[-5] == "/x/bench.py"


def test_bare_multi_gpu_request_fails_clearly_without_gpus():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = ""  # no device visible, even on a GPU box
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode != 0
    assert "--gpus 2 requested but only 0 GPU(s) visible" in p.stderr


def test_whole_job_rate():
    # 2 ranks x 10 steps x 1000 units in 4 s (the slowest rank)
    assert bench.whole_job_rate(1000, 2, 10, 4.0) == 5000.0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _timed_worker(rank, world, port, q):
    import time

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # rank 1 is slower; every rank must report the slowest time
        el, _ = bench.timed(lambda: time.sleep(0.05 + 0.25 * rank), world, torch.device("cpu"))
        q.put((rank, el))
    finally:
        dist.destroy_process_group()


def test_timed_reports_max_over_ranks_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_timed_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out[0] == out[1] >= 0.3


def test_resolve_world_oversubscribe():
    """--oversubscribe launches the ranks even with fewer GPUs than ranks
    (they all use cuda:0 over gloo: the launcher rehearsal of the GPU test)."""
    args = bench.parse_args(["--gpus", "2", "--oversubscribe"])
    assert bench.resolve_world(args, env={}, device_count=1) == ("launch", 2)
    assert bench.resolve_world(args, env={"WORLD_SIZE": "2"}) == ("run", 2)


def test_cpu_baseline_modes_on_a_small_workload():
    """Every mode's CPU leg runs the oracle on its own sample and reports
    ray-samples/s (the ray-shard leg on a sphere of about R/8 rays)."""
    from avr_amd.workloads import WORKLOADS

    w = WORKLOADS["c1_meshrir_plumbing"]
    for mode in ("pose", "ray-shard", "ddp-train"):
        d = bench.cpu_baseline(w, 0.05, mode)
        assert d["value"] > 0 and d["unit"] == "ray-samples/s" and d["kind"] == "port"
    shard = bench.cpu_baseline(WORKLOADS["c1_meshrir_plumbing"].replace(n_azi=48, n_ele=5), 0.05, "ray-shard")
    assert "32 rays (6x5+2)" in shard["sample"]


def _cpu_leg_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from avr_amd.workloads import WORKLOADS

        res = {}
        for mode in ("pose", "ray-shard", "ddp-train"):
            args = bench.parse_args(["--mode", mode, "--workload", "c1_meshrir_plumbing", "--cpu-budget", "0.05"])
            r = {}
            bench.attach_cpu_baseline(r, args, WORKLOADS[args.workload], world, rank)
            res[mode] = r
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_cpu_baseline_in_the_two_rank_line_gloo():
    """World size 2: rank 0's result carries the CPU leg (cores stated) in
    every mode, the other rank's does not, and both pass the barrier."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cpu_leg_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for mode in ("pose", "ray-shard", "ddp-train"):
        cb = out[0][mode]["cpu_baseline"]
        assert cb["value"] > 0 and cb["cores"] >= 1 and "rank 0" in cb["note"]
        assert "cpu_baseline" not in out[1][mode]


def test_cpu_leg_threads(monkeypatch):
    monkeypatch.setenv("AVR_CPU_THREADS", "3")
    assert bench.cpu_leg_threads() == 3
    monkeypatch.delenv("AVR_CPU_THREADS")
    assert bench.cpu_leg_threads() >= torch.get_num_threads()
