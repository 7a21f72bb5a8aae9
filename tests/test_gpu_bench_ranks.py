"""GPU: the N-rank bench path end to end, before the driver's scaling run.

`bench.py --gpus 2` outside torchrun starts its ranks through the same
launcher branch the 8-GPU run takes (a torch.distributed.run child, one
process per rank, rendezvous on 127.0.0.1).  The test box has one GPU, so
`--oversubscribe` puts both ranks on cuda:0 with a gloo process group (RCCL
needs a GPU per rank); everything else -- rank discovery, the sharded
render with its spectrum all-reduce, DDP's gradient all-reduce, the barrier
and max-over-ranks timing, rank 0's single JSON line -- is the code the
scaling run executes.  Reference pattern: avr_runner_ddp.py:37-46, 98."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=400):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--oversubscribe",
           "--steps", "3", "--warmup", "1", "--cpu-budget", "0.2", *args]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, (p.returncode, p.stdout[-3000:], p.stderr[-3000:])
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-3000:]  # rank 0 only
    d = json.loads(lines[0])
    # the CPU leg is in the N-rank line too (north_star: "in the same run")
    cb = d["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] >= 1 and cb["unit"] == "ray-samples/s" and "rank 0" in cb["note"]
    return d


def test_bench_two_ranks_ray_shard():
    d = _bench("--mode", "ray-shard", "--workload", "c1_meshrir_plumbing")
    assert d["n_gpus"] == 2 and d["scaling"] == "strong"
    assert d["config"]["rays_per_rank"] == 16 and d["value"] > 0
    assert "oversubscribed" in d


def test_bench_two_ranks_ddp_train():
    d = _bench("--mode", "ddp-train", "--workload", "c3_raf_furnished_b4")
    assert d["n_gpus"] == 2 and d["scaling"] == "weak"
    assert d["config"]["global_batch"] == 8 and d["config"]["grad_allreduce_bytes"] > 0
    assert d["value"] > 0


def test_bench_two_ranks_pose():
    d = _bench("--mode", "pose", "--workload", "c1_meshrir_plumbing", "--no-network")
    assert d["n_gpus"] == 2 and d["value"] > 0
