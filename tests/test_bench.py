"""bench.py contract: one JSON line with the driver's keys, single process and
a 2-rank gloo run through torch.distributed.run (the multi-GPU launch path,
exercised on CPU)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_single_process(capsys):
    import bench
    assert bench.main(["--steps", "2", "--warmup", "1", "--classes", "40", "--queries", "12"]) == 0
    lines = [l for l in capsys.readouterr().out.splitlines() if l.strip()]
    assert len(lines) == 1
    rec = json.loads(lines[0])
    assert KEYS <= set(rec)
    assert rec["metric"] == "classes indexed/sec" and rec["n_gpus"] == 1 and rec["steps"] == 2
    assert rec["value"] > 0 and rec["higher_is_better"] is True and rec["scaling"] == "weak"
    assert rec["config"]["global_batch"] == 40 and rec["extra"]["classesPerRepo"] == 41
    assert rec["extra"]["graphQueryMs"]["p50"] > 0


@pytest.mark.timeout(600)
def test_bench_two_ranks_gloo():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
           "--steps", "1", "--warmup", "1", "--classes", "30", "--queries", "6"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=540)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["global_batch"] == 60
    assert rec["config"]["parallelism"].startswith("dp2") and rec["value"] > 0


def test_enrich_pool_extra_deals_one_project_over_every_worker(tmp_path):
    """extra.enrichLocalPool (the production layout: ONE project, ONE pool,
    one worker per GPU), rehearsed with model-free echo workers on the CPU:
    every class enriched, each worker got a share."""
    import bench
    from dmcp.enrich.workers import GpuWorkerPool
    args = bench.parse_args(["--pool-classes", "40"])
    pool = GpuWorkerPool(["cpu"] * 3, {"preset": "echo", "step_s": 0.01, "steps": 1, "max_batch": 64},
                         init=False, start_timeout_s=120)
    try:
        rec = bench._enrich_pool(pool, args, str(tmp_path))
    finally:
        pool.close()
    assert rec["classes"] == 41 and rec["enriched"] == 41 and rec["workers"] == 3
    assert rec["classesPerSec"] > 0 and len(rec["classesPerWorker"]) == 3
    assert all(v > 0 for v in rec["classesPerWorker"].values())
