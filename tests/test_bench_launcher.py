"""bench.py's multi-rank plumbing without a device: `--gpus N` with no launcher environment
starts N rank processes itself (torch.distributed.run on 127.0.0.1), the ranks join one group,
the line reports the number of ranks that joined as n_gpus, and rank 0 still times the CPU
baseline.  `--dry-run` replaces the GPU step by a no-op (gloo)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _line(out):
    return json.loads([l for l in out.splitlines() if l.startswith("{")][-1])


def test_gpus2_spawns_two_ranks_with_cpu_baseline():
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run", "--steps", "5",
                        "--warmup", "1", "--cpu-budget", "0.3"], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    d = _line(p.stdout)
    assert d["n_gpus"] == 2 and d["dry_run"] is True
    assert d["config"]["parallelism"] == "replicas x2"
    cb = d["cpu_baseline"]
    assert cb and cb["value"] > 0 and cb["kind"] == "port" and cb["cores"] >= 1


def test_single_rank_dry_run():
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--steps", "3", "--no-cpu"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    d = _line(p.stdout)
    assert d["n_gpus"] == 1 and d["cpu_baseline"] is None


def test_gpus2_sharded_c5_line_carries_cpu_baseline():
    """a two-rank sharded line (configs[4], --workload c5) carries the
    CPU baseline too — rank 0 scans every rank's rows on the host (the dry run: a small index
    in two shards)."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run", "--workload", "c5",
                        "--steps", "3", "--warmup", "1", "--cpu-budget", "0.3"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    d = _line(p.stdout)
    assert d["n_gpus"] == 2 and d["scaling"] == "strong"
    assert d["config"]["parallelism"] == "rows sharded x2"
    cb = d["cpu_baseline"]
    assert cb and cb["value"] > 0 and "2 shards" in cb["sample"]
