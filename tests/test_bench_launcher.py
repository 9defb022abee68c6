"""bench.py's multi-GPU launcher on the CPU (no GPU, no library): `--gpus N` without a launcher starts N rank
processes with the torch.distributed.run environment, a WORLD_SIZE that disagrees with --gpus is an error, and a
node with fewer GPUs than --gpus fails loudly instead of printing a 1-GPU line."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env.update(kw)
    return env


def _run(args, env, timeout=180):
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_flag_starts_n_ranks(n):
    r = _run(["--gpus", str(n), "--plumbing-check", "--points", "2000"], _env())
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints the one line
    d = json.loads(lines[0])
    assert d["world"] == n and d["group_size"] == n and d["gpus_flag"] == n
    assert d["allreduce"] == n * (n + 1) / 2  # every rank joined the group with its own RANK
    # strong scaling: the metric's 2000-point window split p % N == rank, every point on exactly one rank
    assert sum(d["strong_shard_points"]) == 2000 and max(d["strong_shard_points"]) - min(d["strong_shard_points"]) <= 1


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "2", "--plumbing-check"], _env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"))
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in (r.stderr + r.stdout)


def test_too_few_gpus_fails_loudly():
    # this container has no GPU: --gpus 2 must exit non-zero before starting any rank, not print an n_gpus: 1 line
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--no-cpu"], _env())
    assert r.returncode != 0
    assert "visible GPUs" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_single_gpu_workloads_reject_gpus():
    r = _run(["--workload", "track", "--gpus", "2"], _env())
    assert r.returncode != 0 and "single-GPU" in (r.stderr + r.stdout)


def test_count_gpus_reads_the_kfd_topology(tmp_path, monkeypatch):
    """The launcher counts GPUs from the KFD topology (nodes with SIMDs), narrowed by the visibility variables,
    without loading a HIP library."""
    sys.path.insert(0, ROOT)
    import bench
    for i, simds in enumerate([0, 1024, 1024, 1024]):  # node 0: the CPU
        d = tmp_path / str(i)
        d.mkdir()
        (d / "properties").write_text(f"cpu_cores_count {0 if simds else 64}\nsimd_count {simds}\narray_count 32\n")
    for v in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    assert bench.count_gpus(str(tmp_path)) == 3
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,2")
    assert bench.count_gpus(str(tmp_path)) == 2
    assert bench.count_gpus(str(tmp_path / "absent")) == 0
