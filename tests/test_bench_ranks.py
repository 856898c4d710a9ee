"""bench.py's multi-rank path: `bench.py --gpus N` without a
launcher starts N ranks under torch.distributed.run, every rank binds its device before the
process group exists, and the per-epoch merge inside the timed region leaves rank 0 with the
node total.  On CPU the ranks run the engine's CPU backend over gloo (world 2, 127.0.0.1);
the `gpu` case runs the gfx950 path with two ranks sharing cuda:0 over gloo.  --check-merge
compares rank 0's merged state with one engine fed every rank's batch, bit for bit."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, timeout=600, env_extra=None):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=timeout,
                       env=env, cwd=ROOT)
    return p


def _line(p):
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]  # rank 0 prints the only line
    return json.loads(lines[0])


@pytest.mark.parametrize("config,records", [("c3", 200_000), ("c4-remote", 200_000)])
def test_two_rank_cpu_backend_merge(config, records):
    p = _run(["--gpus", "2", "--backend", "gloo", "--cpu-backend", "--config", config, "--records", str(records),
              "--steps", "2", "--warmup", "1", "--check-merge", "--settle-ms", "0", "--no-scrape"])
    d = _line(p)
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["steps"] == 2
    assert d["config"]["parallelism"].startswith("dp2")
    assert d["value"] == pytest.approx(2 * records * 2 * 1000.0 / (d["ms_per_step"] * 2))
    mc = d["merge_check"]
    assert mc["equal"] and mc["series_equal"] and mc["ranks"] == 2 and mc["series"] > 0, mc
    if config == "c3":
        assert mc["cms_equal"] and mc["hll_equal"]
    assert d["merge_ms"] is not None and d["merge_ms"] > 0


def test_world_mismatch_refused():
    """--gpus must agree with the launcher's world size."""
    p = _run(["--gpus", "2", "--cpu-backend", "--backend", "gloo", "--records", "1000"],
             env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and "WORLD_SIZE=1" in p.stderr


def test_rank_device_mapping():
    sys.path.insert(0, ROOT)
    import bench
    assert [bench.rank_device(r, 8, "nccl", 8) for r in range(8)] == list(range(8))
    assert [bench.rank_device(r, 2, "gloo", 1) for r in range(2)] == [0, 0]
    with pytest.raises(SystemExit):
        bench.rank_device(1, 2, "nccl", 1)  # RCCL: one GPU per rank
    with pytest.raises(SystemExit):
        bench.rank_device(0, 1, "nccl", 0)


@pytest.mark.gpu
def test_two_rank_gpu_bench_merge(gpu_device):
    """The driver's scaling command shape on one GPU: two gfx950 ranks (gloo, sharing cuda:0)."""
    p = _run(["--gpus", "2", "--backend", "gloo", "--config", "c3", "--records", "2000000", "--steps", "3",
              "--warmup", "1", "--check-merge", "--settle-ms", "0", "--no-scrape"], timeout=300)
    d = _line(p)
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert d["merge_check"]["equal"], d["merge_check"]
    assert d["roofline"]["kernel"]  # the gfx950 kernels ran
