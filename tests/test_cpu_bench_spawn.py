"""bench.py's multi-rank path on CPU: `--gpus N` without an external launcher spawns
N rank processes itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set before any GPU use), checks
the world size, shards frames with frame_range, times steps between barriers with the max over
ranks (all_reduce), gathers the frames in order to rank 0 and relays rank 0's one JSON line.
--dry-run replaces the HIP chain by placeholder frames on gloo."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _bench(*args, env=None):
    e = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR",
                                                           "MASTER_PORT")}
    e.update(env or {})
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True,
                          timeout=240, env=e)


@pytest.mark.parametrize("n,frames", [(2, 4), (3, 5)])
def test_bench_spawns_n_ranks(n, frames):
    r = _bench("--gpus", str(n), "--dry-run", "--frames", str(frames), "--steps", "3", "--warmup", "1")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout               # exactly one JSON line, from rank 0
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["world_size_verified"] and d["launcher"] == "bench.py spawn"
    assert d["gather_in_order"]
    # contiguous shards covering every frame once (frame_range)
    seen = [f for first, cnt in d["shards"] for f in range(first, first + cnt)]
    assert seen == list(range(n * frames))


def test_bench_single_rank_unchanged():
    r = _bench("--gpus", "1", "--dry-run", "--steps", "2", "--warmup", "1")
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["n_gpus"] == 1 and d["launcher"] == "single process"


def test_bench_rejects_world_mismatch():
    """under an external launcher WORLD_SIZE must equal --gpus"""
    r = _bench("--gpus", "2", "--dry-run", env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def test_bench_rank_failure_fails_fast():
    """a rank that dies at init ends the whole run: the parent polls every rank, terminates the
    survivors (blocked in init_process_group / the first barrier) and exits non-zero"""
    import time
    t0 = time.monotonic()
    r = _bench("--gpus", "3", "--dry-run", "--fail-rank", "1", "--steps", "2", "--warmup", "1")
    dt = time.monotonic() - t0
    assert r.returncode != 0, r.stdout
    assert "rank exit codes" in r.stderr and "--fail-rank" in r.stderr
    assert dt < 30, dt
    assert not r.stdout.strip()                    # no JSON line from a failed run


@pytest.mark.parametrize("n,streams", [(2, 2), (3, 1)])
def test_bench_spawn_stream_sharding(n, streams):
    """`--shard streams` (SURVEY 8(e)'s independent-stream mode): every rank encodes its own TS streams
    (seeds r S + 1 .. r S + S, bench.shard_plan), disjoint and together complete, with no data-path
    collective; timing max-reduced over ranks as for frame sharding"""
    r = _bench("--gpus", str(n), "--dry-run", "--shard", "streams", "--streams", str(streams), "--frames",
               str(4 * streams), "--steps", "2", "--warmup", "1")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["shard"] == "streams" and d["n_gpus"] == n and d["world_size_verified"]
    assert d["seeds_disjoint_complete"] and d["frames_ok"]
    assert d["stream_seeds"] == [list(range(k * streams + 1, k * streams + streams + 1)) for k in range(n)]


def test_shard_plan_modes():
    sys.path.insert(0, str(ROOT))
    import bench
    # frames: disjoint contiguous batches across ranks and the R resident batches
    seen = []
    for rank in range(3):
        for first, cnt, seeds in bench.shard_plan("frames", 8, 2, 2, rank, 3):
            assert seeds == [1, 2] and cnt == 4
            seen += list(range(first, first + cnt))
    assert sorted(seen) == list(range(24)) and len(set(seen)) == 24
    assert bench.shard_plan("streams", 6, 3, 2, 1, 2) == [(0, 2, [4, 5, 6]), (2, 2, [4, 5, 6])]
    with pytest.raises(SystemExit):
        bench.shard_plan("frames", 5, 2, 2, 0, 1)
