"""bench.py --gpus N launches its own ranks (the driver's scaling runs call it
without torchrun) and refuses to run on fewer GPUs than asked for."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


def _run(args, env=None, timeout=240):
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True,
                          env=env or _env(), timeout=timeout)


@pytest.mark.parametrize("world", [2, 3])
def test_launcher_spawns_ranks(world):
    r = _run(["--gpus", str(world), "--dry-run", "--records", "1000"])
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1  # only rank 0 prints
    out = json.loads(lines[0])
    assert out["dry_run"] and out["ranks"] == world
    shards = sorted(out["shards"])
    assert [s[0] for s in shards] == list(range(world))          # distinct RANKs
    assert len({s[3] for s in shards}) == world                   # distinct processes
    assert [(s[1], s[2]) for s in shards] == [(1000 * r, 1000) for r in range(world)]  # disjoint


def test_launcher_refuses_missing_gpus():
    import torch
    want = max(2, torch.cuda.device_count() + 1)
    r = _run(["--gpus", str(want), "--records", "10"])
    assert r.returncode != 0
    assert f"needs {want} GPUs" in r.stderr


def test_world_size_must_match():
    r = _run(["--gpus", "1", "--records", "10"], env=_env(WORLD_SIZE="2", RANK="0"))
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr


def test_default_line_legs():
    """--legs: the default 1M Large encdec line carries configs[1] (small),
    configs[3] (mixed_encode) and the README's Medium and XLarge shapes
    (north_star: all four shapes on the driver's line); other lines none
    unless asked; 'none' and unknown legs (no GPU needed: argument handling
    only)."""
    sys.path.insert(0, ROOT)
    import bench
    assert bench.legs_of(bench.parse_args([])) == ["small", "mixed_encode", "medium", "xlarge"]
    assert bench.legs_of(bench.parse_args(["--legs", "none"])) == []
    assert bench.legs_of(bench.parse_args(["--shape", "small"])) == []
    assert bench.legs_of(bench.parse_args(["--records", "1000"])) == []
    assert bench.legs_of(bench.parse_args(["--mode", "decode"])) == []
    assert bench.legs_of(bench.parse_args(["--shape", "medium", "--legs", "small"])) == ["small"]
    with pytest.raises(SystemExit):
        bench.legs_of(bench.parse_args(["--legs", "small,bogus"]))
    # the legs' configurations: Small / Medium encode + decode, Mixed encode
    # only, XLarge encode + decode of 1/16 the records (64 K) + its zero copy
    assert bench.LEG_SHAPES == {"small": ("small", False, 1, False), "mixed_encode": ("mixed", True, 1, False),
                                "medium": ("medium", False, 1, False), "xlarge": ("xlarge", False, 1 / 16, True)}
    # the order: host path first (a fresh device), the legs right after the
    # main line and before the decode legs' 207 GB records arena
    a = bench.parse_args([])
    assert (a.host_path_at, a.legs_at) == ("first", "after_main")


@pytest.mark.gpu
def test_two_ranks_rehearsal_on_one_gpu():
    """The N > 1 branch of the line (barriers, max over ranks, the all-ranks
    totals, the host path on every rank, the scatter leg and its per-rank
    parse, two shape legs, the decode legs' aggregates) run end to end by two
    ranks on one GPU (--shared-gpu: gloo instead of RCCL, which refuses two
    ranks on one device); every rank's records verified. The timing is not a
    measurement."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    r = _run(["--gpus", "2", "--shared-gpu", "--shape", "small", "--records", "8192", "--steps", "2",
              "--warmup", "1", "--no-cpu-baseline", "--legs", "small,mixed_encode"], timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["verified"] is True
    assert out["config"]["records_per_gpu"] == 8192
    assert out["scatter"]["verified"] is True and out["scatter"]["bytes_sent_by_rank0"] > 0
    assert out["decode"]["verified"] is True and out["decode"]["all_ranks"]["ranks"] == 2
    # the line's order as the driver runs it: host path first, the shape legs
    # right after the main line, then the decode legs; every collective of
    # each leg reached by both ranks
    assert out["host_path"]["all_ranks"]["ranks"] == 2 and out["host_path"]["rows_match"] is True
    assert set(out["legs"]) == {"small", "mixed_encode"}
    assert all(leg["verified"] is True for leg in out["legs"].values())
    assert out["legs_order"] == "after the main line, before the decode legs"
