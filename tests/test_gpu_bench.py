"""bench.py's data paths on the GPU (one MI355X): the N>1 paths -- shard slab,
gather through the process group (backend nccl = RCCL), device re-assembly;
or every rank writing into rank 0's image mapped with HIP IPC -- taken at
world size 1 (`--force-dist`) or with N ranks on the one GPU must give the
frames of the single-GPU path bit for bit, and stdout must hold exactly the
one JSON line (RCCL prints a version banner to fd 1 at communicator init)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--config", "config1", "--steps", "4", "--warmup", "1", "--frames-per-launch", "2",
        "--no-cpu-baseline", "--reuse-steps", "0", "--cull-steps", "0", "--check"]


def _bench(*extra, rc=0):
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *ARGS, *extra],
                       cwd=ROOT, capture_output=True, text=True, timeout=100)
    assert (p.returncode == 0) == (rc == 0), (p.returncode, p.stderr[-2000:])
    lines = p.stdout.splitlines()
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


def _cross_ok(b, n, path):
    """The N>1 line's own pixel check: rank 0 re-rendered the first, middle
    and last row of every rank's shard and found them bit-exact in its image."""
    c = b["cross_rank_check"]
    assert c["bit_exact"] is True and c["mismatched"] == [], c
    assert b["ranks"]["cross_rank_rows_bit_exact"] is True
    assert c["path"] == path and c["ranks_covered"] == n and c["rows_checked"] >= 2 * n
    assert len(b["ranks"]["peer_access"]) == n


@pytest.mark.gpu
@pytest.mark.parametrize("gather", ["rccl", "ipc"])
def test_rccl_gather_path_matches_single_gpu(gather):
    """--force-dist at world 1: the RCCL gather + device re-assembly, and the
    image-layout path (RT_FLAG_IMAGE_OUT into rank 0's own image)."""
    a = _bench()
    b = _bench("--force-dist", "--dist-backend", "nccl", "--gather", gather)
    assert a["config"]["parallelism"] == "single GPU"
    assert ("RCCL gather" if gather == "rccl" else "rank 0's image") in b["config"]["parallelism"]
    assert a["check"] == b["check"] and len(a["check"]) == 2  # the last launch's frames
    assert a["segments_per_frame"] == b["segments_per_frame"]
    assert "cross_rank_check" not in a
    _cross_ok(b, 1, gather if gather == "ipc" else "gather")


@pytest.mark.gpu
@pytest.mark.parametrize("n,gather", [(2, "rccl"), (3, "rccl"), (2, "ipc"), (3, "ipc")])
def test_bench_launches_its_own_ranks(n, gather):
    """`python bench.py --gpus N` with no launcher around it (the driver's
    scaling command) starts the N ranks itself and relays rank 0's line; the
    frames (2-frame launches; 225 rows split unevenly) equal the single-GPU
    run's -- all ranks on the one GPU of this box, either gathered (host-staged
    gloo gather + rt_assemble_shard_frames) or written by every rank straight
    into rank 0's image mapped into it with HIP IPC (RT_FLAG_IMAGE_OUT)."""
    a = _bench()
    b = _bench("--gpus", str(n), "--same-device", "--dist-backend", "gloo", "--gather", gather)
    assert b["n_gpus"] == n and len(b["ranks"]["segments"]) == n
    assert sum(b["ranks"]["segments"]) // 4 == a["segments_per_frame"]  # 4 timed frames
    assert ("rank 0's image" in b["config"]["parallelism"]) == (gather == "ipc")
    assert a["check"] == b["check"]
    assert a["segments_per_frame"] == b["segments_per_frame"]
    _cross_ok(b, n, "ipc" if gather == "ipc" else "gather")
    # every rank on the one device: no peer pairs to query
    assert all(v is None for row in b["ranks"]["peer_access"] for v in row)


@pytest.mark.gpu
@pytest.mark.parametrize("gather", ["rccl", "ipc"])
def test_cross_rank_check_catches_a_stale_shard(gather):
    """Fault injection: rank 1 renders but writes no output (knob
    skip_collect), so its rows of rank 0's image are whatever the buffer held.
    The N>1 line must say so -- cross_rank_rows_bit_exact false, rank 1's rows
    named, rank 0's own rows fine -- and the run must exit non-zero."""
    b = _bench("--gpus", "2", "--same-device", "--dist-backend", "gloo", "--gather", gather,
               "--debug-skip-collect-rank", "1", rc=4)
    c = b["cross_rank_check"]
    assert c["bit_exact"] is False and b["ranks"]["cross_rank_rows_bit_exact"] is False
    assert {k for k, _, _ in c["mismatched"]} == {1}
    assert len(c["mismatched"]) == sum(1 for k, _ in c["rows"] if k == 1)


@pytest.mark.gpu
def test_bench_line_carries_the_contract_fields():
    """The driver-facing line (small run of the default config shape on
    config 1, a 2-row CPU sample): every contract key, the roofline block and
    the CPU baseline, with self-consistent numbers."""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "config1",
                        "--steps", "2", "--warmup", "1", "--frames-per-launch", "2",
                        "--reuse-steps", "0", "--cull-steps", "0", "--cpu-rows", "2"],
                       cwd=ROOT, capture_output=True, text=True, timeout=200)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = p.stdout.splitlines()
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
              "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1
    assert d["higher_is_better"] is True and d["value"] > 0 and "workload" in d["config"]
    rf = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in rf, k
    # SIMD issue from the committed PMC record (none for config 1: achieved,
    # peak and frac are null) and the metric's fp32 algorithm ratio beside it
    assert rf["bound"] == "SIMD issue" and rf["unit"] == "G SIMD-issue cycles/s"
    assert rf["frac"] is None or abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    assert rf["fp32_algorithm_ratio"] > 0 and rf["kernel_ms_per_launch"] > 0
    cb = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in cb, k
    assert cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] == "port"
    assert cb.get("gpu_rows_bit_exact") is True
    assert cb.get("segments_equal") is True and cb.get("gpu_shard_equals_headline") is True
