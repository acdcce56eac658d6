#!/usr/bin/env python3
"""Headline benchmark: Mrays/s + % fp32 roofline, RTIOW final scene 1920x1080 @64spp.

One step = one frame of the hot path: every pixel x spp paths
through the persistent HIP kernel, depth 16, written to an HBM image. Inputs
(scene, camera) are resident on the device before timing starts.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config rtiow1080]

N > 1 runs one process per GPU under torch.distributed.run; a bare
`python bench.py --gpus N` (no WORLD_SIZE in the environment) launches that
itself as a child process before touching the GPU and relays rank 0's line. The image
is row-tiled in blocks dealt serpentine to the ranks; rank 0's
image is mapped into every rank (HIP IPC) and each rank's collect writes its
rows straight into it over xGMI (RT_FLAG_IMAGE_OUT) -- or, if the mapping
fails on some rank, one RCCL gather lands the shards on rank 0, which
re-assembles the image on the device (--gather). Timing: barrier + synchronize around exactly K steps,
max over ranks. value = algorithmic ray segments of the whole frame (all ranks)
per second, every segment traced (primary-hit reuse off for the headline;
its frame time is reported separately as `primary_reuse`).

Roofline: SIMD issue, the resource the kernel executes on:
the render kernel's issue cycles per launch, MEASURED from the rocprofv3 PMC
record of the workload (profiles/pmc_traffic.json, tools/pmc_summary.py):
4 x (SQ_ACTIVE_INST_VALU - SQ_ACTIVE_INST_VALU2) -- the quad-cycles the VALU
issue port was held, gfx950's dual-issued pairs counted once -- + 4 x
SQ_INSTS_MFMA (an MFMA holds the issue 8 cycles), scaled per frame to this
run's launch, over that launch's duration (HIP events
on the stream the kernel runs on), against 1024 SIMDs x this run's own shader
clock (rt_stats.clock_ghz, measured inside the timed launches); the line's
`formula` and `peak_formula` fields say the same. The metric's fp32 roofline
(the reference's 18 x N_spheres fp32 flops per segment over 157.3 TF) is kept
as `fp32_algorithm_ratio`: the kernel runs the brute-force walk's filter as
f16 MFMA tiles and the exact fp32 test only on candidates, so that ratio
exceeds 1. Matrix pipe, VALU busy and HBM traffic come from the same record.
At N > 1 a rank renders a row shard, for which no PMC record exists: its issue
cycles and traffic are the whole-frame record scaled by the rank's pixel share
-- a MODEL, not a measurement, and the line says so
(`roofline.record_scaled_by_pixel_share`, `roofline.modelled`).

N > 1 self-check: after the timed region rank 0 re-renders the first, middle
and last row of every rank's shard of the timed frame on its own GPU and
compares them bit for bit with the rows the ranks delivered into its image
(`cross_rank_check`, `ranks.cross_rank_rows_bit_exact`); a mismatch exits
non-zero. `ranks.peer_access` records hipDeviceCanAccessPeer per rank pair.

cpu_baseline: the C oracle (oracle/, a scalar port of the WGSL) timed on this
host on a bounded row sample of the same frame, rank 0 at N=1 only.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from bevy_raytrace_amd import abi  # noqa: E402
from bevy_raytrace_amd.camera import default_camera_block  # noqa: E402
from bevy_raytrace_amd.configs import HEADLINE, WORKLOADS, pick_row_block  # noqa: E402

METRIC = "Mrays/s + % fp32 roofline, RTIOW final scene 1920×1080 @64spp, 1/2/4/8 GPU"
PEAK_FP32_TFLOPS = 157.3
PEAK_F16_DENSE_TFLOPS = 2500.0  # MI355X_MICROARCH.md MFMA table, BF16/F16 dense
FLOPS_PER_SPHERE_TEST = 18  # intersect.wgsl:97-102, SURVEY §8d


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=24)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--config", default=HEADLINE, choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-rows", type=int, default=0,
                    help="rows of the frame in the CPU sample (0 = auto, ~10 s)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL over xGMI, the product path); gloo = host-staged "
                         "gather, for rehearsing N>1 on a one-GPU box")
    ap.add_argument("--same-device", action="store_true",
                    help="every rank on cuda:0 (rehearsal with --dist-backend gloo)")
    ap.add_argument("--gather", default="auto", choices=["auto", "ipc", "rccl"],
                    help="N>1: ipc = rank 0's image mapped into every rank (HIP IPC), each "
                         "rank writing its rows straight into it (RT_FLAG_IMAGE_OUT: no "
                         "gather, no re-assembly); rccl = one gather of the shard slabs to "
                         "rank 0 and a device re-assembly; auto = ipc, else rccl if "
                         "mapping fails on any rank")
    ap.add_argument("--check", action="store_true",
                    help="add a checksum of the assembled frames to the JSON line")
    ap.add_argument("--no-cross-check", action="store_true",
                    help="N>1: skip the cross-rank row check (by default rank 0 re-renders the "
                         "first, middle and last row of every rank's shard of the timed run's "
                         "frame and compares them bit for bit with its image; a mismatch "
                         "exits non-zero)")
    ap.add_argument("--debug-skip-collect-rank", type=int, default=-1, metavar="K",
                    help="fault injection: rank K's calls write no output (knob skip_collect), "
                         "so its rows in rank 0's image stay stale; the cross-rank check must fail")
    ap.add_argument("--force-dist", action="store_true",
                    help="take the N>1 path (process group, shard gather, assembly) "
                         "even at world size 1")
    ap.add_argument("--frames-per-launch", type=int, default=24,
                    help="frames per persistent launch (rt_render_frames_device)")
    ap.add_argument("--reuse-steps", type=int, default=4,
                    help="extra frames timed with primary-hit reuse on (0 = skip)")
    ap.add_argument("--cull-steps", type=int, default=-1,
                    help="extra frames timed with the culled list, RT_FLAG_CULL (0 = skip; "
                         "default 12 at N=1, skipped at N>1)")
    ap.add_argument("--shim-frames", type=int, default=120,
                    help="--config reference1080: frames timed through the Bevy shim's call "
                         "sequence (rt_wait, dirty check, rt_render_async into a host buffer)")
    ap.add_argument("--lib", default=None,
                    help="A/B only: another build of librt_hip.so (same ABI), e.g. a previous "
                         "round's, to compare on one box")
    ap.add_argument("--tune", action="append", default=[], metavar="KNOB=VALUE",
                    help="A/B only: set a library knob (rt_debug_tune; the defaults are the "
                         "product), e.g. --tune wg_per_cu=6")
    return ap.parse_args()


def load_pmc(workload_key):
    """The committed rocprofv3 PMC record of the render kernel for this
    workload (profiles/pmc_traffic.json, tools/pmc_round.sh +
    tools/pmc_summary.py): HBM bytes and the VALU counters of one launch of
    `frames_per_launch` frames, measured in separate --pmc passes."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            return json.load(f).get(workload_key)
    except (OSError, ValueError):
        return None


def load_traffic(e, frames_per_launch):
    """HBM bytes per render launch from the PMC record, scaled per frame to
    this run's average launch (block sums and tail samples are per frame);
    at N > 1 `frames_per_launch` carries the rank's pixel share too."""
    try:
        return int(e["hbm_bytes_per_launch"] / e["frames_per_launch"] * frames_per_launch)
    except (TypeError, KeyError, ZeroDivisionError):
        return None


def load_executed(workload_key):
    """What the render kernel executes per frame of this workload
    (profiles/executed.json, tools/executed.py + tools/executed_summary.py:
    the RT_PROFILE build's counters of one bench-shaped launch)."""
    path = os.path.join(ROOT, "profiles", "executed.json")
    try:
        with open(path) as f:
            return json.load(f).get(workload_key)
    except (OSError, ValueError):
        return None


def executed_report(ex, frames_per_launch):
    """The executed-work block of the roofline for one launch of this run
    (per-frame counts x frames x pixel share): tiles, MFMA flops, exact
    tests, shading, and the issue shares per phase."""
    if not ex:
        return None
    pf = ex.get("per_frame", {})
    out = {k: (round(v * frames_per_launch) if isinstance(v, (int, float)) else v)
           for k, v in pf.items()}
    for k in ("per_segment", "issue_model", "phase_wave_time_share", "useful_issue_fraction",
              "source", "note"):
        if k in ex:
            out[k] = ex[k]
    return out


def valu_report(e):
    """VALU busy of the render kernel from the PMC record, both forms (see
    tools/pmc_summary.py): AMD's VALUBusy prices every VALU instruction at 4
    cycles (one quad-cycle of SQ_ACTIVE_INST_VALU); the issue form prices
    32-bit integer ops at their measured 2 cycles (tools/ubench/valu_busy)."""
    v = (e or {}).get("valu")
    if not v:
        return None
    out = {"amd_valubusy": round(v["valubusy_amd"], 4), "amd_formula": v["formula_amd"]}
    if "valubusy_issue" in v:
        out["issue_weighted"] = round(v["valubusy_issue"], 4)
        out["issue_formula"] = v["formula_issue"]
    out["source"] = "profiles/pmc_traffic.json (rocprofv3 --pmc, one launch of %d frames)" % (
        e["frames_per_launch"])
    return out


def mfma_report(e):
    """The matrix-core filter's executed work from the PMC record (MFMA pass of
    tools/pmc_round.sh): f16 MFMA flops per launch and the matrix pipe's busy
    share of the SIMD cycles, against the dense f16 peak (MI355X_MICROARCH.md)."""
    m = (e or {}).get("mfma")
    v = (e or {}).get("valu") or {}
    if not m:
        return None
    out = {"mfma_f16_flops_per_launch": m["mfma_f16_flops"], "formula_flops": m["formula_flops"],
           "peak_f16_dense_tflops": PEAK_F16_DENSE_TFLOPS}
    kms = v.get("kernel_ms_under_pmc")
    if kms:
        tf = m["mfma_f16_flops"] / (kms * 1e-3) / 1e12
        out["mfma_f16_tflops_under_pmc"] = round(tf, 2)
        out["frac_f16_dense"] = round(tf / PEAK_F16_DENSE_TFLOPS, 4)
    if m.get("mfma_busy") is not None:
        out["mfma_busy"] = round(m["mfma_busy"], 4)
        out["formula_busy"] = m["formula_busy"]
    return out


def simd_issue_roofline(e, frames_per_launch, kms_launch, clock_run):
    """The bound the kernel runs against: SIMD issue. Issue
    cycles per launch from the PMC record (tools/pmc_summary.py; the
    instruction counts scale with the frames of a launch) over this run's
    launch time (HIP events on the kernel's stream) x this run's own shader
    clock (rt_stats.clock_ghz, measured inside the timed launches) x 1024
    SIMDs: frac = issue cycles / SIMD cycles of the run."""
    si = (e or {}).get("simd_issue")
    if not si:
        return {"bound": "SIMD issue", "achieved": None, "peak": None,
                "unit": "G SIMD-issue cycles/s", "frac": None, "clock_ghz_run": round(clock_run, 4),
                "note": "no PMC record for this workload in profiles/pmc_traffic.json"}
    cycles = si["issue_cycles_per_launch"] / e["frames_per_launch"] * frames_per_launch
    achieved = cycles / (kms_launch * 1e-3) / 1e9
    clock = clock_run if clock_run > 0 else si["clock_ghz"]
    peak = 1024 * clock
    issue = {k: si[k] for k in ("formula", "prices", "price_source", "valu_share", "mfma_share",
                                "busy", "clock_ghz", "kernel_ms_under_pmc") if k in si}
    issue["issue_cycles_per_launch"] = cycles
    issue["source"] = ("profiles/pmc_traffic.json (rocprofv3 --pmc, one launch of %d frames, "
                       "tools/pmc_round.sh)" % e["frames_per_launch"])
    return {"bound": "SIMD issue", "achieved": round(achieved, 1), "peak": round(peak, 1),
            "unit": "G SIMD-issue cycles/s", "frac": round(achieved / peak, 4),
            "clock_ghz_run": round(clock_run, 4),
            "peak_formula": "1024 SIMDs x clock_ghz_run (this run's in-kernel clock)",
            "issue": issue}


def shim_sequence(r, cam, spheres, mats, W, H, S, D, nframes, host_work_ms=1.0):
    """The Bevy shim's per-frame calls (bevy_shim/src/ray_trace_node.rs
    RayTraceNode::update, double-buffered): finish the frame enqueued last
    update (rt_wait), compare the packed scene bytes with the uploaded ones
    (the dirty check; nothing changes here), rt_render_async the next frame
    into the host buffer not on show. Timed per flag set into pageable host
    buffers (a Rust Vec<f32>), the same buffers after rt_host_register (what
    the shim does), page-locked torch buffers, and rt_render_device (no
    device-to-host copy), so the copy's share of a frame is measured, not
    assumed; then pageable vs registered again with `host_work_ms` of busy host
    work per frame standing in for the rest of Bevy's frame, which a
    registered buffer overlaps with the GPU's work and a pageable one cannot."""
    import torch
    sp_bytes, mt_bytes = spheres.tobytes(), mats.tobytes()
    out = {"frames": nframes, "spp": S, "max_depth": D, "host_work_ms": host_work_ms,
           "note": "per-frame latency of the drop-in path: the reference renders into its "
                   "texture on the device; the shim copies the Rgba32Float frame to the host "
                   "for Bevy's write_texture"}

    def busy(ms):
        t = time.perf_counter() + ms * 1e-3
        while time.perf_counter() < t:
            pass

    for fname, flags in (("brute", abi.RT_FLAG_NO_PRIMARY_CACHE), ("cull", abi.RT_FLAG_CULL)):
        r.reserve(1, W, H, S, D, flags=flags)
        res = {}
        # mode: host buffer kind, + renders kept in flight ("_1inflight": the
        # round-3 shim, one; otherwise RT_MAX_PENDING = 2, the shim now), +
        # busy host work per frame
        for mode in ("pageable_1inflight", "registered", "registered_1inflight", "pinned",
                     "device", "device_1inflight", "pageable_1inflight+host_work",
                     "registered+host_work", "registered_1inflight+host_work"):
            base = mode.split("+")[0].replace("_1inflight", "")
            depth = 1 if "_1inflight" in mode else abi.RT_MAX_PENDING
            work = host_work_ms if mode.endswith("host_work") else 0.0
            nbuf = depth + 1  # the shown frame + the ones in flight
            if base in ("pageable", "registered"):
                bufs = [np.empty((H, W, 4), np.float32) for _ in range(nbuf)]
                if base == "registered":
                    for b in bufs:
                        r.host_register(b)
            elif base == "pinned":
                bufs = [torch.empty((H, W, 4), dtype=torch.float32, pin_memory=True).numpy()
                        for _ in range(nbuf)]
            else:
                bufs = [torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
                        for _ in range(nbuf)]
            calls, stats = [], []
            pending, ready, t0 = [], None, 0.0  # pending: (buffer, frame0) oldest first
            shown = None
            for f in range(nframes + 8):  # 8 untimed frames first
                if f == 8:
                    torch.cuda.synchronize()
                    calls, stats, t0 = [], [], time.perf_counter()
                while len(pending) >= depth:  # step 1: rt_wait for the oldest frame
                    stats.append(r.wait())
                    ready, shown = pending.pop(0)
                dirty = spheres.tobytes() != sp_bytes or mats.tobytes() != mt_bytes  # step 2
                assert not dirty
                i = next(k for k in range(nbuf)
                         if k != ready and all(k != p for p, _ in pending))
                tc = time.perf_counter()
                if base == "device":
                    r.render_device(cam, bufs[i].data_ptr(), W, H, S, D, frame0=f, flags=flags)
                else:
                    r.render_async(cam, bufs[i], W, H, S, D, frame0=f, flags=flags)
                calls.append(time.perf_counter() - tc)
                pending.append((i, f))
                busy(work)  # the rest of the app's frame
            while pending:
                stats.append(r.wait())
                ready, shown = pending.pop(0)
            dt = time.perf_counter() - t0
            # the last frame the sequence delivered, against a plain render of it
            last = (bufs[ready].cpu().numpy() if base == "device" else np.array(bufs[ready]))
            ref, _ = r.render(cam, W, H, S, D, frame0=shown, flags=flags)
            exact = bool(np.array_equal(last, ref, equal_nan=True))
            if base == "registered":
                for b in bufs:
                    r.host_unregister(b)
            segs = float(np.mean([s["segments"] for s in stats]))
            res[mode] = {"frame_interval_ms": round(dt / nframes * 1e3, 4),
                         "fps": round(nframes / dt, 1), "in_flight": depth,
                         "enqueue_call_ms": round(float(np.mean(calls)) * 1e3, 4),
                         "gpu_total_ms": round(float(np.mean([s["total_ms"] for s in stats])), 4),
                         "kernel_ms": round(float(np.mean([s["kernel_ms"] for s in stats])), 4),
                         "mrays_per_s": round(segs / (dt / nframes) / 1e6, 1),
                         "last_frame_bit_exact": exact}
        dev = res["device_1inflight"]["gpu_total_ms"]
        for mode in ("pageable_1inflight", "registered_1inflight", "pinned"):
            d2h = res[mode]["gpu_total_ms"] - dev
            res[mode]["d2h_ms"] = round(d2h, 4)
            res[mode]["d2h_share_of_frame"] = round(d2h / res[mode]["frame_interval_ms"], 4)
        out[fname] = res
    return out


def spawn_ranks(args):
    """`--gpus N` (N > 1) without a torch.distributed launcher around us: run
    N ranks as a CHILD `python -m torch.distributed.run` (never an exec: this
    process may not replace itself once anything touched the GPU, and nothing
    has yet), relay rank 0's JSON line and exit with the launcher's status."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, env=env)
    line = None
    for raw in proc.stdout.decode(errors="replace").splitlines():
        t = raw.strip()
        if t.startswith("{") and '"metric"' in t:
            line = t
        elif t:
            print(t, file=sys.stderr)
    if proc.returncode == 0 and line is None:
        print("bench.py: no result line from rank 0", file=sys.stderr)
        return 3
    if line is not None:
        print(line, flush=True)
    return proc.returncode


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    # stdout carries exactly the one JSON line: libraries that print to fd 1
    # (RCCL's version banner at communicator init, HIP runtime notes) are sent
    # to stderr; the result is written to the saved stdout at the end.
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; using the launcher's "
              f"{world} ranks", file=sys.stderr)
    if args.same_device:
        local = 0
    # --force-dist at world 1: the N>1 data path (shard slab, gather through the
    # process group, device re-assembly) on one process, e.g. to exercise the
    # RCCL gather on a one-GPU box
    dist_on = world > 1 or args.force_dist
    if dist_on and world == 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    red_dev = "cuda" if args.dist_backend == "nccl" else "cpu"  # scalar reductions
    torch.cuda.set_device(local)
    if dist_on:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    from bevy_raytrace_amd.renderer import Renderer

    wl = WORKLOADS[args.config]
    sc = wl.make_scene()
    spheres, mats = sc.objects_gpu(), sc.materials_gpu()
    nsph = len(spheres)
    cam = default_camera_block()
    W, H, S, D = wl.width, wl.height, wl.spp, wl.max_depth
    B = pick_row_block(H, world)
    rows = abi.shard_rows(H, B, world, rank)
    max_rows = max(len(abi.shard_rows(H, B, world, k)) for k in range(world))

    r = Renderer(local, lib_path=args.lib)
    for kv in args.tune:
        r.tune(*kv.split("=", 1))
    if rank == args.debug_skip_collect_rank:
        r.tune("skip_collect", 1)
    # every rank's device and whether it can reach every other rank's device
    # (hipDeviceCanAccessPeer; None = the same device, a one-GPU rehearsal)
    peer_access = None
    if dist_on:
        from bevy_raytrace_amd import distributed as rdist
        devs = [None] * world
        dist.all_gather_object(devs, local)
        mine = [rdist.can_access_peer(local, d) for d in devs]
        peer_access = [None] * world
        dist.all_gather_object(peer_access, mine)
    r.set_scene(spheres, mats)
    # work buffers of the largest launch this run makes, allocated before any
    # step (rt_reserve) so no allocation lands inside a timed region
    biggest = min(max(1, args.frames_per_launch),
                  max(args.steps, args.warmup, args.reuse_steps, args.cull_steps, 1))
    r.reserve(biggest, W, H, S, D, row_block=B, shard_count=world, shard_index=rank)
    # All device work of a step runs on ONE dedicated stream (non-null handle,
    # so the library enqueues on it rather than on its own stream).
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    # Frames per launch: consecutive frames (frame i = samples i*spp ...) go
    # through one persistent launch (rt_render_frames_device), so only the
    # launch -- not every frame -- pays the drain of its last waves.
    FPL = max(1, args.frames_per_launch)
    image = (torch.empty((FPL, H, W, 4), dtype=torch.float32, device="cuda")
             if rank == 0 else None)
    # N>1: rank 0's image mapped into every rank, unless the
    # mapping fails on some rank (then every rank takes the gather path)
    use_ipc, img_ptr, ipc_map, ipc_errors = False, None, None, None
    if dist_on and args.gather in ("auto", "ipc"):
        blob, err = None, None
        if rank == 0:
            try:
                blob = rdist.ipc_export(image.data_ptr())
            except Exception as e:  # noqa: BLE001 -- reported, then the gather path
                err = f"export: {e}"
                print(f"bench.py: IPC export failed: {e}", file=sys.stderr)
        objs = [blob]
        dist.broadcast_object_list(objs, src=0)
        ok = objs[0] is not None
        if ok and rank == 0:
            img_ptr = image.data_ptr()
        elif ok:
            try:
                ipc_map, img_ptr = rdist.ipc_import(objs[0])
            except Exception as e:  # noqa: BLE001
                err = f"open: {e}"
                print(f"bench.py: IPC import failed on rank {rank}: {e}", file=sys.stderr)
                ok = False
        # every rank's outcome (and error text) reaches rank 0's line
        res = [None] * world
        dist.all_gather_object(res, (ok, err))
        use_ipc = all(o for o, _ in res)
        ipc_errors = {str(k): e for k, (_, e) in enumerate(res) if e}
        if not use_ipc:
            if ipc_map is not None:
                rdist.ipc_close(ipc_map)
                ipc_map = None
            if args.gather == "ipc":
                raise RuntimeError("--gather ipc: mapping rank 0's image failed")
    # N=1: the single shard is the image; render straight into it.
    gather_path = dist_on and not use_ipc
    shard = image if not dist_on else (torch.empty((FPL, max_rows, W, 4), dtype=torch.float32,
                                                   device="cuda") if gather_path else None)
    gathered = (torch.empty((world, FPL, max_rows, W, 4), dtype=torch.float32, device="cuda")
                if (rank == 0 and gather_path) else None)
    # The library writes frame i of a launch at i * rows * W (this rank's own
    # row count); the gather needs equal slabs of max_rows. With uneven shards
    # (H not a multiple of B*world) a shorter rank renders into its own buffer
    # and copies each frame into the padded slab.
    packed = (torch.empty((FPL, len(rows), W, 4), dtype=torch.float32, device="cuda")
              if gather_path and len(rows) != max_rows else None)

    gather_events = []  # (start, end) CUDA events around each launch's gather + assembly

    def launch(first, nf, flags):
        """Enqueue frames [first, first + nf): render, then (N > 1) one RCCL
        gather of the nf shard slabs to rank 0 and the device re-assembly --
        or, with rank 0's image mapped, render the rank's rows straight into it."""
        if use_ipc:
            r.render_frames_device(cam, nf, img_ptr, W, H, S, D, first * S, B, world, rank,
                                   flags | abi.RT_FLAG_IMAGE_OUT, stream=stream.cuda_stream)
            return
        dst = shard if packed is None else packed
        r.render_frames_device(cam, nf, dst.data_ptr(), W, H, S, D, first * S, B, world, rank,
                               flags, stream=stream.cuda_stream)
        if packed is not None:
            shard[:nf, :len(rows)].copy_(packed[:nf])
        if dist_on:
            # rank k's nf frames land as slab k of a (world, nf, max_rows, W)
            # view, the layout rt_assemble_shard_frames reads: one assembly
            # launch for the launch's frames
            ev0 = torch.cuda.Event(enable_timing=True)
            ev0.record(stream)
            g = (gathered.view(-1)[:world * nf * max_rows * W * 4].view(world, nf, max_rows, W, 4)
                 if rank == 0 else None)
            if args.dist_backend == "nccl":
                dist.gather(shard[:nf], [g[k] for k in range(world)] if rank == 0 else None, dst=0)
            else:  # rehearsal: host-staged gather
                host = shard[:nf].cpu()
                parts = [torch.empty_like(host) for _ in range(world)] if rank == 0 else None
                dist.gather(host, parts, dst=0)
                if rank == 0:
                    for k in range(world):
                        g[k].copy_(parts[k])
            if rank == 0:
                r.assemble_shard_frames(g.data_ptr(), max_rows, nf, image.data_ptr(), W, H, B,
                                        world, stream=stream.cuda_stream)
            ev1 = torch.cuda.Event(enable_timing=True)
            ev1.record(stream)
            gather_events.append((ev0, ev1))

    def run(nsteps, flags):
        """nsteps frames in launches of <= FPL frames (near-equal sizes), two
        launches in flight on the one stream (the CPU enqueues launch j+1
        while j runs; the GPU never idles between them)."""
        nl = max(1, -(-nsteps // FPL))
        sizes = [nsteps // nl + (1 if j < nsteps % nl else 0) for j in range(nl)]
        stats, first, pending = [], 0, 0
        for nf in sizes:
            if pending == abi.RT_MAX_PENDING:
                stats.append(r.wait())
                pending -= 1
            launch(first, nf, flags)
            first += nf
            pending += 1
        while pending:
            stats.append(r.wait())
            pending -= 1
        return stats, sizes

    NO_REUSE = abi.RT_FLAG_NO_PRIMARY_CACHE

    if args.warmup > 0:
        run(args.warmup, NO_REUSE)

    def timed(nsteps, flags):
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        stats, sizes = run(nsteps, flags)
        torch.cuda.synchronize()
        if dist_on:
            dist.barrier()
        if use_ipc and rank == 0:
            # every rank's rows are in rank 0's image (system-scope
            # write-through stores, acknowledged before each collect wave
            # retires; each rank's launch complete before the barrier): the
            # acquire makes them visible to what rank 0 runs next
            r.acquire(stream.cuda_stream)
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if dist_on:
            t = torch.tensor([dt], dtype=torch.float64, device=red_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        return dt, stats, sizes

    gather_events.clear()
    dt, stats, sizes = timed(args.steps, NO_REUSE)
    gather_ms = sum(a.elapsed_time(b) for a, b in gather_events) if gather_events else 0.0
    # the timed headline run's first frame of its last launch, kept for the
    # parity check below before the reuse / cull runs overwrite the buffer
    head_idx = args.steps - sizes[-1]
    head_frame = image[0].clone() if rank == 0 else None
    # --check: the headline run's last launch's frames, hashed now (the reuse
    # and cull runs below render into the same buffer from frame 0 on)
    check = None
    if args.check and rank == 0:
        import hashlib
        check = {f"frame{head_idx + i}": hashlib.sha1(image[i].cpu().numpy().tobytes()).hexdigest()[:16]
                 for i in range(sizes[-1])}
    if dist_on:
        # on the IPC path the other ranks' next launch writes into rank 0's
        # image: none starts before rank 0 has copied (and hashed) the frames
        torch.cuda.synchronize()
        dist.barrier()
    segs_local = sum(s["segments"] for s in stats)
    traced_local = sum(s["traced_segments"] for s in stats)
    kms = [s["kernel_ms"] for s in stats]
    tot = torch.tensor([segs_local, traced_local], dtype=torch.float64, device=red_dev)
    if dist_on:
        dist.all_reduce(tot)
    segs_all, traced_all = float(tot[0].item()), float(tot[1].item())
    per_rank = None
    if dist_on:
        # per rank, over the timed steps: the render kernels (load balance of
        # the row tiling), the rest of the library calls (the pixel table and
        # the collect -- on the IPC path the collect's system-scope writes of
        # the rank's rows into rank 0's image, over xGMI), and on the gather
        # path the RCCL gather + re-assembly (CUDA events on the bench stream)
        call_ms = float(sum(s["total_ms"] for s in stats))
        mine = torch.tensor([float(sum(kms)), float(segs_local), call_ms, gather_ms, dt * 1e3],
                            dtype=torch.float64, device=red_dev)
        parts = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(parts, mine)
        per_rank = {"path": ("ipc" if use_ipc else
                             "rccl" if args.dist_backend == "nccl" else "gloo"),
                    "kernel_ms": [round(float(p[0].item()), 3) for p in parts],
                    "render_ms": [round(float(p[0].item()), 3) for p in parts],
                    "transfer_ms": [round(float(p[2].item() - p[0].item()) if use_ipc
                                          else float(p[3].item()), 3) for p in parts],
                    "call_ms": [round(float(p[2].item()), 3) for p in parts],
                    "wall_ms": [round(float(p[4].item()), 3) for p in parts],
                    "segments": [int(p[1].item()) for p in parts],
                    "peer_access": peer_access,
                    "ipc_errors": ipc_errors,
                    "note": ("render_ms: the rank's render kernels; transfer_ms: ipc -- its library "
                             "calls beyond the render (pixel table + collect writing its rows into "
                             "rank 0's image), rccl/gloo -- the gather + re-assembly; wall_ms: the "
                             "timed region on that rank before the max")}

    reuse = None
    if args.reuse_steps > 0:
        run(1, 0)
        rdt, rstats, _ = timed(args.reuse_steps, 0)
        reuse = {"frame_ms": round(rdt / args.reuse_steps * 1e3, 3),
                 "kernel_ms_per_frame": round(sum(s["kernel_ms"] for s in rstats)
                                              / args.reuse_steps, 3),
                 "traced_fraction": round(sum(s["traced_segments"] for s in rstats)
                                          / max(1, sum(s["segments"] for s in rstats)), 4),
                 "note": "RT_FLAG_NO_PRIMARY_CACHE off: the pixel-only primary hit is reused "
                         "across a sample block (bit-identical image)"}

    culled = None
    if args.cull_steps < 0:
        args.cull_steps = 12 if world == 1 else 0
    if args.cull_steps > 0:
        CULLF = NO_REUSE | abi.RT_FLAG_CULL
        run(min(args.cull_steps, FPL), CULLF)  # warm-up launch of the timed size
        cdt, cstats, csizes = timed(args.cull_steps, CULLF)
        csegs = torch.tensor([float(sum(s["segments"] for s in cstats))], dtype=torch.float64,
                             device=red_dev)
        if dist_on:
            dist.all_reduce(csegs)
        cval = float(csegs[0].item()) / cdt / 1e6
        culled = {"value": round(cval, 2), "unit": "Mrays/s",
                  "frame_ms": round(cdt / args.cull_steps * 1e3, 3),
                  "kernel_ms_per_launch": round(sum(s["kernel_ms"] for s in cstats)
                                                / max(1, sum(s["kernel_launches"] for s in cstats)), 3),
                  "launch_sizes": csizes,
                  "note": "RT_FLAG_CULL: spatially grouped list with conservative group bounds; "
                          "identical frames and segment counts, less filter work (no roofline: "
                          "the brute-force 18*N flops per segment are no longer all executed)"}

    if rank != 0:  # (all of its writes into rank 0's image completed in timed())
        if ipc_map is not None:
            from bevy_raytrace_amd import distributed as rdist
            rdist.ipc_close(ipc_map)
        if dist_on:
            dist.destroy_process_group()
        return

    value = segs_all / dt / 1e6
    ms_per_step = dt / args.steps * 1e3
    launches = sum(s["kernel_launches"] for s in stats)
    kernel_ms_total = float(sum(kms))
    # render launches: the average launch's algorithmic flops / its average
    # duration (HIP events on the stream the kernel runs on)
    flops_total = traced_local * FLOPS_PER_SPHERE_TEST * nsph
    achieved = flops_total / (kernel_ms_total * 1e-3) / 1e12
    pmc = load_pmc(wl.key)
    # the PMC and executed-work records are of whole frames on one GPU: a
    # rank of N renders its rows' share of every frame
    px_share = len(rows) / H
    fpl_eff = args.steps / max(1, len(sizes)) * px_share
    traffic = load_traffic(pmc, fpl_eff)
    kms_launch = kernel_ms_total / launches
    # the shader clock the timed launches ran at (rt_stats.clock_ghz: the
    # render waves' s_memtime ticks over their 100 MHz ticks), launch-time weighted
    clock_run = (sum(s["kernel_ms"] * s["clock_ghz"] for s in stats) / kernel_ms_total
                 if kernel_ms_total > 0 else 0.0)

    roofline = simd_issue_roofline(pmc, fpl_eff, kms_launch, clock_run)
    if px_share < 1.0:
        # no PMC record of a row shard: the whole frame's, scaled (a model)
        roofline["record_scaled_by_pixel_share"] = round(px_share, 6)
        roofline["modelled"] = True
    roofline.update({
        "executed": executed_report(load_executed(wl.key), fpl_eff),
        "traffic": traffic,
        # HBM GB/s of the render kernel: PMC bytes per launch / this run's
        # HIP-event launch time (peak ~8,000 GB/s: not the bound)
        "hbm_gbps": round(traffic / (kms_launch * 1e-3) / 1e9, 2) if traffic else None,
        "hbm_peak_gbps": 8000.0,
        "valu_busy": valu_report(pmc),
        "matrix_core": mfma_report(pmc),
        # the render kernel of this workload (rt_render_kernel: lists of <= 16
        # blocks; rt_render_multi_kernel: longer ones)
        "kernel": (pmc or {}).get("render_kernel", "rt_render_kernel"),
        "kernel_ms_per_launch": round(kms_launch, 3),
        # the metric's fp32 roofline, kept as a ratio: the reference
        # algorithm's 18 x N fp32 flops per traced segment at this rate over
        # the 157.3 TF fp32 peak -- above 1 because the kernel does not execute
        # them (the filter runs as f16 MFMA tiles, the exact fp32 test only on
        # candidates)
        "fp32_algorithm_tflops": round(achieved, 3),
        "fp32_algorithm_ratio": round(achieved / PEAK_FP32_TFLOPS, 4),
        "fp32_algorithm_basis": ("traced segments x 18 x N_spheres (intersect.wgsl:97-102, SURVEY "
                                 "8d) per render launch / its HIP-event duration, over 157.3 TF"),
    })

    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": f"synthetic: seeded RTIOW final scene ({nsph} spheres), camera (13,2,3)->0",
        "config": {"workload": f"{wl.key}: {W}x{H} {S}spp depth {D}, {nsph} spheres",
                   "width": W, "height": H, "spp": S, "max_depth": D, "spheres": nsph,
                   "frames_per_launch": FPL, "launch_sizes": sizes,
                   "parallelism": (f"row-tiled x{world} (blocks of {B} rows) + "
                                   + ("rows written into rank 0's image (HIP IPC, xGMI)"
                                      if use_ipc else
                                      "RCCL gather" if args.dist_backend == "nccl"
                                      else "host-staged gloo gather (rehearsal)"))
                   if dist_on else "single GPU"},
        "roofline": roofline,
        "segments_per_frame": int(segs_all / args.steps),
        "traced_segments_per_frame": int(traced_all / args.steps),
        "primary_reuse": reuse,
        "culled": culled,
    }
    if culled is not None:
        culled["speedup"] = round(culled["value"] / value, 3)
    if per_rank is not None:
        out["ranks"] = per_rank

    if check is not None:
        out["check"] = check
    rc = 0
    if dist_on and not args.no_cross_check:
        out["cross_rank_check"] = cross_rank_check(r, cam, W, H, S, D, B, world, head_idx,
                                                   head_frame, NO_REUSE, stream,
                                                   "ipc" if use_ipc else "gather")
        out["ranks"]["cross_rank_rows_bit_exact"] = out["cross_rank_check"]["bit_exact"]
        if not out["cross_rank_check"]["bit_exact"]:
            print("bench.py: cross-rank check FAILED: rows %s differ from rank 0's image"
                  % out["cross_rank_check"]["mismatched"], file=sys.stderr)
            rc = 4
    if args.tune:
        out["tune"] = args.tune
    if args.lib:
        out["lib"] = os.path.relpath(os.path.abspath(args.lib), ROOT)
    if world == 1 and wl.key == "reference1080" and args.shim_frames > 0:
        out["shim_sequence"] = shim_sequence(r, cam, spheres, mats, W, H, S, D, args.shim_frames)
    if world == 1 and not args.no_cpu_baseline:
        def gpu_shard(K, j):
            """Rows of shard j of K (one-row blocks, dealt serpentine: spread
            over the whole frame) of the headline frame, rendered again on the
            GPU with the headline's flags: (image rows, exact segment count)."""
            rows_j = abi.shard_rows(H, 1, K, j)
            buf = torch.empty((len(rows_j), W, 4), dtype=torch.float32, device="cuda")
            r.render_device(cam, buf.data_ptr(), W, H, S, D, head_idx * S, 1, K, j, NO_REUSE,
                            stream=stream.cuda_stream)
            st = r.wait()
            return rows_j, buf.cpu().numpy(), int(st["segments"])
        out["cpu_baseline"] = cpu_baseline(cam, spheres, mats, W, H, S, D, args.cpu_rows,
                                           head_frame.cpu().numpy(), head_idx, gpu_shard)
    os.write(json_fd, (json.dumps(out) + "\n").encode())
    if dist_on:
        dist.destroy_process_group()
    return rc


def cross_rank_check(r, cam, W, H, S, D, B, world, head_idx, head_frame, flags, stream, path):
    """N>1 self-check of the image path: rank 0 re-renders on its own GPU the
    first, middle and last row owned by every rank (row y alone = shard y of H
    with one-row blocks) of the timed run's frame `head_idx` and compares them
    bit for bit (NaN payloads included) with the rows the ranks delivered into
    its image -- through HIP IPC after rt_acquire, or the RCCL gather after the
    re-assembly. A stale or torn row from any rank shows as a mismatch."""
    import torch
    from bevy_raytrace_amd import distributed as rdist
    rows = [abi.shard_rows(H, B, world, k) for k in range(world)]
    picks = rdist.check_rows(rows)
    buf = torch.empty((1, W, 4), dtype=torch.float32, device="cuda")
    bad = []
    t0 = time.perf_counter()
    for k, y in picks:
        r.render_device(cam, buf.data_ptr(), W, H, S, D, head_idx * S, 1, H, y, flags,
                        stream=stream.cuda_stream)
        r.wait()
        ndiff = int((buf[0].view(torch.int32) != head_frame[y].view(torch.int32)).any(-1).sum().item())
        if ndiff:
            bad.append([k, y, ndiff])
    return {"bit_exact": not bad, "path": path, "frame": head_idx,
            "rows_checked": len(picks), "ranks_covered": len({k for k, _ in picks}),
            "rows": [[k, y] for k, y in picks], "mismatched": bad,
            "check_s": round(time.perf_counter() - t0, 3),
            "note": "rank 0 re-renders the first, middle and last row of every rank's shard of "
                    "the timed run's first frame of its last launch and compares the bits with "
                    "its image; mismatched = [rank, row, differing pixels]"}


def cpu_quota():
    """CPUs granted by the cgroup v2 quota (cpu.max), or None when unlimited."""
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(period), 2)
    except (OSError, ValueError):
        return None


def cpu_baseline(cam, spheres, mats, W, H, S, D, nrows, head_frame, head_idx, gpu_shard):
    """Time the C oracle (scalar port of the WGSL) on a bounded row sample of
    the timed headline frame and check it: the sample is shard j of K with
    one-row blocks (rows spread over the frame, top to bottom), the oracle's
    rows must equal the headline frame's rows bit for bit, and its segment
    count the GPU's count for the same rows (the same shard rendered again)."""
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    # every host core this process may run on -- unless the cgroup grants
    # fewer CPUs than that (the GPU box: 256 cores visible, a 16-CPU quota),
    # where more threads than the quota only time-slice (measured: 11.8
    # Mrays/s with 256 threads vs ~20 with 16); both counts are reported
    host = len(os.sched_getaffinity(0)) or 1
    quota = cpu_quota()
    cores = min(host, max(1, int(math.ceil(quota)))) if quota else host
    frame0 = head_idx * S
    # calibrate on `cores` spread rows (one row per thread), then size the
    # sample for ~10 s of wall time
    rows = [int(i * H / cores) for i in range(cores)]
    t0 = time.perf_counter()
    O.render_rows(cam, spheres, mats, W, H, S, D, rows, frame0=frame0, nthreads=cores)
    t1 = time.perf_counter() - t0
    if nrows <= 0:
        nrows = int(max(cores, min(H, cores * 10.0 / max(t1, 1e-3))))
    K = max(1, -(-H // max(1, nrows)))
    j = K // 2
    rows, gpu_rows, gpu_segs = gpu_shard(K, j)
    t0 = time.perf_counter()
    img, segs = O.render_rows(cam, spheres, mats, W, H, S, D, rows, frame0=frame0, nthreads=cores)
    dt = time.perf_counter() - t0
    exact = bool(np.array_equal(img, head_frame[rows], equal_nan=True))
    return {"value": round(segs / dt / 1e6, 3), "unit": "Mrays/s", "cores": cores,
            "host_cores": host, "cpu_quota_cores": quota, "kind": "port",
            "sample": f"{len(rows)} rows spread over the {W}x{H} {S}spp headline frame {head_idx} "
                      f"(rows {rows[0]}..{rows[-1]}: shard {j} of {K}, one-row blocks dealt "
                      f"serpentine), {segs} segments in {dt:.2f} s",
            "frame": head_idx,
            "gpu_rows_bit_exact": exact,
            "segments_equal": bool(segs == gpu_segs),
            "gpu_segments": gpu_segs,
            "gpu_shard_equals_headline": bool(np.array_equal(gpu_rows, head_frame[rows],
                                                             equal_nan=True))}


if __name__ == "__main__":
    sys.exit(main() or 0)
