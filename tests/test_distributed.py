"""N>1 path on CPU: world_size-2/3/8 gloo runs of the row tiling + gather +
re-assembly that bench.py drives over RCCL. Each rank's shard is rendered by
the oracle (the checker; on the GPU box the same code path takes rt_render
output), gathered to rank 0 with torch.distributed.gather, re-assembled and
compared with a full single-process render."""
import os
import socket

import numpy as np
import pytest

W, H, S, D = 20, 21, 2, 5


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, B, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    from bevy_raytrace_amd import scene
    from bevy_raytrace_amd.camera import default_camera_block
    from bevy_raytrace_amd.distributed import ShardLayout, assemble_host, gather_to_root
    from oracle import oracle as O

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sc = scene.rtiow_final_scene()
        sp, mt = sc.objects_gpu(), sc.materials_gpu()
        cam = default_camera_block()
        lay = ShardLayout(H, B, world)
        part, segs = O.render(cam, sp, mt, W, H, S, D, row_block=B, shard_count=world,
                              shard_index=rank, nthreads=1)
        slab = torch.zeros((lay.max_rows, W, 4), dtype=torch.float32)
        slab[:part.shape[0]] = torch.from_numpy(part)
        g = gather_to_root(dist, slab, world, rank)
        tot = torch.tensor([segs], dtype=torch.float64)
        dist.all_reduce(tot)
        if rank == 0:
            img = assemble_host(g.numpy(), lay)
            q.put((img, int(tot.item())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,B", [(2, 1), (2, 4), (3, 2), (8, 1)])
def test_gloo_row_tiling(world, B):
    """world 8 rehearses the driver's N=8 layout (21 rows: uneven shards,
    padded slabs, serpentine deal over 3 groups)."""
    import torch.multiprocessing as mp

    from bevy_raytrace_amd import scene
    from bevy_raytrace_amd.camera import default_camera_block
    from oracle import oracle as O

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, B, q)) for r in range(world)]
    for p in procs:
        p.start()
    img, segs = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sc = scene.rtiow_final_scene()
    full, fsegs = O.render(default_camera_block(), sc.objects_gpu(), sc.materials_gpu(), W, H, S, D,
                           nthreads=2)
    assert segs == fsegs
    assert np.array_equal(img, full, equal_nan=True)


@pytest.mark.parametrize("H,world", [(225, 2), (225, 3), (1080, 8), (4320, 8), (7, 8), (1, 2)])
def test_cross_check_rows_cover_every_rank(H, world):
    """bench.py's N>1 self-check re-renders, per rank, the first, middle and
    last row it owns (distributed.check_rows): every rank that owns rows is
    covered, each picked row is owned by the rank it is attributed to, and
    both ends of every shard are checked."""
    from bevy_raytrace_amd import abi, distributed as rdist
    from bevy_raytrace_amd.configs import pick_row_block
    B = pick_row_block(H, world)
    rows = [abi.shard_rows(H, B, world, k) for k in range(world)]
    picks = rdist.check_rows(rows)
    ys = [y for _, y in picks]
    assert len(ys) == len(set(ys))
    owners = {k for k, _ in picks}
    assert owners == {k for k in range(world) if rows[k]}
    for k, y in picks:
        assert y in rows[k]
    for k, rk in enumerate(rows):
        if rk:
            assert (k, rk[0]) in picks and (k, rk[-1]) in picks
