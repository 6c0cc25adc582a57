"""Multi-GPU frame sharding: one process per GPU, rows interleaved across
ranks, one framebuffer gather to rank 0 at the end of the frame.

The reference parallelises Camera::render over pixels with rayon
(src/camera.rs:179-181); pixels are independent and the world is read-only,
so each rank holds the whole world and renders rows y = rank, rank + N, ...
(interleaving balances cheap sky rows against expensive ground rows).  The
only exchange is the gather of the linear f32 framebuffer --
RCCL over xGMI with backend "nccl", gloo in CPU tests.
"""
import torch
import torch.distributed as dist


def shard_rows(height, rank, world_size):
    """Rows rank, rank+N, ... (rt_render_opts row_offset=rank, row_stride=N)."""
    if rank >= height:
        return 0
    return (height - rank + world_size - 1) // world_size


def assemble(gathered, height, width, world_size):
    """gathered: (N, rows_max, W, 3) padded shards -> (H, W, 3) frame."""
    rows_max = gathered.shape[1]
    # frame row y = k*N + r  <-  gathered[r, k]
    full = gathered.permute(1, 0, 2, 3).reshape(rows_max * world_size, width, 3)
    return full[:height]


def gather_frame(local, height, width, group=None):
    """Gathers every rank's (rows_r, W, 3) shard to rank 0 and returns the
    (H, W, 3) frame there (None on other ranks).  One collective per frame."""
    world_size = dist.get_world_size(group)
    rank = dist.get_rank(group)
    rows_max = (height + world_size - 1) // world_size
    if local.shape[0] != rows_max:
        pad = torch.zeros((rows_max, width, 3), dtype=local.dtype, device=local.device)
        pad[: local.shape[0]] = local
        local = pad
    if rank == 0:
        bufs = [torch.empty_like(local) for _ in range(world_size)]
        dist.gather(local, bufs, dst=0, group=group)
        return assemble(torch.stack(bufs), height, width, world_size)
    dist.gather(local, None, dst=0, group=group)
    return None
