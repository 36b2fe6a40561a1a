"""Multi-GPU sharding of the two hot paths: one process per GPU, torch.distributed
(backend "nccl" = RCCL over xGMI on MI355X; "gloo" for CPU tests).

Path tracer — sample-index shard. Rank g of G renders global samples s = g, g+G, g+2G, ...
(ptgs_trace_camera with frame_count = frame0 + g, frame_stride = G, PTGS_ACCUM_SUM) into an RGBA32F
sum buffer (rgb = radiance sum, a = sample count). One reduce(SUM) of W*H*4 floats to the root, then
mean = rgb / a. Equals the reference's running mean (raygen_camera.rgen:80-87) up to float
summation order (~1e-7 relative); integer outputs (ray counts) are unaffected.

3DGS — screen-tile shard. Gaussians are replicated; rank g renders tile rows [r0, r1) (global tile
ids, so tile/bin indices are identical to the single-GPU frame) into a zeroed frame; the disjoint
partial frames are summed with the same reduce (a gather of W*H*16/G bytes per rank).
"""
from __future__ import annotations


def sample_shard(rank: int, world: int, frame0: int = 0) -> tuple[int, int]:
    """(frame_count, frame_stride) for rank's samples: global sample k*world + rank."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    return frame0 + rank, world


def tile_row_shard(rank: int, world: int, height: int, tile: int = 16) -> tuple[int, int]:
    """Contiguous, balanced [begin, end) range of tile rows for `rank` (may be empty if world > rows)."""
    rows = (height + tile - 1) // tile
    base, extra = divmod(rows, world)
    begin = rank * base + min(rank, extra)
    end = begin + base + (1 if rank < extra else 0)
    return begin, end


def pixel_rows(tile_rows: tuple[int, int], height: int, tile: int = 16) -> tuple[int, int]:
    return min(tile_rows[0] * tile, height), min(tile_rows[1] * tile, height)


def reduce_sum(tensor, dst: int = 0, group=None):
    """In-place SUM reduce to `dst` (RCCL over xGMI for device tensors; gloo for host tensors)."""
    import torch.distributed as dist
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.reduce(tensor, dst=dst, op=dist.ReduceOp.SUM, group=group)
    return tensor


def all_reduce_sum(tensor, group=None):
    import torch.distributed as dist
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(tensor, op=dist.ReduceOp.SUM, group=group)
    return tensor


def init_native_comm(renderer, group=None):
    """The library's own RCCL communicator (ptgs_comm_create) on every rank: rank 0 makes the unique
    id, torch.distributed ships it (any backend). After this, renderer.reduce_radiance /
    allreduce_radiance run the frame reduce through the C-ABI instead of torch."""
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    box = [renderer.comm_unique_id() if rank == 0 else None]
    if world > 1:
        dist.broadcast_object_list(box, src=0, group=group)
    renderer.comm_create(box[0], world, rank)
    return rank, world


def resolve_mean(sum_rgba):
    """rgb / count, alpha = 1 (the running-mean image the reference keeps in rt_output_image)."""
    out = sum_rgba.clone()
    cnt = sum_rgba[..., 3:4].clamp_min(1.0)
    out[..., :3] = sum_rgba[..., :3] / cnt
    out[..., 3] = 1.0
    return out


def render_path_traced_frame(renderer, ubo, width: int, height: int, accum, spp_per_rank: int, rank: int,
                             world: int, frame0: int = 0, stream=None):
    """One sample-sharded frame on this rank's GPU followed by the reduce; the root gets the sums."""
    from ._abi import ACCUM_SUM
    f, stride = sample_shard(rank, world, frame0)
    ubo.frame_count = f
    accum.zero_()
    renderer.trace_camera(ubo, width, height, accum, spp=spp_per_rank, frame_stride=stride, mode=ACCUM_SUM,
                          stream=stream)
    return reduce_sum(accum)


def render_gaussian_frame(renderer, gaussians: dict, ubo, width: int, height: int, out, rank: int, world: int,
                          bg=(0.0, 0.0, 0.0), stream=None):
    """Tile-row-sharded 3DGS frame; the root gets the composed image."""
    out.zero_()
    rows = tile_row_shard(rank, world, height)
    if rows[1] > rows[0]:
        renderer.splat_gaussians(gaussians, ubo, width, height, out, bg=bg, tile_rows=rows, stream=stream)
    return reduce_sum(out)
