"""Multi-GPU sharding of the two hot paths: one process per GPU, torch.distributed
(backend "nccl" = RCCL over xGMI on MI355X; "gloo" for CPU tests).

Path tracer — sample-index shard. Rank g of G renders global samples s = g, g+G, g+2G, ...
(ptgs_trace_camera with frame_count = frame0 + g, frame_stride = G, PTGS_ACCUM_SUM) into an RGBA32F
sum buffer (rgb = radiance sum, a = sample count). One reduce(SUM) of W*H*4 floats to the root, then
mean = rgb / a. Equals the reference's running mean (raygen_camera.rgen:80-87) up to float
summation order (~1e-7 relative); integer outputs (ray counts) are unaffected.

3DGS — screen-tile shard. Gaussians are replicated; rank g renders tile rows [r0, r1) (global tile
ids, so tile/bin indices are identical to the single-GPU frame); the root gathers every rank's rows
(W*H*16/G bytes each: ptgs_gather_rows over RCCL send/recv with the library's communicator, or
torch.distributed send/recv). Row ranges are balanced by per-tile-row pair counts (the work of the
blend) from an earlier frame (balanced_tile_rows).

With the library's own communicator (init_native_comm) the collectives run through the C-ABI
(ptgs_reduce_radiance / ptgs_gather_rows); otherwise through torch.distributed.
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


def balanced_tile_rows(row_pairs, world: int, tiles_x: int, tile_cost: float = 32.0) -> list[tuple[int, int]]:
    """Contiguous tile-row ranges, one per rank, with about equal blend work: a tile row costs its
    (Gaussian, tile) pairs plus tile_cost per tile (the per-tile fixed work). row_pairs: pairs per
    tile row (e.g. from a previous frame's tile ranges)."""
    import numpy as np
    return _split_rows(np.asarray(row_pairs, np.float64) + tile_cost * tiles_x, world)


def rebalance_tile_rows(split, band_ms, row_pairs, tiles_x: int, tile_cost: float = 32.0) -> list[tuple[int, int]]:
    """Re-split tile rows from measured band times (a multi-GPU renderer times each rank's band every frame:
    pair counts alone miss what else a band costs, e.g. the chunks its front end keeps). Each row of band b
    is given band_ms[b] x its share of the band's pair-based weight (balanced_tile_rows' weights) and the
    cumulative cost is cut into equal parts again. 10M Gaussians at 4K, 8 bands: slowest band 1.451 ms from
    the pair split (bands 1.156 - 1.451 ms), see DESIGN §6."""
    import numpy as np
    w = np.asarray(row_pairs, np.float64) + tile_cost * tiles_x
    cost = np.zeros_like(w)
    for (a, b), ms in zip(split, band_ms):
        if b > a:
            cost[a:b] = float(ms) * w[a:b] / max(w[a:b].sum(), 1e-30)
    return _refine_split(_split_rows(cost, len(split)), cost)


def _refine_split(split, cost, iters: int = 64) -> list[tuple[int, int]]:
    """Lower the costliest band of a contiguous split by moving its edge row to a neighbour while that lowers
    the larger of the two (the equal-share cut places each boundary independently; with rows of ~0.14 ms at
    the 10M / 4K frame's centre it left a band one row above its neighbours, r06e: 1.435 vs 1.276 ms)."""
    import numpy as np
    c = np.concatenate([[0.0], np.cumsum(np.asarray(cost, np.float64))])
    b = [s for s, _ in split] + [split[-1][1]]
    band = lambda i: c[b[i + 1]] - c[b[i]]
    for _ in range(iters):
        i = max(range(len(split)), key=band)
        best = None
        if i > 0 and b[i + 1] - b[i] > 1:  # its first row to the band before
            m = max(c[b[i] + 1] - c[b[i - 1]], c[b[i + 1]] - c[b[i] + 1])
            best = (m, i, +1)
        if i + 1 < len(split) and b[i + 1] - b[i] > 1:  # its last row to the band after
            m = max(c[b[i + 1] - 1] - c[b[i]], c[b[i + 2]] - c[b[i + 1] - 1])
            if best is None or m < best[0]:
                best = (m, i + 1, -1)
        if best is None or best[0] >= band(i) - 1e-12:
            break
        b[best[1]] += best[2]
    return [(b[i], b[i + 1]) for i in range(len(split))]


def _split_rows(w, world: int) -> list[tuple[int, int]]:
    """Contiguous row ranges, one per rank, of about equal total weight (w: per row)."""
    import numpy as np
    rows = len(w)
    cum = np.concatenate([[0.0], np.cumsum(w)])
    bounds = [0]
    for g in range(1, world):
        t = cum[-1] * g / world
        b = int(np.searchsorted(cum, t, side="left"))
        if b > 0 and (b > rows or t - cum[b - 1] < cum[b] - t):  # the nearer of the two boundaries
            b -= 1
        bounds.append(min(max(b, bounds[-1]), rows))
    bounds.append(rows)
    return [(bounds[g], bounds[g + 1]) for g in range(world)]


def splat_policy(frame_ms: float, width: int, height: int, world: int, link_gbs: float = 50.0) -> str:
    """How several GPUs split 3DGS frames: "tile_rows" (every rank renders a band of each frame,
    rank 0 gathers the rows) when a rank's share of the frame (frame_ms / world, the ideal band) takes longer
    than rank 0's intake of a peer's rows over its own xGMI link (W*H*16/world bytes at link_gbs per link,
    all peers in parallel); else "replicas" (each rank renders whole frames of its own - other views or
    other frames - and nothing crosses the links). C2 (100k Gaussians, 1080p, ~0.053 ms): the band would be
    ~7 us against ~83 us of gather at 8 ranks -> replicas; C5's splat (10M Gaussians, 4K, ~8.5 ms): ~1.07 ms
    against ~0.33 ms -> tile rows. world 1: "single"."""
    if world <= 1:
        return "single"
    gather_ms = width * height * 16.0 / world / (link_gbs * 1e9) * 1e3
    return "tile_rows" if frame_ms / world > gather_ms else "replicas"


def row_pairs_from_ranges(tile_ranges, tiles_x: int):
    """Per-tile-row pair counts from a frame's tile ranges ((tiles, 2) uint32: [begin, end) per tile)."""
    import numpy as np
    r = np.asarray(tile_ranges, np.int64).reshape(-1, 2)
    return (r[:, 1] - r[:, 0]).reshape(-1, tiles_x).sum(axis=1)


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


def gather_rows(image, pixel_ranges, dst: int = 0, renderer=None, group=None, stream=None):
    """Every rank's pixel rows [r0, r1) of image ((H, W, 4) float32) to the same rows of dst's image.
    Through the library's communicator when the renderer has one (ordered on `stream`), else
    torch.distributed send/recv, issued after the work already on `stream` (the rows it renders)."""
    import torch.distributed as dist
    if not (dist.is_initialized() and dist.get_world_size(group) > 1):
        return image
    if len(pixel_ranges) != dist.get_world_size(group):
        raise ValueError("gather_rows needs one (r0, r1) per rank")
    if renderer is not None and getattr(renderer, "comm_world", 0) > 1:
        renderer.gather_rows(image, pixel_ranges, root=dst, stream=stream)
        return image
    with _on_stream(image, stream):
        rank = dist.get_rank(group)
        if rank == dst:
            for g, (r0, r1) in enumerate(pixel_ranges):
                if g != dst and r1 > r0:
                    dist.recv(image[r0:r1], src=g, group=group)
        else:
            r0, r1 = pixel_ranges[rank]
            if r1 > r0:
                dist.send(image[r0:r1].contiguous(), dst=dst, group=group)
    return image


def reduce_scatter_rows(image, pixel_ranges, renderer=None, group=None, stream=None):
    """Afterwards every rank's own pixel rows [r0, r1) of image ((H, W, 4) float32) hold the SUM over
    the ranks of those rows (other rows unspecified): ptgs_reduce_scatter_rows through the library's
    communicator (one ncclReduce per rank's rows, grouped), else one torch.distributed reduce per
    rank's rows to that rank. About one frame per rank on the wire instead of an all-reduce's two."""
    import torch.distributed as dist
    if not (dist.is_initialized() and dist.get_world_size(group) > 1):
        return image
    if len(pixel_ranges) != dist.get_world_size(group):
        raise ValueError("reduce_scatter_rows needs one (r0, r1) per rank")
    if renderer is not None and getattr(renderer, "comm_world", 0) > 1:
        renderer.reduce_scatter_rows(image, pixel_ranges, stream=stream)
        return image
    with _on_stream(image, stream):
        for g, (r0, r1) in enumerate(pixel_ranges):
            if r1 > r0:
                dist.reduce(image[r0:r1], dst=g, op=dist.ReduceOp.SUM, group=group)
    return image


class _on_stream:
    """torch.cuda.stream(stream) for device tensors (collectives issued after the stream's work);
    nothing for host tensors or stream=None."""

    def __init__(self, tensor, stream):
        self.ctx = None
        if stream is not None and not isinstance(stream, int) and getattr(tensor, "is_cuda", False):
            import torch
            self.ctx = torch.cuda.stream(stream)

    def __enter__(self):
        if self.ctx is not None:
            self.ctx.__enter__()
        return self

    def __exit__(self, *exc):
        if self.ctx is not None:
            return self.ctx.__exit__(*exc)
        return False


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
    if getattr(renderer, "comm_world", 0) > 1:
        renderer.reduce_radiance(accum, root=0, stream=stream)
        return accum
    return reduce_sum(accum)


class _DeferredReport:
    """PTGS_EINCOMPLETE / PTGS_EBADIDS from a splat call report an EARLIER frame (ptgs.h): this call's frame
    was rendered. Raising it before the frame's collective would leave the other ranks blocked in it (a
    multi-rank hang), so the splat calls of a sharded frame run inside this context, which holds
    such a report until the collective has been issued (`raise_pending`). Any other error raises at once."""

    def __init__(self):
        self.err = None

    def __enter__(self):
        return self

    def __exit__(self, et, ev, tb):
        from ._abi import PTGS_EBADIDS, PTGS_EINCOMPLETE, PtgsError
        # (codes of their own for reports about earlier frames: no message matching)
        if et is not None and issubclass(et, PtgsError) and ev.code in (PTGS_EINCOMPLETE, PTGS_EBADIDS):
            self.err = ev
            return True
        return False

    def raise_pending(self):
        if self.err is not None:
            raise self.err


def render_gaussian_frame(renderer, gaussians: dict, ubo, width: int, height: int, out, rank: int, world: int,
                          bg=(0.0, 0.0, 0.0), stream=None, tile_rows=None):
    """Tile-row-sharded 3DGS frame; the root gets the composed image. tile_rows: every rank's
    (begin, end) tile rows (default: equal row counts, tile_row_shard). A report about an earlier frame of
    this rank's workspace is raised after the row gather (every rank joins the collective)."""
    if tile_rows is None:
        tile_rows = [tile_row_shard(g, world, height) for g in range(world)]
    rows = tile_rows[rank]
    rep = _DeferredReport()
    if rows[1] > rows[0]:
        with rep:
            renderer.splat_gaussians(gaussians, ubo, width, height, out, bg=bg, tile_rows=rows, stream=stream)
    img = gather_rows(out, [pixel_rows(r, height) for r in tile_rows], dst=0, renderer=renderer, stream=stream)
    rep.raise_pending()
    return img


class RowGatherPipeline:
    """Tile-row-sharded 3DGS frames with the row gather of frame f overlapped with the band of frame f + 1
    (VERDICT r4 next #3c; render_gaussian_frame serialises them on one stream). Two images alternate:
    frame f renders this rank's rows into image f % 2 on the compute stream; its gather to rank 0 is issued
    on a second (gather) stream behind an event of that frame, so the band of frame f + 1 (the other image)
    runs while the rows of frame f are on the wire; the band of frame f + 2 (image f % 2 again) waits for
    frame f's gather. Host tensors (gloo) and stream=None run the same steps in order.
      pipe = RowGatherPipeline(renderer, W, H, tile_rows, rank, world, stream=s)
      for ubo in views: img = pipe.submit(gaussians, ubo)   # rank 0: frame complete after pipe.wait(img)
    The images equal render_gaussian_frame's bit for bit (the same splat calls and the same gather)."""

    def __init__(self, renderer, width: int, height: int, tile_rows, rank: int, world: int, stream=None,
                 device: str = "cuda", bg=(0.0, 0.0, 0.0)):
        import torch
        self.r, self.W, self.H, self.rank, self.world, self.bg = renderer, width, height, rank, world, bg
        self.tile_rows = list(tile_rows)
        self.px = [pixel_rows(t, height) for t in self.tile_rows]
        self.images = [torch.zeros((height, width, 4), dtype=torch.float32, device=device) for _ in range(2)]
        self.cuda = self.images[0].is_cuda and stream is not None
        self.stream = stream
        self.gstream = torch.cuda.Stream(device=self.images[0].device) if self.cuda else None
        self.gathered = [None, None]  # gather-stream events: image k may be overwritten after it
        self.count = 0

    def submit(self, gaussians, ubo):
        """Render this rank's rows of one frame and issue their gather; returns the frame's image (rank 0:
        the composed frame once wait(image) returns)."""
        import torch
        k = self.count % 2
        img = self.images[k]
        if self.cuda and self.gathered[k] is not None:
            self.stream.wait_event(self.gathered[k])  # frame f - 2's rows have left this image
        rows = self.tile_rows[self.rank]
        rep = _DeferredReport()
        if rows[1] > rows[0]:
            with rep:
                self.r.splat_gaussians(gaussians, ubo, self.W, self.H, img, bg=self.bg, tile_rows=rows,
                                       stream=self.stream)
        if self.cuda:
            done = torch.cuda.Event()
            done.record(self.stream)
            self.gstream.wait_event(done)
            gather_rows(img, self.px, dst=0, renderer=self.r, stream=self.gstream)
            ev = torch.cuda.Event()
            ev.record(self.gstream)
            self.gathered[k] = ev
        else:
            gather_rows(img, self.px, dst=0, renderer=self.r, stream=self.stream)
        self.count += 1
        rep.raise_pending()  # (after the collective: see _DeferredReport)
        return img

    def wait(self, img=None):
        """The compute stream waits for the gathers (of `img`, or of every frame in flight)."""
        if not self.cuda:
            return
        for k in range(2):
            if self.gathered[k] is not None and (img is None or self.images[k] is img):
                self.stream.wait_event(self.gathered[k])


def render_hybrid_frame(renderer, gaussians: dict, ubo, width: int, height: int, accum, depth, out, spp_total: int,
                        rank: int, world: int, frame0: int = 0, tile_rows=None, stream=None, **splat_kw):
    """The C5 hybrid frame ("both, with the depth composite done after the reduce"), sharded
    so that each rank moves only what its rows need:
      1. rank g traces samples g, g + G, ... (spp_total / G of them, SUM) of the whole frame into accum;
      2. reduce-scatter of accum by the ranks' tile rows (reduce_scatter_rows): rank g ends up with the
         full radiance sum of its own rows only;
      3. their running mean (rgb / count, a = 1) into out's rows, the primary-hit depth of its rows;
      4. the 3DGS splat-over composite of its tile rows (ptgs_splat_gaussians_over, out as "under");
      5. the row gather to rank 0 (gather_rows): out is the composed frame there.
    accum: (H, W, 4) sum buffer; depth: (H, W); out: (H, W, 4). tile_rows: every rank's (begin, end)
    tile rows (default tile_row_shard). Equals the single-process frame (trace spp_total, mean, depth,
    splat over) up to the float order of the radiance sums (~1e-7 relative)."""
    from ._abi import ACCUM_SUM
    if spp_total % world:
        raise ValueError(f"spp_total {spp_total} is not a multiple of the world size {world}")
    if tile_rows is None:
        tile_rows = [tile_row_shard(g, world, height) for g in range(world)]
    px = [pixel_rows(r, height) for r in tile_rows]
    f, stride = sample_shard(rank, world, frame0)
    ubo.frame_count = f
    with _on_stream(accum, stream):
        accum.zero_()
    renderer.trace_camera(ubo, width, height, accum, spp=spp_total // world, frame_stride=stride, mode=ACCUM_SUM,
                          stream=stream)
    reduce_scatter_rows(accum, px, renderer=renderer, stream=stream)
    p0, p1 = px[rank]
    if p1 > p0:  # the primary-hit depth of this rank's rows only (the composite reads no other)
        renderer.trace_depth(ubo, width, height, depth, stream=stream, rows=(p0, p1))
    rep = _DeferredReport()
    if p1 > p0:
        with _on_stream(out, stream):
            out[p0:p1] = resolve_mean(accum[p0:p1])
        with rep:
            renderer.splat_gaussians(gaussians, ubo, width, height, out, tile_rows=tile_rows[rank],
                                     over=(depth, out), stream=stream, **splat_kw)
    img = gather_rows(out, px, dst=0, renderer=renderer, stream=stream)
    rep.raise_pending()  # (after the collective: see _DeferredReport)
    return img
