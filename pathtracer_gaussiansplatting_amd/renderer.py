"""Renderer: the device-side API over libptgs.so (the drop-in for the reference's RT pipeline).

Mirrors what Engine does around the hot path (Vulkan_Engine/engine.cpp):
  upload_scene(scene)              createGlobalBindlessBuffers + buildBlas/initStaticTlas
  trace_camera(ubo, accum, spp)    vkCmdTraceRaysKHR(W,H,1) x spp + running mean (:1971, :2684-2708)
  trace_torus(...)                 torus trace (:1893-1900, :2787-2794)
  splat_points(...)                point-cloud draw (:1945-1961)
  splat_gaussians(...)             3DGS forward (absent from the reference)
  encode_srgb8(...)                rgba32f -> sRGB8 blit (:2004-2020)
Device buffers are torch tensors on the context's device (or raw device pointers as ints).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi
from ._abi import BvhBuffers, Gaussians, RayPush, SceneInfo, SplatBuffers, SplatStats, SplatStatus, TraceStats, Ubo


def _ptr(x) -> int:
    if x is None:
        return 0
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        if not x.is_cuda:
            raise _abi.PtgsError("expected a device tensor (got a host tensor): the renderer has no CPU path")
        if not x.is_contiguous():
            raise _abi.PtgsError("device tensor must be contiguous")
        return x.data_ptr()
    raise TypeError(f"cannot take a device pointer of {type(x)}")


def _gaussians(g: dict) -> Gaussians:
    """ptgs_gaussians of a dict of device tensors (means, scales, rotations, opacities, colors[, ids])."""
    gs = Gaussians()
    gs.means, gs.scales, gs.rotations = _ptr(g["means"]), _ptr(g["scales"]), _ptr(g["rotations"])
    gs.opacities, gs.colors = _ptr(g["opacities"]), _ptr(g["colors"])
    gs.count = int(g["means"].shape[0])
    gs.ids = _ptr(g.get("ids"))
    gs.chunk_bounds = _ptr(g.get("chunk_bounds"))
    return gs


def _stream(stream) -> int:
    if stream is None:
        try:
            import torch
            return torch.cuda.current_stream().cuda_stream
        except Exception:
            return 0
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


class Renderer:
    def __init__(self, device: int = 0, lib_path: str | None = None, publish_splat_buffers: bool = False,
                 wavefront: bool = False):
        """publish_splat_buffers: every synchronised splat (want_stats) also publishes its sorted
        keys / values for splat_buffers() (PTGS_FLAG_SPLAT_PUBLISH); "tight": and bins them like the
        stream-ordered frames (PTGS_FLAG_SPLAT_PUBLISH_TIGHT, parity tests of the timed path); wavefront:
        trace_camera runs the wavefront path tracer (PTGS_FLAG_PT_WAVEFRONT). All are kept across set_flags."""
        self.lib = _abi.load_library(lib_path)
        self._publish = _abi.FLAG_PT_WAVEFRONT if wavefront else 0
        if publish_splat_buffers:
            self._publish |= _abi.FLAG_SPLAT_PUBLISH
        if publish_splat_buffers == "tight":
            self._publish |= _abi.FLAG_SPLAT_PUBLISH_TIGHT
        h = C.c_void_p()
        rc = self.lib.ptgs_create(int(device), C.byref(h))
        _abi.check(rc, f"ptgs_create(device={device})")
        self._h = h
        self.device = device
        self.scene = None
        self.set_flags(0)

    def close(self):
        if getattr(self, "_h", None):
            self.lib.ptgs_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _err(self) -> str:
        return (self.lib.ptgs_last_error(self._h) or b"").decode()

    def _chk(self, rc: int, what: str):
        _abi.check(rc, what, self._err())

    # ---------------------------------------------------------------- scene
    def upload_scene(self, scene) -> SceneInfo:
        d = scene.desc()
        self._chk(self.lib.ptgs_scene_upload(self._h, C.byref(d)), "ptgs_scene_upload")
        self.scene = scene
        return self.scene_info()

    def scene_info(self) -> SceneInfo:
        info = SceneInfo()
        self._chk(self.lib.ptgs_scene_get_info(self._h, C.byref(info)), "ptgs_scene_get_info")
        return info

    # ---------------------------------------------------------------- path tracer
    def trace_camera(self, ubo: Ubo, width: int, height: int, accum, spp: int = 1, frame_stride: int = 1,
                     mode: int = _abi.ACCUM_RUNNING_MEAN, rows: tuple | None = None, stream=None):
        if rows is None:
            rc = self.lib.ptgs_trace_camera(self._h, C.byref(ubo), width, height, _ptr(accum), spp, frame_stride,
                                            mode, _stream(stream))
        else:
            rc = self.lib.ptgs_trace_camera_rows(self._h, C.byref(ubo), width, height, rows[0], rows[1],
                                                 _ptr(accum), spp, frame_stride, mode, _stream(stream))
        self._chk(rc, "ptgs_trace_camera")

    def trace_torus(self, ubo: Ubo, push: RayPush, samples, n: int, hits, stream=None):
        rc = self.lib.ptgs_trace_torus(self._h, C.byref(ubo), C.byref(push), _ptr(samples), n, _ptr(hits),
                                       _stream(stream))
        self._chk(rc, "ptgs_trace_torus")

    def trace_depth(self, ubo: Ubo, width: int, height: int, depth, stream=None, rows=None):
        """Primary-hit view depth per pixel (+inf on a miss) into a device float[H, W] tensor; rows =
        (begin, end) pixel rows traces only those (ptgs_trace_depth_rows)."""
        if rows is not None:
            rc = self.lib.ptgs_trace_depth_rows(self._h, C.byref(ubo), width, height, int(rows[0]), int(rows[1]),
                                                _ptr(depth), _stream(stream))
            self._chk(rc, "ptgs_trace_depth_rows")
            return
        rc = self.lib.ptgs_trace_depth(self._h, C.byref(ubo), width, height, _ptr(depth), _stream(stream))
        self._chk(rc, "ptgs_trace_depth")

    # ---------------------------------------------------------------- 3DGS initialisation (§8f #3)
    def knn3_mean_dist2(self, xyz, dist2, stream=None):
        """dist2[i] = mean squared distance of point i to its 3 nearest other points (device tensors:
        xyz float32 [N, 3], dist2 float32 [N])."""
        n = int(xyz.shape[0])
        self._chk(self.lib.ptgs_knn3_mean_dist2(self._h, _ptr(xyz), n, _ptr(dist2), _stream(stream)),
                  "ptgs_knn3_mean_dist2")

    def gaussians_from_points(self, xyz, rgb=None, stream=None) -> dict:
        """Kerbl et al. create_from_pcd in post-activation form -> dict of device tensors in the
        splat_gaussians layout (means, scales, rotations, opacities, colors)."""
        import torch
        n = int(xyz.shape[0])
        dev = xyz.device
        g = {"means": torch.empty((n, 3), dtype=torch.float32, device=dev),
             "scales": torch.empty((n, 3), dtype=torch.float32, device=dev),
             "rotations": torch.empty((n, 4), dtype=torch.float32, device=dev),
             "opacities": torch.empty((n,), dtype=torch.float32, device=dev),
             "colors": torch.empty((n, 3), dtype=torch.float32, device=dev)}
        rc = self.lib.ptgs_gaussians_from_points(self._h, _ptr(xyz), _ptr(rgb), n, _ptr(g["means"]), _ptr(g["scales"]),
                                                 _ptr(g["rotations"]), _ptr(g["opacities"]), _ptr(g["colors"]),
                                                 _stream(stream))
        self._chk(rc, "ptgs_gaussians_from_points")
        return g

    # ---------------------------------------------------------------- RCCL frame reduce (§8e)
    def comm_unique_id(self) -> bytes:
        buf = (C.c_uint8 * 128)()
        self._chk(self.lib.ptgs_comm_unique_id(buf), "ptgs_comm_unique_id")
        return bytes(buf)

    def comm_create(self, unique_id: bytes, nranks: int, rank: int):
        buf = (C.c_uint8 * 128).from_buffer_copy(unique_id)
        self._chk(self.lib.ptgs_comm_create(self._h, buf, nranks, rank), "ptgs_comm_create")
        self.comm_world = nranks

    def comm_destroy(self):
        self._chk(self.lib.ptgs_comm_destroy(self._h), "ptgs_comm_destroy")
        self.comm_world = 0

    def reduce_radiance(self, accum, root: int = 0, stream=None):
        rc = self.lib.ptgs_reduce_radiance(self._h, _ptr(accum), accum.numel(), root, _stream(stream))
        self._chk(rc, "ptgs_reduce_radiance")

    def allreduce_radiance(self, accum, stream=None):
        rc = self.lib.ptgs_allreduce_radiance(self._h, _ptr(accum), accum.numel(), _stream(stream))
        self._chk(rc, "ptgs_allreduce_radiance")

    def gather_rows(self, image, row_ranges, root: int = 0, stream=None):
        """Every rank's pixel rows [r0, r1) of the (H, W, 4) float32 image to root (ptgs_gather_rows);
        row_ranges: one (r0, r1) per rank, identical on every rank."""
        H, W = int(image.shape[0]), int(image.shape[1])
        world = getattr(self, "comm_world", 0)
        if len(row_ranges) != world:  # the library reads 2 x nranks entries
            raise ValueError(f"gather_rows needs one (r0, r1) per rank: {len(row_ranges)} given, world {world}")
        rr = np.asarray(row_ranges, np.uint32).reshape(-1)
        if rr.size != 2 * world:
            raise ValueError("gather_rows: every row range is a (r0, r1) pair")
        rc = self.lib.ptgs_gather_rows(self._h, _ptr(image), W, H, rr.ctypes.data, root, _stream(stream))
        self._chk(rc, "ptgs_gather_rows")

    def reduce_scatter_rows(self, image, row_ranges, stream=None):
        """ptgs_reduce_scatter_rows: afterwards this rank's pixel rows of the (H, W, 4) float32 image hold
        the SUM over the ranks of those rows; row_ranges: one (r0, r1) per rank, identical everywhere."""
        H, W = int(image.shape[0]), int(image.shape[1])
        world = getattr(self, "comm_world", 0)
        if len(row_ranges) != world:
            raise ValueError(f"reduce_scatter_rows needs one (r0, r1) per rank: {len(row_ranges)} given, world {world}")
        rr = np.asarray(row_ranges, np.uint32).reshape(-1)
        if rr.size != 2 * world:
            raise ValueError("reduce_scatter_rows: every row range is a (r0, r1) pair")
        rc = self.lib.ptgs_reduce_scatter_rows(self._h, _ptr(image), W, H, rr.ctypes.data, _stream(stream))
        self._chk(rc, "ptgs_reduce_scatter_rows")

    def set_flags(self, flags: int):
        self._flags = flags
        self._chk(self.lib.ptgs_set_flags(self._h, flags | self._publish), "ptgs_set_flags")

    def set_wavefront(self, on: bool):
        """Select the path tracer of trace_camera: wavefront stages (True) or the one-kernel path loop."""
        self._publish = (self._publish & ~_abi.FLAG_PT_WAVEFRONT) | (_abi.FLAG_PT_WAVEFRONT if on else 0)
        self.set_flags(getattr(self, "_flags", 0))

    def set_splat_overlap(self, on: bool):
        """Frames in flight for splat_gaussians (PTGS_FLAG_SPLAT_OVERLAP): the front end of each
        stream-ordered call runs on a second stream while the previous call's blend runs on the caller's.
        The Gaussians must not be rewritten on the stream between two such calls (see ptgs.h)."""
        self._publish = (self._publish & ~_abi.FLAG_SPLAT_OVERLAP) | (_abi.FLAG_SPLAT_OVERLAP if on else 0)
        self.set_flags(getattr(self, "_flags", 0))

    def stats_reset(self, stream=None):
        self._chk(self.lib.ptgs_stats_reset(self._h, _stream(stream)), "ptgs_stats_reset")

    def stats(self) -> TraceStats:
        s = TraceStats()
        self._chk(self.lib.ptgs_stats_read(self._h, C.byref(s)), "ptgs_stats_read")
        return s

    # ---------------------------------------------------------------- rasterizers
    def splat_points(self, ubo: Ubo, push: RayPush, hits, samples, n: int, width: int, height: int, rgba8, depth,
                     stream=None):
        rc = self.lib.ptgs_splat_points(self._h, C.byref(ubo), C.byref(push), _ptr(hits), _ptr(samples), n, width,
                                        height, _ptr(rgba8), _ptr(depth), _stream(stream))
        self._chk(rc, "ptgs_splat_points")

    def splat_gaussians(self, g: dict, ubo: Ubo, width: int, height: int, out, bg=(0.0, 0.0, 0.0),
                        tile_rows: tuple | None = None, want_stats: bool = False, stream=None, over=None):
        """over=(depth, under): the hybrid composite of ptgs_splat_gaussians_over (device depth[H, W],
        under RGBA32F[H, W, 4]; out may be under itself)."""
        gs = _gaussians(g)
        bgc = np.asarray(bg, np.float32)
        t0, t1 = (0, 0xFFFFFFFF) if tile_rows is None else tile_rows
        st = SplatStats()
        if over is not None:
            rc = self.lib.ptgs_splat_gaussians_over(self._h, C.byref(gs), C.byref(ubo), width, height, _ptr(over[0]),
                                                    _ptr(over[1]), t0, t1, _ptr(out),
                                                    C.byref(st) if want_stats else None, _stream(stream))
            self._chk(rc, "ptgs_splat_gaussians_over")
            return st if want_stats else None
        rc = self.lib.ptgs_splat_gaussians(self._h, C.byref(gs), C.byref(ubo), width, height, _abi.fptr(bgc), t0,
                                           t1, _ptr(out), C.byref(st) if want_stats else None, _stream(stream))
        self._chk(rc, "ptgs_splat_gaussians")
        return st if want_stats else None

    def splat_gaussians_views(self, g: dict, ubos, width: int, height: int, outs, bg=(0.0, 0.0, 0.0), stream=None):
        """ptgs_splat_gaussians_views: len(ubos) views of the same Gaussians in one stream-ordered call
        (outs: one RGBA32F[H, W, 4] device tensor per view)."""
        n = len(ubos)
        if len(outs) != n:
            raise ValueError("one output per view")
        gs = _gaussians(g)
        bgc = np.asarray(bg, np.float32)
        arr = (Ubo * n)(*ubos)
        optrs = (C.c_void_p * n)(*[_ptr(o) for o in outs])
        rc = self.lib.ptgs_splat_gaussians_views(self._h, C.byref(gs), n, arr, width, height, _abi.fptr(bgc), optrs,
                                                 _stream(stream))
        self._chk(rc, "ptgs_splat_gaussians_views")

    def sort_gaussians_spatial(self, g: dict, stream=None) -> dict:
        """ptgs_gaussians_sort_spatial: a copy of the device Gaussians `g` in 3D Morton order of the means
        plus "ids" (int32 tensor: the original index of each copy); splatting the copy renders exactly like
        `g` (scene preparation: synchronises)."""
        import torch
        out = {k: torch.empty_like(g[k]) for k in ("means", "scales", "rotations", "opacities", "colors")}
        n = int(g["means"].shape[0])
        out["ids"] = torch.empty(n, dtype=torch.int32, device=g["means"].device)
        rc = self.lib.ptgs_gaussians_sort_spatial(self._h, C.byref(_gaussians(g)), _ptr(out["means"]), _ptr(out["scales"]),
                                                  _ptr(out["rotations"]), _ptr(out["opacities"]), _ptr(out["colors"]),
                                                  _ptr(out["ids"]), _stream(stream))
        self._chk(rc, "ptgs_gaussians_sort_spatial")
        return out

    def gaussians_chunk_bounds(self, g: dict, stream=None):
        """ptgs_gaussians_chunk_bounds: per chunk of 256 Gaussians the box of the means and the largest
        scale (float32 tensor [chunks, 8]); put it in g["chunk_bounds"] so that tile-row-restricted
        frames skip the chunks that cannot reach their rows."""
        import torch
        n = int(g["means"].shape[0])
        out = torch.empty((max(1, (n + 255) // 256), 8), dtype=torch.float32, device=g["means"].device)
        self._chk(self.lib.ptgs_gaussians_chunk_bounds(self._h, C.byref(_gaussians(g)), _ptr(out), _stream(stream)),
                  "ptgs_gaussians_chunk_bounds")
        return out

    def splat_status(self, stream=None) -> SplatStatus:
        """ptgs_splat_status_read: waits for `stream` and the view streams, returns and clears the
        counts since the last query: frames left incomplete (spill pool exhausted), tiles completed
        through the spill pool, tiles left incomplete; buffer capacities."""
        st = SplatStatus()
        self._chk(self.lib.ptgs_splat_status_read(self._h, C.byref(st), _stream(stream)), "ptgs_splat_status_read")
        return st

    def splat_reserve(self, pairs: int):
        """Grow every view slot's pair buffer and spill pool to at least `pairs` (frames of up to that
        many pairs are always complete)."""
        self._chk(self.lib.ptgs_splat_reserve(self._h, int(pairs)), "ptgs_splat_reserve")

    def bvh_buffers(self) -> BvhBuffers:
        """Device pointers of the uploaded 4-wide BVH nodes and leaf-order triangle records."""
        b = BvhBuffers()
        self._chk(self.lib.ptgs_scene_get_bvh(self._h, C.byref(b)), "ptgs_scene_get_bvh")
        return b

    def splat_buffers(self) -> SplatBuffers:
        b = SplatBuffers()
        self._chk(self.lib.ptgs_splat_get_buffers(self._h, C.byref(b)), "ptgs_splat_get_buffers")
        return b

    def splat_tile_rows(self) -> tuple[int, int]:
        """ptgs_splat_get_tile_rows: (device pointer, row capacity) of the latest splat's fused slot rows
        (its front end's unsorted (depth bits << 32 | gaussian) pairs, tile t at t * capacity); (0, 0) when
        that frame ran the three-launch front end."""
        p, cap = C.c_void_p(), C.c_uint32()
        self._chk(self.lib.ptgs_splat_get_tile_rows(self._h, C.byref(p), C.byref(cap)), "ptgs_splat_get_tile_rows")
        return (p.value or 0), cap.value

    def splat_stage_ms(self) -> np.ndarray:
        """[preprocess+count, colscan, scatter, large-tile sort, 0, sort+blend] ms of the last splat
        (FLAG_TIME_STAGES)."""
        out = np.zeros(6, np.float32)
        self._chk(self.lib.ptgs_splat_stage_ms(self._h, _abi.fptr(out)), "ptgs_splat_stage_ms")
        return out

    def encode_srgb8(self, rgba32f, width: int, height: int, rgba8, stream=None):
        rc = self.lib.ptgs_encode_srgb8(self._h, _ptr(rgba32f), width, height, _ptr(rgba8), _stream(stream))
        self._chk(rc, "ptgs_encode_srgb8")

    # ---------------------------------------------------------------- memory helpers
    def copy_d2h(self, dst: np.ndarray, src_ptr: int, nbytes: int):
        self._chk(self.lib.ptgs_memcpy_d2h(self._h, dst.ctypes.data, src_ptr, nbytes), "ptgs_memcpy_d2h")

    def synchronize(self):
        self._chk(self.lib.ptgs_synchronize(self._h), "ptgs_synchronize")


def torus_push(model=None, major_radius: float = 3.5, minor_radius: float = 1.0, height: float = 3.0,
               mode: int = 0) -> RayPush:
    p = RayPush()
    m = np.eye(4, dtype=np.float32).reshape(16) if model is None else np.asarray(model, np.float32).reshape(16)
    p.model[:] = [float(x) for x in m]
    p.mode = mode
    p.major_radius = major_radius
    p.minor_radius = minor_radius
    p.height = height
    return p
