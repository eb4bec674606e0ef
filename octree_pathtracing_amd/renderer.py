"""HipRenderer -- the RenderingBackend / FrameInFlight surface over liboctpt.

Mirrors trait RenderingBackend (reference src/renderer/renderer_trait.rs:19-35),
FrameInFlight / FrameInFlightPoll (:37-46) and the progressive controls of TileRenderer
(src/renderer/tile_renderer.rs:139-296: set_target_spp, get_current_spp, get_image,
reset_render).  Every render goes to the gfx950 kernels; there is no CPU path.
"""
from __future__ import annotations

import ctypes as C
import enum

import numpy as np

from . import _lib
from .scene import Camera, RenderSettings, Scene


class RendererStatus(enum.IntEnum):  # tile_renderer.rs:30-60
    Running = 0
    Paused = 1
    Stopped = 2


class RendererMode(enum.Enum):  # tile_renderer.rs:62-66
    Preview = "Preview"
    PathTraced = "Path Traced"


class FrameInFlightPoll(enum.Enum):  # renderer_trait.rs:37-41
    Ready = "ready"
    NotReady = "not_ready"
    Cancelled = "cancelled"


class FrameInFlight:
    """One progressive pass batch in flight (renderer_trait.rs:42-46)."""

    def __init__(self, renderer: "HipRenderer", handle: C.c_void_p, accum: np.ndarray, rgba: np.ndarray,
                 spp_after: int):
        self._r = renderer
        self._h = handle
        self.accum = accum
        self.rgba = rgba
        self._spp_after = spp_after
        self._done = False

    def _finish(self, cancelled: bool = False):
        if not self._done:
            self._done = True
            self._r._frame_done(self, cancelled)
            self._r._lib.octpt_frame_release(self._h)

    def poll(self):
        """FrameInFlight::poll -> (FrameInFlightPoll, image | self | None)."""
        lib = self._r._lib
        st = lib.octpt_frame_poll(self._h)
        if st == _lib.NOT_READY:
            return FrameInFlightPoll.NotReady, self
        if st == _lib.CANCELLED:
            self._finish(cancelled=True)
            return FrameInFlightPoll.Cancelled, None
        _lib.check(lib, self._r._ctx, st)
        self._finish()
        return FrameInFlightPoll.Ready, self.rgba

    def wait_for(self) -> np.ndarray:
        """FrameInFlight::wait_for -> the tone-mapped image."""
        lib = self._r._lib
        st = lib.octpt_frame_wait(self._h)
        if st == _lib.CANCELLED:
            self._finish(cancelled=True)
            raise _lib.OctptError(st, "frame cancelled")
        _lib.check(lib, self._r._ctx, st)
        self._finish()
        return self.rgba

    def cancel(self) -> None:
        self._r._lib.octpt_frame_cancel(self._h)


class HipRenderer:
    """RenderingBackend implemented on one MI355X (HIP device `device`), or on several GPUs of the node
    through one context (`devices`: a list of HIP device ids, octpt_create_multi; ids may repeat)."""

    def __init__(self, device: int = 0, resolution=(500, 500), target_spp: int = 1, seed: int = 1,
                 max_depth: int = 5, lib_path=None, devices=None):
        # lib_path: another build of the same ABI (bench.py's issued-bytes diagnostic library)
        self._lib = _lib.load(lib_path) if lib_path else _lib.load()
        ctx = C.c_void_p()
        if devices is None:
            st = self._lib.octpt_create(int(device), C.byref(ctx))
            what = f"octpt_create(device={device})"
        else:
            devs = (C.c_int32 * len(devices))(*map(int, devices))
            st = self._lib.octpt_create_multi(devs, len(devices), C.byref(ctx))
            what = f"octpt_create_multi(devices={list(devices)})"
        if st != _lib.OK:
            raise _lib.OctptError(st, f"{what} failed: no usable gfx950 device")
        self._ctx = ctx
        self.device_entries = int(self._lib.octpt_device_entries(ctx))
        self._camera = Camera()
        self._resolution = tuple(resolution)
        self._mode = RendererMode.PathTraced
        self._status = RendererStatus.Stopped
        self.target_spp = target_spp
        self.seed = seed
        self.max_depth = max_depth
        self.branch_count = 1  # TileRenderer branch count; 1 = one path per sample
        self._scene_keep = None
        self._accum = None
        self._spp = 0
        self._in_flight = None
        self.set_camera(self._camera)

    # ------------------------------------------------------------ lifecycle
    def close(self):
        if self._ctx:
            self._lib.octpt_destroy(self._ctx)
            self._ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def _check(self, st):
        _lib.check(self._lib, self._ctx, st)

    # ------------------------------------------------------------ RenderingBackend
    def get_camera(self) -> Camera:
        return self._camera

    def set_camera(self, camera: Camera) -> None:
        c = _lib.Camera((C.c_float * 3)(*camera.eye), (C.c_float * 3)(*camera.direction),
                        (C.c_float * 3)(*camera.up), camera.fov, 0.0, 0.0)
        self._check(self._lib.octpt_set_camera(self._ctx, C.byref(c)))
        self._camera = camera
        self.reset_render()

    def which_backend(self) -> str:
        return "HIP (gfx950)"

    def set_resolution(self, resolution) -> None:
        self._resolution = (int(resolution[0]), int(resolution[1]))
        self.reset_render()

    def get_resolution(self):
        return self._resolution

    def get_status(self) -> RendererStatus:
        return self._status

    def set_mode(self, mode: RendererMode) -> None:
        """TileRenderer::set_mode (tile_renderer.rs:188-191): stops and restarts the accumulation."""
        self._mode = RendererMode(mode)
        self.reset_render()

    def get_mode(self) -> RendererMode:
        return self._mode

    def update_scene(self, *_args) -> None:
        """RenderingBackend::update_scene (egui hook) -- nothing to do for HIP."""

    def set_scene(self, scene: Scene) -> None:
        desc, keep = scene.to_desc()
        self._check(self._lib.octpt_scene_upload(self._ctx, C.byref(desc)))
        self._scene_keep = keep
        self.reset_render()

    def set_scene_built(self, scene: Scene, depth: int, compact: bool = False) -> None:
        """set_scene with the octree built on this GPU and kept there (octpt_scene_build_device): the
        device scene equals set_scene(scene) after scene.build_octree(depth, compact=compact), without
        the host round trip.  scene.octree is left untouched."""
        desc, keep = scene.to_desc(octree=False, depth=depth)
        self._check(self._lib.octpt_scene_build_device(self._ctx, C.byref(desc), _lib.BUILD_COMPACT if compact else 0))
        self._scene_keep = keep
        self.reset_render()

    def render_frame(self, spp_count: int | None = None) -> FrameInFlight:
        """RenderingBackend::render_frame: enqueue the next pass batch, return a FrameInFlight."""
        if self._in_flight is not None:
            raise RuntimeError("a frame is already in flight")
        W, H = self._resolution
        if self._accum is None:
            self._accum = np.zeros((H, W, 4), np.float32)
            self._accum[..., 3] = 1.0
        preview = self._mode is RendererMode.Preview
        n = spp_count if spp_count is not None else max(self.target_spp - self._spp, 1)
        if self.branch_count > 1:  # whole passes of the branch schedule (C20), as TileRenderer runs them
            n = branch_pass_end(self._spp, n, self.branch_count) - self._spp
        if preview:  # render_preview (tile_renderer.rs:339-374): one replacing pass, current_spp stays 0
            n = 0
        p = self.params(W, H, self._spp, n, preview=preview)
        rgba = np.zeros((H, W, 4), np.uint8)
        h = C.c_void_p()
        self._check(self._lib.octpt_render_async(self._ctx, C.byref(p), self._accum.ctypes.data_as(C.c_void_p),
                                                 rgba.ctypes.data_as(C.c_void_p), C.byref(h)))
        self._status = RendererStatus.Running
        f = FrameInFlight(self, h, self._accum, rgba, self._spp + n)
        self._in_flight = f
        return f

    def _frame_done(self, f: FrameInFlight, cancelled: bool = False):
        if not cancelled:  # a cancelled frame leaves the accumulation untouched
            self._spp = f._spp_after
        self._in_flight = None
        self._status = RendererStatus.Stopped

    # ------------------------------------------------------------ TileRenderer-style controls
    def reset_render(self) -> None:
        self._accum = None
        self._spp = 0

    def set_target_spp(self, spp: int) -> None:
        self.target_spp = max(self.target_spp, int(spp))

    def get_current_spp(self) -> int:
        return self._spp

    def get_float_image(self) -> np.ndarray | None:
        return self._accum

    # ------------------------------------------------------------ direct entry points
    def params(self, W, H, spp_start, spp_count, shard_index=0, shard_count=1, compact=False,
               megakernel=False, kernel_timing=False, preview=False) -> "_lib.RenderParams":
        flags = ((_lib.RENDER_SHARD_COMPACT if compact else 0) | (_lib.RENDER_MEGAKERNEL if megakernel else 0)
                 | (_lib.RENDER_KERNEL_TIMING if kernel_timing else 0) | (_lib.RENDER_PREVIEW if preview else 0))
        return _lib.RenderParams(W, H, spp_start, spp_count, self.max_depth, self.branch_count, self.seed,
                                 shard_index, shard_count, flags)

    def render(self, settings: RenderSettings, accum: np.ndarray | None = None, spp_start: int = 0,
               with_rgba: bool = False):
        """Synchronous progressive render into host memory: returns (accum[H,W,4], rgba or None)."""
        W, H = settings.width, settings.height
        if accum is None:
            accum = np.zeros((H, W, 4), np.float32)
            accum[..., 3] = 1.0
        accum = np.ascontiguousarray(accum, np.float32)
        rgba = np.zeros((H, W, 4), np.uint8) if with_rgba else None
        self.max_depth = settings.max_depth
        self.seed = settings.seed
        p = self.params(W, H, spp_start, settings.spp)
        self._check(self._lib.octpt_render(self._ctx, C.byref(p), accum.ctypes.data_as(C.c_void_p),
                                           rgba.ctypes.data_as(C.c_void_p) if rgba is not None else None))
        return accum, rgba

    def render_device(self, params: "_lib.RenderParams", d_accum: int, d_seg_count: int | None = None,
                      stream: int | None = None) -> None:
        """Enqueue a render on device buffers (raw device pointers, e.g. torch tensor.data_ptr())."""
        self._check(self._lib.octpt_render_device(self._ctx, C.byref(params), C.c_void_p(d_accum),
                                                  C.c_void_p(d_seg_count) if d_seg_count else None,
                                                  C.c_void_p(stream) if stream else None))

    def tonemap_device(self, d_accum: int, d_rgba: int, n_pixels: int, stream: int | None = None) -> None:
        self._check(self._lib.octpt_tonemap_device(self._ctx, C.c_void_p(d_accum), C.c_void_p(d_rgba), n_pixels,
                                                   C.c_void_p(stream) if stream else None))

    def unshard_device(self, W, H, shard_count, d_shards: int, stride: int, d_frame: int, stream=None) -> None:
        self._check(self._lib.octpt_unshard_device(self._ctx, W, H, shard_count, C.c_void_p(d_shards), stride,
                                                   C.c_void_p(d_frame), C.c_void_p(stream) if stream else None))

    def set_tile_order(self, W: int, H: int, order: np.ndarray | None) -> None:
        """The tile deal for W x H renders (octpt_set_tile_order): order[s] = the frame tile at dealing position s
        (shard k owns positions k + u * N); None = round robin."""
        if order is None:
            self._check(self._lib.octpt_set_tile_order(self._ctx, W, H, None))
            return
        o = np.ascontiguousarray(order, np.uint32)
        self._check(self._lib.octpt_set_tile_order(self._ctx, W, H, o.ctypes.data_as(C.c_void_p)))

    def intersect(self, rays: np.ndarray, last_prim=None, last_normal=None):
        """Batch Scene::hit: returns (t, prim, normal, steps)."""
        rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 6)
        n = len(rays)
        t = np.zeros(n, np.float32)
        prim = np.zeros(n, np.uint32)
        nrm = np.zeros((n, 3), np.float32)
        steps = np.zeros(n, np.uint32)
        lp = None if last_prim is None else np.ascontiguousarray(last_prim, np.uint32)
        ln = None if last_normal is None else np.ascontiguousarray(last_normal, np.float32)

        def P(a):
            return a.ctypes.data_as(C.c_void_p) if a is not None else None

        self._check(self._lib.octpt_intersect(self._ctx, P(rays), P(lp), P(ln), n, P(t), P(prim), P(nrm), P(steps)))
        return t, prim, nrm, steps

    def stats(self) -> dict:
        s = _lib.Stats()
        self._check(self._lib.octpt_get_stats(self._ctx, C.byref(s)))
        return s.as_dict()

    def reset_stats(self) -> None:
        self._check(self._lib.octpt_reset_stats(self._ctx))


def current_branch_count(current_spp: int, scene_branch_count: int) -> int:
    """TileRenderer::get_current_branch_count (tile_renderer.rs:196-206), f32 square root."""
    if current_spp < scene_branch_count:
        if current_spp <= int(np.sqrt(np.float32(scene_branch_count))):
            return 1
        return scene_branch_count - current_spp
    return scene_branch_count


def branch_pass_end(spp_start: int, spp_count: int, scene_branch_count: int) -> int:
    """The first pass boundary of the branch schedule at or after spp_start + spp_count (C20)."""
    spp = 0
    while spp < spp_start + spp_count:
        spp += current_branch_count(spp, scene_branch_count)
    return spp


def shard_pixels(W: int, H: int, shard_index: int, shard_count: int) -> int:
    return int(_lib.load().octpt_shard_pixels(W, H, shard_index, shard_count))


def balance_tiles(W: int, H: int, shard_count: int, seg_count: np.ndarray) -> np.ndarray:
    """octpt_balance_tiles: a tile order that balances shard_count shards by a previous render's per-pixel
    segment counts (W * H, image order)."""
    seg = np.ascontiguousarray(seg_count, np.uint32).reshape(-1)
    if seg.size != W * H:
        raise ValueError(f"seg_count holds {seg.size} pixels, not {W} x {H}")
    T = ((W + 7) // 8) * ((H + 7) // 8)
    order = np.zeros(T, np.uint32)
    st = _lib.load().octpt_balance_tiles(W, H, shard_count, seg.ctypes.data_as(C.c_void_p),
                                         order.ctypes.data_as(C.c_void_p))
    if st != 0:
        raise _lib.OctptError(st, "octpt_balance_tiles")
    return order
