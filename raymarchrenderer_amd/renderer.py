"""Python front-end of librmr.so: a Renderer context plus the reference's host interfaces.

`Renderer` owns one rmr_ctx (one GPU). `Graphics`, `Camera` and `Screen` mirror the reference's
static host classes (Graphics.h:15-134, Camera.h:4-32, Screen.h:4-15) with the same member names
and argument meaning, so driver code written against the reference reads the same here.
"""
import ctypes as C
import json
import math
import os
import time as _time

import numpy as np

from . import abi
from ._lib import RMRError, lib


def _fp(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _check(ctx, code, L=None):
    if code != abi.RMR_OK:
        msg = (L or lib()).rmr_last_error(ctx) if ctx else b""
        raise RMRError(code, (msg or b"").decode(errors="replace"))


def time_schedule(nspp, frame=0, first_sample=0):
    """Seed schedule of SURVEY §8d: time(frame f, sample s) = 1000*f + 0.016*s (as float32)."""
    s = np.arange(first_sample, first_sample + nspp, dtype=np.float64)
    return (1000.0 * frame + 0.016 * s).astype(np.float32)


def parity_schedule(nspp):
    """Seed schedule for converged-parity checks: time(s) = s * 0.016 / 256 (float32).

    The reference hash rand() (RayMarch.glsl:43-57) feeds dot(co, (12.9898, 78.233)), co ~ pixel +
    time, through mod(., 3.14) in float32: once |dot| reaches ~1e4-1e5 the argument of sin() is
    quantised to a few hundred values and the stream's distribution starts to depend on the
    driver's sin() rounding (measured: +8.7% Cornell-5 mean between two implementations at
    time ~ 4000). Small, densely spaced seeds keep both implementations in the well-conditioned
    regime, so their converged images are comparable."""
    s = np.arange(nspp, dtype=np.float64)
    return (s * (0.016 / 256.0)).astype(np.float32)


def camera_view(eye, direction, aspect, fov):
    """Camera::calculateRays + setView swap (librmr's rmr_camera_view): 15 floats in shader order."""
    e = (C.c_double * 3)(*[float(x) for x in eye])
    d = (C.c_double * 3)(*[float(x) for x in direction])
    out = np.zeros(15, np.float32)
    p = out.ctypes.data
    fsz = 4
    lib().rmr_camera_view(e, d, C.c_float(aspect), C.c_float(fov),
                          *[C.cast(p + 3 * i * fsz, C.POINTER(C.c_float)) for i in range(5)])
    return out


def default_camera_view(W, H):
    """Program.cpp:102 camera for an image of W x H."""
    m = math.sqrt(0.0 + 9.0 + 36.0)
    pi = np.float32(3.141592653)
    return camera_view((0.0, 4.0, -6.0), (0.0, -3.0 / m, 6.0 / m), float(W) / float(H), float(pi / np.float32(4)))


class Renderer:
    """One rmr context on one GPU (device index `device`)."""

    def __init__(self, device=0, width=1024, height=1024, diag=None):
        """diag=True: the context lives in the diagnostic build librmr_diag.so, which also reads the
        experiments' environment switches (RMR_GRID, RMR_JIT_OPTS, ...; tools/, A/B tests); the
        release librmr.so reads none. None: the release library unless RMR_LIB=diag (tools/)."""
        self._L = lib(diag=diag)
        self._ctx = C.c_void_p()
        rc = self._L.rmr_create(C.byref(self._ctx), device)
        if rc != abi.RMR_OK:
            raise RMRError(rc, "rmr_create failed (no HIP device %d?)" % device)
        self.set_image_size(width, height)
        self.reload()
        self.variant = None

    # -- lifetime --
    def close(self):
        if self._ctx:
            self._L.rmr_destroy(self._ctx)
            self._ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def ctx(self):
        return self._ctx

    @property
    def lib(self):
        """The ctypes library this context lives in (librmr.so, or librmr_diag.so with diag=True)."""
        return self._L

    def _chk(self, code):
        _check(self._ctx, code, self._L)

    # -- configuration --
    def set_image_size(self, w, h):
        self._chk(self._L.rmr_set_image_size(self._ctx, int(w), int(h)))

    def image_size(self):
        w, h = C.c_int(), C.c_int()
        self._chk(self._L.rmr_get_image_size(self._ctx, C.byref(w), C.byref(h)))
        return w.value, h.value

    def set_params(self, params=None, **kw):
        p = params if params is not None else abi.default_params()
        for k, v in kw.items():
            setattr(p, k, v)
        self._chk(self._L.rmr_set_params(self._ctx, C.byref(p)))

    def params(self):
        p = abi.Params()
        self._chk(self._L.rmr_get_params(self._ctx, C.byref(p)))
        return p

    def set_view(self, view15):
        v = np.ascontiguousarray(view15, np.float32).reshape(15)
        parts = [np.ascontiguousarray(v[3 * i:3 * i + 3]) for i in range(5)]
        self._chk(self._L.rmr_set_view(self._ctx, *[_fp(x) for x in parts]))
        self._view = v

    def load_scene(self, scene, variant):
        """scene: path, JSON text or dict in the reference's v1/v2 scene format."""
        if isinstance(variant, str):
            variant = abi.VARIANTS[variant]
        if isinstance(scene, dict):
            text = json.dumps(scene)
        elif isinstance(scene, str) and os.path.exists(scene):
            with open(scene, "r") as f:
                text = f.read()
        else:
            text = scene
        b = text.encode()
        self._chk(self._L.rmr_load_scene_json(self._ctx, variant, b, len(b)))
        self.variant = variant

    def load_builtin(self, variant):
        if isinstance(variant, str):
            variant = abi.VARIANTS[variant]
        self._chk(self._L.rmr_load_builtin_scene(self._ctx, variant))
        self.variant = variant

    def load_tables(self, tables):
        s = tables.to_ctypes()
        self._chk(self._L.rmr_load_scene_tables(self._ctx, C.byref(s)))
        self.variant = tables.variant

    def reload(self):
        self._chk(self._L.rmr_reload(self._ctx))

    def set_kernel(self, k):
        self._chk(self._L.rmr_set_kernel(self._ctx, int(k)))

    def set_tuning(self, shade_threshold=0, grid_per_cu=-1, samp_budget=0):
        self._chk(self._L.rmr_set_tuning(self._ctx, int(shade_threshold), int(grid_per_cu), int(samp_budget)))

    def set_grid_reserve(self, blocks):
        """Workgroups the persistent trace launch leaves free (rmr_set_grid_reserve; scheduling only)."""
        self._chk(self._L.rmr_set_grid_reserve(self._ctx, int(blocks)))
        self._grid_reserve = int(blocks)

    @property
    def grid_reserve(self):
        """The reserve last set through this object (0, the context's default, until then)."""
        return getattr(self, "_grid_reserve", 0)

    def set_env_map(self, rgba8):
        """envTex for skyColor (used with params use_env_tex=1): (h, w, 4) uint8, row 0 = up. None clears."""
        if rgba8 is None:
            self._chk(self._L.rmr_set_env_map(self._ctx, None, 0, 0))
            return
        a = np.ascontiguousarray(rgba8, np.uint8)
        self._env = a
        self._chk(self._L.rmr_set_env_map(self._ctx, a.ctypes.data, a.shape[1], a.shape[0]))

    def set_jit(self, mode):
        """hipRTC per-scene kernel specialisation: 0 off, 1 always, 2 auto (large launches)."""
        self._chk(self._L.rmr_set_jit(self._ctx, int(mode)))

    def set_instrument(self, flags):
        """Instrumented specialised kernels (abi.INSTR_*; rmr_set_instrument): the same images, extra
        counters (INSTR_COUNT_FLOPS: executed flops per map() in counters() [11..13])."""
        self._chk(self._L.rmr_set_instrument(self._ctx, int(flags)))

    def set_culling(self, flags):
        """Exact work-skipping switches (abi.CULL_*; results are bit-identical either way)."""
        self._chk(self._L.rmr_set_culling(self._ctx, int(flags)))

    def set_stream(self, hip_stream_handle):
        self._chk(self._L.rmr_set_stream(self._ctx, C.c_void_p(hip_stream_handle)))

    # -- rendering --
    def render(self, time, vmin, vmax, current_sample):
        """Graphics::Render(currentTime, min, max, currentSample)."""
        self._chk(self._L.rmr_render(self._ctx, float(time), float(vmin[0]), float(vmin[1]),
                                           float(vmax[0]), float(vmax[1]), int(current_sample)))

    def set_call_batching(self, mode):
        """rmr_set_call_batching: 1 on, 0 off, -1 auto (the default: on while the context owns its stream
        and accumulator). Batched render() calls go to the GPU together at the next other call."""
        self._chk(self._L.rmr_set_call_batching(self._ctx, int(mode)))

    def set_launch_streams(self, n):
        """rmr_set_launch_streams: n >= 2 (the library's default: 2, or 4 with 8 or more hardware queues)
        overlaps consecutive trace launches on n private streams (one sample-plane buffer each); 0 runs
        them on the context's stream. Same bits."""
        self._chk(self._L.rmr_set_launch_streams(self._ctx, int(n)))

    @property
    def launch_streams(self):
        """rmr_get_launch_streams: the context's launch streams (default 2, or 4 with 8 or more hardware
        queues per process)."""
        return int(self._L.rmr_get_launch_streams(self._ctx))

    def render_spp(self, times, rect=None, first_sample=0):
        times = np.ascontiguousarray(times, np.float32)
        if rect is None:
            w, h = self.image_size()
            rect = (0, 0, w, h)
        x0, y0, x1, y1 = rect
        self._chk(self._L.rmr_render_spp(self._ctx, _fp(times), x0, y0, x1, y1, int(first_sample), len(times)))

    def render_tiles(self, times, tiles_xy, tile_size, first_sample=0):
        times = np.ascontiguousarray(times, np.float32)
        t = np.ascontiguousarray(tiles_xy, np.int32).reshape(-1, 2)
        self._chk(self._L.rmr_render_tiles(self._ctx, _fp(times), t.ctypes.data_as(C.POINTER(C.c_int32)),
                                                 len(t), int(tile_size), int(first_sample), len(times)))

    def trace_samples(self, times, rect):
        times = np.ascontiguousarray(times, np.float32)
        x0, y0, x1, y1 = rect
        out = np.zeros((len(times), y1 - y0, x1 - x0, 4), np.float32)
        self._chk(self._L.rmr_trace_samples(self._ctx, _fp(times), x0, y0, x1, y1, len(times), _fp(out)))
        return out

    def sync(self):
        self._chk(self._L.rmr_sync(self._ctx))

    def read_accum(self):
        w, h = self.image_size()
        out = np.zeros((h, w, 4), np.float32)
        self._chk(self._L.rmr_read_accum(self._ctx, _fp(out), out.nbytes))
        return out

    def write_accum(self, a):
        a = np.ascontiguousarray(a, np.float32)
        self._chk(self._L.rmr_write_accum(self._ctx, _fp(a), a.nbytes))

    def accum_device_ptr(self):
        return self._L.rmr_accum_device_ptr(self._ctx)

    def bind_accum(self, dev_ptr, nbytes):
        self._chk(self._L.rmr_bind_accum(self._ctx, C.c_void_p(dev_ptr), int(nbytes)))

    def save_bmp(self, path):
        self._chk(self._L.rmr_save_bmp(self._ctx, path.encode()))

    def save_accum(self, path, samples_done):
        self._chk(self._L.rmr_save_accum(self._ctx, path.encode(), int(samples_done)))

    def load_accum(self, path):
        n = C.c_uint32()
        self._chk(self._L.rmr_load_accum(self._ctx, path.encode(), C.byref(n)))
        return n.value

    def display(self, centre, zoom, vmin, vmax, screen=None, screen_size=None):
        """Graphics::Display(centre, zoom, min, max) headless (rmr_display): the accumulator drawn into
        an RGBA8 screen image (h, w, 4) uint8, row 0 = top. `screen` is the image behind it (kept
        where the quad draws alpha 0); without it a zeroed image of `screen_size` (w, h)."""
        if screen is None:
            w, h = screen_size
            screen = np.zeros((int(h), int(w), 4), np.uint8)
        screen = np.ascontiguousarray(screen, np.uint8)
        if screen.ndim != 3 or screen.shape[2] != 4:
            raise ValueError("display: screen must be an (h, w, 4) RGBA8 image, got shape %s" % (screen.shape,))
        h, w = screen.shape[:2]
        self._chk(self._L.rmr_display(self._ctx, float(centre[0]), float(centre[1]), float(zoom),
                                            float(vmin[0]), float(vmin[1]), float(vmax[0]), float(vmax[1]),
                                            w, h, screen.ctypes.data, screen.nbytes))
        return screen

    def display_device(self, centre, zoom, vmin, vmax, dev, screen_w, screen_h, nbytes=None):
        """rmr_display_device: the same into a device RGBA8 buffer on the renderer's stream. `dev` is a
        torch tensor on the GPU (its size is numel * element_size) or a raw device pointer, which needs
        `nbytes`, the buffer's size in bytes (the library checks it against screen_w * screen_h * 4)."""
        if hasattr(dev, "data_ptr"):
            if not dev.is_contiguous():
                raise ValueError("display_device: the tensor must be contiguous")
            size = dev.numel() * dev.element_size()
            if nbytes is not None and int(nbytes) > size:
                raise ValueError("display_device: nbytes %d exceeds the tensor's %d bytes" % (nbytes, size))
            nbytes = size if nbytes is None else int(nbytes)
            dev_ptr = dev.data_ptr()
        else:
            if nbytes is None:
                raise ValueError("display_device: a raw device pointer needs nbytes (the buffer's size in bytes)")
            dev_ptr = int(dev)
        self._chk(self._L.rmr_display_device(self._ctx, float(centre[0]), float(centre[1]), float(zoom),
                                                   float(vmin[0]), float(vmin[1]), float(vmax[0]), float(vmax[1]),
                                                   int(screen_w), int(screen_h), C.c_void_p(dev_ptr), int(nbytes)))

    def stats(self):
        s = abi.Stats()
        self._chk(self._L.rmr_get_stats(self._ctx, C.byref(s)))
        return s

    def reset_stats(self):
        self._chk(self._L.rmr_reset_stats(self._ctx))

    def counters(self):
        """The kernels' 16 raw device counters (rmr_get_counters; rmr_trace.h documents the slots)."""
        raw = (C.c_uint64 * 16)()
        self._chk(self._L.rmr_get_counters(self._ctx, raw))
        return [int(v) for v in raw]


def jit_compile_scene(scene, variant, diag=None):
    """Compile the hipRTC-specialised trace kernel of a scene (no GPU needed). Returns the
    code-object key; raises RMRError with the compiler log on failure. diag: through the
    diagnostic build (which reads the experiments' RMR_JIT_* environment switches)."""
    if isinstance(variant, str):
        variant = abi.VARIANTS[variant]
    if scene is None:
        text = b""
    elif isinstance(scene, dict):
        text = json.dumps(scene).encode()
    elif os.path.exists(scene):
        text = open(scene, "rb").read()
    else:
        text = scene.encode()
    log = C.create_string_buffer(65536)
    rc = lib(diag=diag).rmr_jit_compile_scene(int(variant), text or None, len(text), log, len(log))
    if rc != abi.RMR_OK:
        raise RMRError(rc, log.value.decode(errors="replace"))
    return log.value.decode()


def encode_bmp(rgba, path):
    """Graphics::SaveImage encoding of a host RGBA32F image (h, w, 4)."""
    a = np.ascontiguousarray(rgba, np.float32)
    h, w = a.shape[:2]
    rc = lib().rmr_encode_bmp(_fp(a), w, h, path.encode())
    if rc != abi.RMR_OK:
        raise RMRError(rc, "rmr_encode_bmp(%s)" % path)


# ------------------------------------------------------------------------------------------
# Reference-shaped facades
# ------------------------------------------------------------------------------------------
class Screen:
    """Screen.h:4-15 — static screen size / window position / delta time."""
    _size = (0.0, 0.0)
    _pos = (0.0, 0.0)
    _dt = 0.0

    @staticmethod
    def setScreenSize(size):
        Screen._size = tuple(size)

    @staticmethod
    def getScreenSize():
        return Screen._size

    @staticmethod
    def setWindowPos(pos):
        Screen._pos = tuple(pos)

    @staticmethod
    def getWindowPos():
        return Screen._pos

    @staticmethod
    def getDeltaTime():
        return Screen._dt

    @staticmethod
    def setDeltaTime(t):
        if t != 0:  # Screen.cpp:35-40
            Screen._dt = t


class Graphics:
    """Graphics.h:118-133 static interface over one Renderer (variant selectable; the reference
    hard-wires RayMarch3, Graphics.cpp:272)."""
    _r = None
    _materials = []
    _objects = []
    _size = (1024, 1024)
    variant = abi.RMR_VARIANT_RM3
    device = 0

    @staticmethod
    def Init():
        Graphics._r = Renderer(Graphics.device, *Graphics._size)
        Graphics.Reload()

    @staticmethod
    def _scene_dict():
        return {"materials": list(Graphics._materials), "objects": list(Graphics._objects)}

    @staticmethod
    def Reload():
        r = Graphics._r
        if Graphics.variant == abi.RMR_VARIANT_RM3:
            r.load_builtin(abi.RMR_VARIANT_RM3)
        else:
            r.load_scene(Graphics._scene_dict(), Graphics.variant)
        r.set_image_size(*Graphics._size)
        r.reload()

    @staticmethod
    def Render(currentTime, vmin, vmax, currentSample):
        Graphics._r.render(currentTime, vmin, vmax, currentSample)

    @staticmethod
    def SaveImage(path):
        Graphics._r.save_bmp(path)

    @staticmethod
    def Display(centre, zoom, vmin, vmax, screen=None):
        """Graphics::Display (Graphics.cpp:356-390) into a screen image of Screen.getScreenSize()."""
        size = tuple(int(v) for v in Screen.getScreenSize())
        return Graphics._r.display(centre, zoom, vmin, vmax, screen=screen, screen_size=size)

    @staticmethod
    def addMaterial(material):
        Graphics._materials.append(material)

    @staticmethod
    def addObject(obj):
        Graphics._objects.append(obj)

    @staticmethod
    def clearScene():
        Graphics._materials = []
        Graphics._objects = []

    @staticmethod
    def setImageSize(size):
        Graphics._size = (int(size[0]), int(size[1]))
        if Graphics._r is not None:
            Graphics._r.set_image_size(*Graphics._size)

    @staticmethod
    def getImageSize():
        return Graphics._size

    @staticmethod
    def setView(eye, ray00, ray01, ray10, ray11):
        """Same argument order as the reference (Graphics.cpp:827): uniform ray10 <- 3rd arg... note
        the reference binds the 3rd parameter (named ray01) to the uniform "ray01"."""
        v = np.array(list(eye) + list(ray00) + list(ray01) + list(ray10) + list(ray11), np.float32)
        Graphics._r.set_view(v)


class Camera:
    """Camera.h:4-32 — corner-ray camera; calculateRays() pushes the view to Graphics."""

    def __init__(self, eyePos=(0.0, 4.0, -6.0), lookDir=None, aspect=1.0, fov=None):
        if lookDir is None:
            m = math.sqrt(45.0)
            lookDir = (0.0, -3.0 / m, 6.0 / m)
        self.eye = tuple(float(x) for x in eyePos)
        self.dir = tuple(float(x) for x in lookDir)
        self.aspect = float(aspect)
        self.fov = float(np.float32(3.141592653) / np.float32(4)) if fov is None else float(fov)
        self.calculateRays()

    def setAspect(self, a):
        self.aspect = float(a)

    def calculateRays(self):
        v = camera_view(self.eye, self.dir, self.aspect, self.fov)
        # v is already in uniform order; Graphics.setView(eye, ray00, ray10, ray01, ray11) as
        # Camera.cpp:101 calls it maps to the same uniforms.
        if Graphics._r is not None:
            Graphics._r.set_view(v)
        self.view = v
        return v


def tile_spiral(gridW, gridH):
    """The outward spiral tile order of Program.cpp:113-115 / 203-222."""
    x = int(math.ceil(gridW / 2.0)) - 1
    y = int(math.ceil(gridH / 2.0)) - 1
    d = (-1, 0)
    passed, last, dist = 0, 0, 0
    order = []
    while passed < gridW * gridH:
        order.append((x, y))
        x -= gridW // 2
        y -= gridH // 2
        if dist * 2 == passed - last:
            dist += 1
            last = passed
            d = (d[1], -d[0])
        elif dist == passed - last:
            d = (d[1], -d[0])
        passed += 1
        x += d[0]
        y += d[1]
        x += gridW // 2
        y += gridH // 2
    return order


def save_name(now=None):
    """Program.cpp:71-84 file name: output\\%Y-%m-%d_%H-%M-%S.bmp."""
    t = _time.localtime(now)
    return _time.strftime("%Y-%m-%d_%H-%M-%S", t) + ".bmp"


def srgb_thresholds():
    """rmr_srgb_thresholds: the 256 linear-space decision points of the display's sRGB encode."""
    out = np.zeros(256, np.float32)
    rc = lib().rmr_srgb_thresholds(_fp(out))
    if rc != abi.RMR_OK:
        raise RMRError(rc, "rmr_srgb_thresholds")
    return out


def candidate_grid(prims, n_large, E, target=0.0, pad=0.0):
    """rmr_candidate_grid (test hook, no GPU): the nearest-primitive cache's candidate grid for
    `prims` (n x 8 float32 rows in leaf order: c.xyz, r.xyz, type, mat_id; the first n_large
    evaluated everywhere). Returns a dict with dim, lo, inv, sbox, eps, margin, cells (n_cells x 2
    uint32) and list (uint16), or None when no grid applies."""
    prims = np.ascontiguousarray(prims, np.float32)
    n = prims.shape[0]
    idims = (C.c_int32 * 5)()
    geom = np.zeros(12, np.float32)
    rc = lib().rmr_candidate_grid(_fp(prims), n, int(n_large), float(E), float(target), float(pad), idims, _fp(geom),
                                  None, 0, None, 0)
    if rc not in (abi.RMR_OK, -1):   # -1 RMR_E_INVALID: buffers not given yet (sizes returned)
        raise RMRError(rc, "rmr_candidate_grid")
    if not idims[4]:
        return None
    ncell = idims[0] * idims[1] * idims[2]
    cells = np.zeros(2 * ncell, np.uint32)
    lst = np.zeros(max(1, idims[3]), np.uint16)
    rc = lib().rmr_candidate_grid(_fp(prims), n, int(n_large), float(E), float(target), float(pad), idims, _fp(geom),
                                  cells.ctypes.data_as(C.POINTER(C.c_uint32)), cells.size,
                                  lst.ctypes.data_as(C.POINTER(C.c_uint16)), lst.size)
    if rc != abi.RMR_OK:
        raise RMRError(rc, "rmr_candidate_grid")
    return {"dim": (idims[0], idims[1], idims[2]), "lo": geom[0:3].copy(), "inv": geom[3], "sbox": geom[4:10].copy(),
            "eps": float(geom[10]), "margin": float(geom[11]), "cells": cells.reshape(-1, 2), "list": lst[:idims[3]]}
