"""oracle/oracle.py — TEST INFRASTRUCTURE: ctypes front-end of liboracle.so (the CPU oracle).

Import only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
import ctypes as C
import os
import subprocess

import numpy as np

from raymarchrenderer_amd import abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RMR_ORACLE_LIB") or os.path.join(HERE, "liboracle.so")   # (sanitizer test)
WAVE_LIB_PATH = os.path.join(HERE, "libcpu_wave.so")
_lib = None
_wave = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = load(LIB_PATH)
    return _lib


def wave_lib():
    """libcpu_wave.so (oracle/rmr_cpu_wave.c): bench.py's CPU baseline for RM1 scenes, the oracle's
    path 8 lanes at a time on AVX2, bitwise the oracle's results."""
    global _wave
    if _wave is None:
        if not os.path.exists(WAVE_LIB_PATH):
            build()
        _wave = load(WAVE_LIB_PATH)
        fp = C.POINTER(C.c_float)
        _wave.oracle_render_wave.argtypes = [C.c_void_p, fp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint32,
                                             C.c_uint32, fp, C.c_int, C.POINTER(C.c_uint64)]
        _wave.oracle_render_wave.restype = C.c_int
        _wave.oracle_render_wave_rows.argtypes = [C.c_void_p, fp, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int32),
                                                  C.c_int, C.c_uint32, C.c_uint32, fp, C.c_int, C.POINTER(C.c_uint64)]
        _wave.oracle_render_wave_rows.restype = C.c_int
    return _wave


def literal_lib():
    """The oracle built with the reference's literal expressions where the default build
    reformulates them (RMR_HEMI_ALGEBRAIC=0: randHemisphere through acos / sin / cos as RM1:270-304;
    RMR_MB_POLY=0: the power-8 Mandelbulb through angle doubling): oracle/_lit/liboracle_lit.so."""
    path = os.path.join(HERE, "_lit", "liboracle_lit.so")
    subprocess.check_call(["make", "-s", "-C", HERE, "lit"])
    return load(path)


def load(path):
    """dlopen one build of the oracle and declare its entry points."""
    L = C.CDLL(path)
    fp = C.POINTER(C.c_float)
    L.oracle_sample.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_float, fp, C.POINTER(C.c_uint64)]
    L.oracle_render.argtypes = [C.c_void_p, fp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint32,
                                C.c_uint32, fp, C.c_int, C.POINTER(C.c_uint64)]
    L.oracle_trace_samples.argtypes = [C.c_void_p, fp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint32,
                                       fp, C.c_int, C.POINTER(C.c_uint64)]
    for n in ["oracle_det_sin", "oracle_det_cos", "oracle_det_acos", "oracle_det_log", "oracle_det_exp"]:
        getattr(L, n).argtypes = [C.c_float]
        getattr(L, n).restype = C.c_float
    L.oracle_det_atan2.argtypes = [C.c_float, C.c_float]
    L.oracle_det_atan2.restype = C.c_float
    L.oracle_map.argtypes = [C.POINTER(abi.Scene), C.c_float, fp, fp]
    L.oracle_march.argtypes = [C.POINTER(abi.Scene), C.POINTER(abi.Params), fp, fp, C.c_float, fp]
    L.oracle_trace.argtypes = [C.POINTER(Job), C.c_int, C.c_int, C.c_float, fp, fp, fp]
    L.oracle_normal.argtypes = [C.POINTER(abi.Scene), C.c_float, fp, fp]
    L.oracle_rand_chain.argtypes = [C.c_int, C.c_int, C.c_float, fp, C.c_int, fp]
    L.oracle_hemisphere.argtypes = [C.c_int, C.c_int, C.c_float, C.c_float, fp, fp, fp, fp]
    L.oracle_wl2rgb.argtypes = [C.c_uint32, fp]
    return L


def _fp(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


class Job(C.Structure):
    _fields_ = [("scene", C.POINTER(abi.Scene)), ("params", abi.Params), ("view", C.c_float * 15),
                ("W", C.c_int), ("H", C.c_int), ("env", C.POINTER(C.c_float)), ("env_w", C.c_int),
                ("env_h", C.c_int)]


class Oracle:
    """One scene + params + view + image size, mirroring the GL state the reference renders with."""

    def __init__(self, tables, params, view, W, H, env=None):
        """env: optional envTex as an (h, w, 4) uint8 RGBA texture (used when params.use_env_tex)."""
        self.tables = tables
        self.scene = tables.to_ctypes()
        self.job = Job()
        self.job.scene = C.pointer(self.scene)
        self.job.params = params
        self.job.view[:] = [float(x) for x in np.asarray(view, np.float32).reshape(15)]
        self.job.W, self.job.H = W, H
        if env is not None:
            env = np.asarray(env, np.uint8)
            self._env = np.ascontiguousarray(env.astype(np.float32) / np.float32(255.0))  # GL unorm8
            self.job.env = self._env.ctypes.data_as(C.POINTER(C.c_float))
            self.job.env_h, self.job.env_w = env.shape[:2]
        self.W, self.H = W, H
        self.map_evals = 0

    def sample(self, px, py, time):
        out = np.zeros(3, np.float32)
        n = C.c_uint64(0)
        lib().oracle_sample(C.byref(self.job), px, py, C.c_float(time), _fp(out), C.byref(n))
        self.map_evals += n.value
        return out

    def render(self, times, rect=None, first_sample=0, accum=None, nthreads=0):
        times = np.ascontiguousarray(times, np.float32)
        x0, y0, x1, y1 = rect if rect is not None else (0, 0, self.W, self.H)
        if accum is None:
            accum = np.zeros((self.H, self.W, 4), np.float32)
        n = C.c_uint64(0)
        lib().oracle_render(C.byref(self.job), _fp(times), x0, y0, x1, y1, first_sample, len(times),
                            _fp(accum), nthreads, C.byref(n))
        self.map_evals += n.value
        return accum

    def render_wave(self, times, rect=None, first_sample=0, accum=None, nthreads=0):
        """render() through the 8-lane AVX2 wavefront (oracle/rmr_cpu_wave.c), RM1 scenes only (None
        otherwise): the same accumulator bit for bit, several times faster per core."""
        times = np.ascontiguousarray(times, np.float32)
        x0, y0, x1, y1 = rect if rect is not None else (0, 0, self.W, self.H)
        if accum is None:
            accum = np.zeros((self.H, self.W, 4), np.float32)
        n = C.c_uint64(0)
        rc = wave_lib().oracle_render_wave(C.byref(self.job), _fp(times), x0, y0, x1, y1, first_sample, len(times),
                                           _fp(accum), nthreads, C.byref(n))
        if rc != 0:
            return None
        self.map_evals += n.value
        return accum

    def render_wave_rows(self, times, rows, first_sample=0, accum=None, nthreads=0):
        """render_wave() of whole rows `rows` (distinct row indices) in one call: one batch of
        len(rows) x W x len(times) samples shared by every thread (fewer lane drains than a call per
        row). None for RM2 / RM3 scenes."""
        times = np.ascontiguousarray(times, np.float32)
        r = np.ascontiguousarray(rows, np.int32)
        if accum is None:
            accum = np.zeros((self.H, self.W, 4), np.float32)
        n = C.c_uint64(0)
        rc = wave_lib().oracle_render_wave_rows(C.byref(self.job), _fp(times), 0, self.W, 0,
                                                r.ctypes.data_as(C.POINTER(C.c_int32)), len(r), first_sample,
                                                len(times), _fp(accum), nthreads, C.byref(n))
        if rc == -1:
            return None
        if rc != 0:
            raise ValueError("oracle_render_wave_rows: row out of range")
        self.map_evals += n.value
        return accum

    def trace(self, gx, gy, time, o, d):
        """trace(o, d) of the reference for invocation (gx, gy), seed `time`, channels = 1."""
        out = np.zeros(3, np.float32)
        lib().oracle_trace(C.byref(self.job), gx, gy, C.c_float(time), _fp(np.asarray(o, np.float32)),
                           _fp(np.asarray(d, np.float32)), _fp(out))
        return out

    def trace_samples(self, times, rect=None, nthreads=0):
        times = np.ascontiguousarray(times, np.float32)
        x0, y0, x1, y1 = rect if rect is not None else (0, 0, self.W, self.H)
        out = np.zeros((len(times), y1 - y0, x1 - x0, 4), np.float32)
        n = C.c_uint64(0)
        lib().oracle_trace_samples(C.byref(self.job), _fp(times), x0, y0, x1, y1, len(times), _fp(out),
                                   nthreads, C.byref(n))
        self.map_evals += n.value
        return out


def det(name, *args):
    return getattr(lib(), "oracle_det_" + name)(*[C.c_float(a) for a in args])


def map_p(tables, p, max_dist=1000.0, L=None):
    s = tables.to_ctypes()
    P = np.asarray(p, np.float32)
    out = np.zeros(2, np.float32)
    (L or lib()).oracle_map(C.byref(s), max_dist, _fp(P), _fp(out))
    return out


def march(tables, o, d, dist_mult=1.0, params=None):
    s = tables.to_ctypes()
    prm = params if params is not None else abi.default_params()
    out = np.zeros(2, np.float32)
    lib().oracle_march(C.byref(s), C.byref(prm), _fp(np.asarray(o, np.float32)), _fp(np.asarray(d, np.float32)),
                       dist_mult, _fp(out))
    return out


def normal(tables, p, max_dist=1000.0):
    s = tables.to_ctypes()
    out = np.zeros(3, np.float32)
    lib().oracle_normal(C.byref(s), max_dist, _fp(np.asarray(p, np.float32)), _fp(out))
    return out


def rand_chain(gx, gy, time, cos):
    cos = np.ascontiguousarray(cos, np.float32).reshape(-1, 2)
    out = np.zeros(len(cos), np.float32)
    lib().oracle_rand_chain(gx, gy, time, _fp(cos), len(cos), _fp(out))
    return out


def hemisphere(gx, gy, time, rc0, s1, s2, n, L=None):
    out = np.zeros(3, np.float32)
    (L or lib()).oracle_hemisphere(gx, gy, time, rc0, _fp(np.asarray(s1, np.float32)), _fp(np.asarray(s2, np.float32)),
                            _fp(np.asarray(n, np.float32)), _fp(out))
    return out


def wl2rgb(wl):
    out = np.zeros(3, np.float32)
    lib().oracle_wl2rgb(wl, _fp(out))
    return out
