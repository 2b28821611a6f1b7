"""ctypes binding of librmr.so (the C ABI in include/rmr.h).

librmr.so is built in-tree by raymarchrenderer_amd/csrc/Makefile (``__graft_entry__.build()``).
There is no fallback: if the library is missing, every entry point raises.
"""
import ctypes as C
import os

from . import abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "librmr.so")
# the diagnostic build (csrc/Makefile `diag`, -DRMR_DIAG=1): the same library plus the experiments'
# environment switches (RMR_GRID, RMR_JIT_OPTS, ...), for tools/ and the A/B tests
LIB_DIAG_PATH = os.path.join(HERE, "librmr_diag.so")
_libs = {}

EXPORTS = [
    "rmr_create", "rmr_destroy", "rmr_last_error", "rmr_build_info", "rmr_set_stream",
    "rmr_set_image_size", "rmr_get_image_size", "rmr_set_params", "rmr_get_params",
    "rmr_default_params", "rmr_set_view", "rmr_camera_view", "rmr_load_scene_json",
    "rmr_load_scene_tables", "rmr_load_builtin_scene", "rmr_reload", "rmr_render",
    "rmr_render_spp", "rmr_render_tiles", "rmr_read_accum", "rmr_write_accum",
    "rmr_accum_device_ptr", "rmr_bind_accum", "rmr_save_bmp", "rmr_encode_bmp",
    "rmr_save_accum", "rmr_load_accum", "rmr_sync", "rmr_get_stats", "rmr_reset_stats", "rmr_get_section_cycles", "rmr_get_counters", "rmr_set_culling",
    "rmr_set_kernel", "rmr_set_tuning", "rmr_set_grid_reserve", "rmr_trace_samples", "rmr_abi_sizes", "rmr_set_jit", "rmr_set_instrument", "rmr_jit_compile_scene", "rmr_set_env_map",
    "rmr_scene_compile", "rmr_scene_view", "rmr_scene_free", "rmr_display", "rmr_display_device",
    "rmr_srgb_thresholds", "rmr_candidate_grid", "rmr_set_call_batching", "rmr_set_launch_streams", "rmr_get_launch_streams",
]


class RMRError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s (%d): %s" % (abi.ERRORS.get(code, "RMR_E?"), code, msg))
        self.code = code


def build():
    import subprocess
    subprocess.check_call(["make", "-s", "-C", os.path.join(HERE, "csrc"), "-j8"])


def lib(diag=None):
    """The ctypes handle of librmr.so, or of librmr_diag.so with diag=True, or of the library file
    diag names (a str: another build of the same ABI, for same-process A/B runs). diag=None: the release
    library unless the environment selects the diagnostic one with RMR_LIB=diag (tools/ scripts;
    the selection is made here, in Python: the release library itself reads no such switch)."""
    if diag is None:
        diag = os.environ.get("RMR_LIB", "") == "diag"
    if isinstance(diag, str):   # a library file (tools/abrun.py: another build of the same ABI)
        path = os.path.abspath(diag)
    else:
        path = LIB_DIAG_PATH if diag else LIB_PATH
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        raise RuntimeError("%s not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
                           "(expected at %s)" % (os.path.basename(path), path))
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64, and once librmr has brought
    # in /opt/rocm's, torch can no longer initialise the GPU ("No HIP GPUs are available", measured on
    # the MI355X box). Loading torch first makes librmr bind to the runtime already in the process, so
    # torch tensors and rmr contexts can share one device (FrameRenderer, rmr_bind_accum).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(path)
    vp, fp, ip = C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_int)
    dp = C.POINTER(C.c_double)
    sig = {
        "rmr_create": (C.c_int, [C.POINTER(vp), C.c_int]),
        "rmr_destroy": (None, [vp]),
        "rmr_last_error": (C.c_char_p, [vp]),
        "rmr_build_info": (C.c_char_p, []),
        "rmr_set_stream": (C.c_int, [vp, vp]),
        "rmr_set_image_size": (C.c_int, [vp, C.c_int, C.c_int]),
        "rmr_get_image_size": (C.c_int, [vp, ip, ip]),
        "rmr_set_params": (C.c_int, [vp, C.POINTER(abi.Params)]),
        "rmr_get_params": (C.c_int, [vp, C.POINTER(abi.Params)]),
        "rmr_default_params": (None, [C.POINTER(abi.Params)]),
        "rmr_set_view": (C.c_int, [vp, fp, fp, fp, fp, fp]),
        "rmr_camera_view": (None, [dp, dp, C.c_float, C.c_float, fp, fp, fp, fp, fp]),
        "rmr_load_scene_json": (C.c_int, [vp, C.c_int, C.c_char_p, C.c_size_t]),
        "rmr_load_scene_tables": (C.c_int, [vp, C.POINTER(abi.Scene)]),
        "rmr_load_builtin_scene": (C.c_int, [vp, C.c_int]),
        "rmr_reload": (C.c_int, [vp]),
        "rmr_render": (C.c_int, [vp, C.c_float, C.c_float, C.c_float, C.c_float, C.c_float, C.c_uint32]),
        "rmr_render_spp": (C.c_int, [vp, fp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint32, C.c_uint32]),
        "rmr_render_tiles": (C.c_int, [vp, fp, C.POINTER(C.c_int32), C.c_int, C.c_int, C.c_uint32, C.c_uint32]),
        "rmr_read_accum": (C.c_int, [vp, fp, C.c_size_t]),
        "rmr_write_accum": (C.c_int, [vp, fp, C.c_size_t]),
        "rmr_accum_device_ptr": (vp, [vp]),
        "rmr_bind_accum": (C.c_int, [vp, vp, C.c_size_t]),
        "rmr_save_bmp": (C.c_int, [vp, C.c_char_p]),
        "rmr_encode_bmp": (C.c_int, [fp, C.c_int, C.c_int, C.c_char_p]),
        "rmr_save_accum": (C.c_int, [vp, C.c_char_p, C.c_uint32]),
        "rmr_load_accum": (C.c_int, [vp, C.c_char_p, C.POINTER(C.c_uint32)]),
        "rmr_sync": (C.c_int, [vp]),
        "rmr_get_stats": (C.c_int, [vp, C.POINTER(abi.Stats)]),
        "rmr_reset_stats": (C.c_int, [vp]),
        "rmr_get_section_cycles": (C.c_int, [vp, C.POINTER(C.c_uint64)]),
        "rmr_get_counters": (C.c_int, [vp, C.POINTER(C.c_uint64)]),
        "rmr_set_culling": (C.c_int, [vp, C.c_int]),
        "rmr_set_kernel": (C.c_int, [vp, C.c_int]),
        "rmr_set_tuning": (C.c_int, [vp, C.c_int, C.c_int, C.c_longlong]),
        "rmr_set_grid_reserve": (C.c_int, [vp, C.c_int]),
        "rmr_set_call_batching": (C.c_int, [vp, C.c_int]),
        "rmr_set_launch_streams": (C.c_int, [vp, C.c_int]),
        "rmr_get_launch_streams": (C.c_int, [vp]),
        "rmr_set_jit": (C.c_int, [vp, C.c_int]),
        "rmr_set_instrument": (C.c_int, [vp, C.c_int]),
        "rmr_set_env_map": (C.c_int, [vp, C.c_void_p, C.c_int, C.c_int]),
        "rmr_jit_compile_scene": (C.c_int, [C.c_int, C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t]),
        "rmr_trace_samples": (C.c_int, [vp, fp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint32, fp]),
        "rmr_abi_sizes": (C.c_int, [C.POINTER(C.c_int32), C.c_int]),
        "rmr_scene_compile": (C.c_int, [C.c_int, C.c_char_p, C.c_size_t, C.POINTER(vp), C.c_char_p, C.c_size_t]),
        "rmr_scene_view": (C.c_int, [vp, C.POINTER(abi.Scene)]),
        "rmr_scene_free": (None, [vp]),
        "rmr_display": (C.c_int, [vp] + [C.c_float] * 7 + [C.c_int, C.c_int, C.c_void_p, C.c_size_t]),
        "rmr_display_device": (C.c_int, [vp] + [C.c_float] * 7 + [C.c_int, C.c_int, C.c_void_p, C.c_size_t]),
        "rmr_srgb_thresholds": (C.c_int, [fp]),
        "rmr_candidate_grid": (C.c_int, [fp, C.c_int, C.c_int, C.c_double, C.c_double, C.c_double,
                                         C.POINTER(C.c_int32), fp, C.POINTER(C.c_uint32), C.c_size_t,
                                         C.POINTER(C.c_uint16), C.c_size_t]),
        # diagnostic library only (rmr_api.cpp RMR_DIAG): ray_exit at given rays
        "rmr_diag_ray_exit": (C.c_int, [vp, fp, C.c_int, fp, fp, C.c_int, ip]),
    }
    for name, (res, args) in sig.items():
        if not hasattr(L, name):   # (an older build given by path may lack a newer entry point)
            continue
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _libs[path] = L
    return L
