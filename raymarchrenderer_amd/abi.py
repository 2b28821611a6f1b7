"""ctypes mirror of include/rmr.h and include/rmr_tables.h (data layout only).

Every struct here must match the C declaration byte for byte; tests/test_abi.py checks the sizes
against the values the shared library reports.
"""
import ctypes as C

RMR_MAX_VARS = 16
RMR_MAX_PRIMS = 4096
RMR_MAX_OPS = 8192
RMR_MAX_CONSTS = 8192
RMR_MAX_MATERIALS = 256

RMR_VARIANT_RM1 = 1
RMR_VARIANT_RM2 = 2
RMR_VARIANT_RM3 = 3
VARIANTS = {"rm1": RMR_VARIANT_RM1, "rm2": RMR_VARIANT_RM2, "rm3": RMR_VARIANT_RM3}

RMR_PRIM_SPHERE = 1
RMR_PRIM_BOX = 2
RMR_PRIM_PROGRAM = 3
RMR_PRIM_MANDELBULB = 4

RMR_OPND_NONE = -1000000
RMR_OPND_P = -1
RMR_OPND_CONST0 = -2


def opnd_const(k):
    return RMR_OPND_CONST0 - k


# opcodes (rmr_opcode)
OP = {}
_obj = ["GET_X", "GET_Y", "GET_Z", "ADD", "SUB", "MUL", "DIV", "SIN", "COS", "MAP_SPHERE",
        "MAP_BOX", "UNION", "SUBTRACT", "INTERSECT", "DOMAIN_REPEAT", "MAP_MANDELBULB"]
for i, n in enumerate(_obj):
    OP[n] = 1 + i
_mat = ["M_FACING", "M_INSIDE", "M_ADD", "M_SUB", "M_MUL", "M_DIV", "M_MIX", "M_DIFFUSE",
        "M_GLOSSY", "M_REFRACTION", "M_VOLUME", "M_EMISSION"]
for i, n in enumerate(_mat):
    OP[n] = 32 + i
for i, n in enumerate(["V2_DIFFUSE", "V2_GLOSSY", "V2_FRESNEL", "V2_MIX"]):
    OP[n] = 64 + i

RMR_OK = 0
ERRORS = {-1: "RMR_E_INVALID", -2: "RMR_E_HIP", -3: "RMR_E_SCENE", -4: "RMR_E_IO",
          -5: "RMR_E_STATE", -6: "RMR_E_NOMEM", -7: "RMR_E_UNSUPPORTED"}


class Prim(C.Structure):
    _fields_ = [("type", C.c_int32), ("mat_id", C.c_float), ("prog_begin", C.c_int32),
                ("prog_end", C.c_int32), ("c", C.c_float * 3), ("dist_var", C.c_int32),
                ("r", C.c_float * 3), ("n_vars", C.c_int32)]


class Op(C.Structure):
    _fields_ = [("code", C.c_int32), ("inp", C.c_int32 * 7), ("out", C.c_int32 * 4)]


class Material(C.Structure):
    _fields_ = [("defined", C.c_int32), ("prog_begin", C.c_int32), ("prog_end", C.c_int32),
                ("n_vars", C.c_int32), ("color_var", C.c_int32), ("dir_var", C.c_int32),
                ("inside_var", C.c_int32), ("hit_var", C.c_int32)]


class Spectral(C.Structure):
    _fields_ = [("defined", C.c_int32), ("min_wave", C.c_uint32), ("max_wave", C.c_uint32),
                ("power", C.c_float), ("terminates", C.c_int32), ("pad", C.c_int32 * 3)]


class RM2Consts(C.Structure):
    _fields_ = [("albedo", (C.c_float * 3) * RMR_MAX_MATERIALS), ("light_pos", C.c_float * 3),
                ("light_power", C.c_float), ("node_mat_id", C.c_int32), ("pad", C.c_int32 * 3)]


class Scene(C.Structure):
    _fields_ = [("variant", C.c_int32),
                ("n_prims", C.c_int32), ("prims", C.POINTER(Prim)),
                ("n_ops", C.c_int32), ("ops", C.POINTER(Op)),
                ("n_consts", C.c_int32), ("consts", C.POINTER(C.c_float)),
                ("n_materials", C.c_int32), ("materials", C.POINTER(Material)),
                ("spectral", C.POINTER(Spectral)),
                ("spectral_sky", Spectral),
                ("v2_prog_begin", C.c_int32), ("v2_prog_end", C.c_int32), ("v2_n_slots", C.c_int32),
                ("rm2", C.POINTER(RM2Consts)),
                ("sky", C.c_float * 3)]


class Params(C.Structure):
    _fields_ = [("max_dist", C.c_float), ("max_steps", C.c_int32), ("max_bounces", C.c_int32),
                ("step_multiply", C.c_float), ("separate_channels", C.c_int32),
                ("use_env_tex", C.c_int32)]


def default_params(**kw):
    """Graphics::Render's uniform constants (Graphics.cpp:326-340)."""
    p = Params(1000.0, 512, 16, 0.5, 0, 0)
    for k, v in kw.items():
        setattr(p, k, v)
    return p


class Stats(C.Structure):
    _fields_ = [("map_evals", C.c_uint64), ("samples", C.c_uint64), ("trace_launches", C.c_uint64),
                ("trace_ms", C.c_double), ("fold_ms", C.c_double), ("flops_per_map", C.c_double),
                ("map_iters", C.c_uint64), ("shade_batches", C.c_uint64), ("jit_launches", C.c_uint64)]

# rmr_set_culling flags (rmr.h)
CULL_ESCAPE = 1
CULL_NPC = 2
CULL_APPROX = 4
CULL_EYE = 8
CULL_ALL = CULL_ESCAPE | CULL_NPC | CULL_APPROX | CULL_EYE
# rmr_set_instrument flags (rmr.h)
INSTR_COUNT_FLOPS = 1
