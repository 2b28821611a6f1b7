"""oracle/scene_compile.py — TEST INFRASTRUCTURE: restatement of the reference's scene code generator.

The reference turns each JSON scene into GLSL text (Graphics.cpp:38-113 marker expansion, v1
object/material compiler Graphics.cpp:513-703, v2 material compiler Graphics.cpp:392-509 + 705-739)
and lets the GL driver reject what does not type-check. This module restates that generator as a
*table* compiler so the CPU oracle (liboracle.so) can run the same scenes, and so
tests/test_scene_compile.py can compare it with the product compiler in librmr.so. Anything the
generated GLSL would fail to compile on raises SceneError.
"""
import ctypes as C
import json
import struct

import numpy as np

from raymarchrenderer_amd import abi


class SceneError(ValueError):
    pass


def f32(x):
    return struct.unpack("f", struct.pack("f", float(x)))[0]


def quant_v1(x):
    """std::to_string(input.asFloat()) ("%f") then the GLSL float literal (Graphics.cpp:542,670)."""
    return f32(float("%f" % f32(x)))


# (n_in, n_out) of the GLSL node functions, RayMarch.glsl:121-215 (objects) / 313-479 (materials)
OBJ_NODES = {
    "misc_getX": ("GET_X", 1, 1), "misc_getY": ("GET_Y", 1, 1), "misc_getZ": ("GET_Z", 1, 1),
    "math_add": ("ADD", 2, 1), "math_subtract": ("SUB", 2, 1), "math_multiply": ("MUL", 2, 1),
    "math_divide": ("DIV", 2, 1), "math_sine": ("SIN", 1, 1), "math_cosine": ("COS", 1, 1),
    "map_sphere": ("MAP_SPHERE", 3, 1), "map_box": ("MAP_BOX", 3, 1),
    "op_union": ("UNION", 2, 1), "op_subtract": ("SUBTRACT", 2, 1), "op_intersect": ("INTERSECT", 2, 1),
    "domain_repeat": ("DOMAIN_REPEAT", 2, 1),
    "map_mandelbulb": ("MAP_MANDELBULB", 3, 1),  # rmr extension
}
MAT_NODES = {
    "misc_facing": ("M_FACING", 0, 1), "misc_inside": ("M_INSIDE", 0, 1),
    "math_add": ("M_ADD", 2, 1), "math_subtract": ("M_SUB", 2, 1), "math_multiply": ("M_MUL", 2, 1),
    "math_divide": ("M_DIV", 2, 1),
    "shader_mix": ("M_MIX", 7, 3), "shader_diffuse": ("M_DIFFUSE", 1, 2),
    "shader_glossy": ("M_GLOSSY", 2, 2), "shader_refraction": ("M_REFRACTION", 3, 3),
    "shader_volumeScatter": ("M_VOLUME", 2, 4), "shader_emission": ("M_EMISSION", 2, 1),
}
PRIM_FAST = {"map_sphere": abi.RMR_PRIM_SPHERE, "map_box": abi.RMR_PRIM_BOX,
             "map_mandelbulb": abi.RMR_PRIM_MANDELBULB}


def _is_int(v):
    return isinstance(v, int) and not isinstance(v, bool)


class Tables:
    """Scene tables + a ctypes rmr_scene view (buffers kept alive by this object)."""

    def __init__(self, variant):
        self.variant = variant
        self.prims = []
        self.ops = []
        self.consts = []
        self.materials = []
        self.spectral = []
        self.spectral_sky = (0, 0, 0, 0.0, 0)
        self.v2 = (0, 0, 0)
        self.rm2 = None
        self.sky = (f32(0.015), f32(0.015), f32(0.015))
        self._keep = []

    def const(self, v):
        self.consts.append(tuple(f32(x) for x in v))
        return abi.opnd_const(len(self.consts) - 1)

    def to_ctypes(self):
        s = abi.Scene()
        s.variant = self.variant
        P = (abi.Prim * max(1, len(self.prims)))()
        for i, p in enumerate(self.prims):
            P[i] = p
        O = (abi.Op * max(1, len(self.ops)))()
        for i, o in enumerate(self.ops):
            O[i] = o
        K = (C.c_float * max(3, 3 * len(self.consts)))()
        for i, c in enumerate(self.consts):
            K[3 * i:3 * i + 3] = list(c)
        M = (abi.Material * max(1, len(self.materials)))()
        for i, m in enumerate(self.materials):
            M[i] = m
        S = (abi.Spectral * max(1, len(self.spectral)))()
        for i, m in enumerate(self.spectral):
            S[i] = abi.Spectral(m[0], m[1], m[2], m[3], m[4])
        s.n_prims, s.prims = len(self.prims), C.cast(P, C.POINTER(abi.Prim))
        s.n_ops, s.ops = len(self.ops), C.cast(O, C.POINTER(abi.Op))
        s.n_consts, s.consts = len(self.consts), C.cast(K, C.POINTER(C.c_float))
        if self.variant == abi.RMR_VARIANT_RM3:
            s.n_materials = len(self.spectral)
        else:
            s.n_materials = len(self.materials)
        s.materials = C.cast(M, C.POINTER(abi.Material))
        s.spectral = C.cast(S, C.POINTER(abi.Spectral))
        sk = self.spectral_sky
        s.spectral_sky = abi.Spectral(sk[0], sk[1], sk[2], sk[3], sk[4])
        s.v2_prog_begin, s.v2_prog_end, s.v2_n_slots = self.v2
        R = abi.RM2Consts()
        if self.rm2 is not None:
            for i, a in self.rm2["albedo"].items():
                R.albedo[i][0], R.albedo[i][1], R.albedo[i][2] = a
            R.light_pos[:] = self.rm2["light_pos"]
            R.light_power = self.rm2["light_power"]
            R.node_mat_id = self.rm2["node_mat_id"]
        s.rm2 = C.pointer(R)
        s.sky[:] = list(self.sky)
        self._keep = [P, O, K, M, S, R]
        return s

    # canonical comparable form (for product-vs-oracle compile tests)
    def canonical(self):
        prims = [(p.type, p.mat_id, p.prog_begin, p.prog_end, tuple(p.c), p.dist_var, tuple(p.r), p.n_vars)
                 for p in self.prims]
        ops = [(o.code, tuple(o.inp), tuple(o.out)) for o in self.ops]
        mats = [(m.defined, m.prog_begin, m.prog_end, m.n_vars, m.color_var, m.dir_var, m.inside_var,
                 m.hit_var) for m in self.materials]
        return {"prims": prims, "ops": ops, "consts": list(self.consts), "materials": mats,
                "v2": self.v2}


def _op(code, ins=(), outs=()):
    o = abi.Op()
    o.code = abi.OP[code]
    for i in range(7):
        o.inp[i] = ins[i] if i < len(ins) else abi.RMR_OPND_NONE
    for i in range(4):
        o.out[i] = outs[i] if i < len(outs) else -1
    return o


def _vec_literal(v):
    v = list(v) + [0, 0, 0]
    return tuple(quant_v1(v[i]) if v[i] is not None else 0.0 for i in range(3))


def _total_vars(obj, what):
    tv = obj.get("total_vars")
    if not _is_int(tv) or tv <= 0:
        raise SceneError("%s: total_vars must be a positive int (vec3 vars[%r])" % (what, tv))
    if tv > abi.RMR_MAX_VARS:
        raise SceneError("%s: total_vars %d exceeds RMR_MAX_VARS" % (what, tv))
    return tv


def _check_var(k, tv, what):
    if not (0 <= k < tv):
        raise SceneError("%s: vars[%d] out of range for vec3 vars[%d]" % (what, k, tv))
    return k


def compile_objects_v1(t, objects):
    """obj_func_j generation, Graphics.cpp:647-702, + the //#OBJINSERT fold, Graphics.cpp:94-113."""
    for j, obj in enumerate(objects):
        what = "object %d" % j
        tv = _total_vars(obj, what)
        nodes = obj.get("nodes", [])
        dist = obj.get("distance")
        if not _is_int(dist):
            raise SceneError("%s: distance must be an int var index" % what)
        _check_var(dist, tv, what)
        mat = obj.get("matID", 0)
        mat = int(mat) if _is_int(mat) else 0
        # fast path: a single primitive node on p with literal centre/size
        if len(nodes) == 1 and nodes[0].get("name") in PRIM_FAST:
            n = nodes[0]
            ins, outs = n.get("inputs", []), n.get("outputs", [])
            if (len(ins) == 3 and ins[0] == -1 and isinstance(ins[1], list) and isinstance(ins[2], list)
                    and len(outs) == 1 and outs[0] == dist):
                p = abi.Prim()
                p.type = PRIM_FAST[n["name"]]
                p.mat_id = float(mat)
                p.c[:] = list(_vec_literal(ins[1]))
                p.r[:] = list(_vec_literal(ins[2]))
                p.dist_var = dist
                p.n_vars = tv
                t.prims.append(p)
                continue
        begin = len(t.ops)
        for n in nodes:
            name = n.get("name")
            if name not in OBJ_NODES:
                raise SceneError("%s: no GLSL function %r" % (what, name))
            code, n_in, n_out = OBJ_NODES[name]
            args = []
            for a in n.get("inputs", []):
                if isinstance(a, list):
                    args.append(("c", _vec_literal(a)))
                elif _is_int(a):
                    args.append(("p", None) if a == -1 else ("v", _check_var(a, tv, what)))
                else:
                    raise SceneError("%s: object input %r is not an int or literal" % (what, a))
            for a in n.get("outputs", []):
                if not _is_int(a):
                    raise SceneError("%s: object output %r is not an int" % (what, a))
                args.append(("v", _check_var(a, tv, what)))
            if len(args) != n_in + n_out:
                raise SceneError("%s: %s takes %d arguments, got %d" % (what, name, n_in + n_out, len(args)))
            ins, outs = [], []
            for i, (kind, val) in enumerate(args):
                if i < n_in:
                    ins.append(t.const(val) if kind == "c" else (abi.RMR_OPND_P if kind == "p" else val))
                else:
                    if kind != "v":
                        raise SceneError("%s: %s out argument is not an l-value" % (what, name))
                    outs.append(val)
            t.ops.append(_op(code, ins, outs))
        p = abi.Prim()
        p.type = abi.RMR_PRIM_PROGRAM
        p.mat_id = float(mat)
        p.prog_begin, p.prog_end = begin, len(t.ops)
        p.dist_var = dist
        p.n_vars = tv
        t.prims.append(p)


def compile_materials_v1(t, materials):
    """mat_func_<id> generation, Graphics.cpp:513-645, + //#CASEINSERT, Graphics.cpp:69-88."""
    n = len(materials)
    by_id = {}
    for m in materials:
        mid = m.get("id")
        if not _is_int(mid):
            raise SceneError("material id %r is not an int" % (mid,))
        if mid in by_id:
            raise SceneError("mat_func_%d redefined" % mid)
        by_id[mid] = m
    for j in range(n):
        if j not in by_id:
            raise SceneError("case %d calls undefined mat_func_%d" % (j, j))
    compiled = {}
    for m in materials:  # generation order = file order
        mid = m["id"]
        what = "material %d" % mid
        tv = _total_vars(m, what)
        names = {}
        begin = len(t.ops)
        for nd in m.get("nodes", []):
            name = nd.get("name")
            if name not in MAT_NODES:
                raise SceneError("%s: no GLSL function %s(RayData, ...)" % (what, name))
            code, n_in, n_out = MAT_NODES[name]
            args = []
            for a in nd.get("inputs", []):
                if isinstance(a, list):
                    args.append(("c", _vec_literal(a)))
                elif isinstance(a, str):
                    if a in names:
                        args.append(("v", names[a]))
                    # unknown names are silently dropped by the generator (Graphics.cpp:546-550)
                elif _is_int(a):
                    args.append(("v", a))
            for a in nd.get("outputs", []):
                if isinstance(a, str):
                    if a not in names:
                        names[a] = len(names)
                    args.append(("v", names[a]))
                elif _is_int(a):
                    args.append(("v", a))
            if len(args) != n_in + n_out:
                raise SceneError("%s: %s takes %d arguments, got %d" % (what, name, n_in + n_out, len(args)))
            ins, outs = [], []
            for i, (kind, val) in enumerate(args):
                if kind == "v":
                    _check_var(val, tv, what)
                if i < n_in:
                    ins.append(t.const(val) if kind == "c" else val)
                else:
                    if kind != "v":
                        raise SceneError("%s: %s out argument is not an l-value" % (what, name))
                    outs.append(val)
            t.ops.append(_op(code, ins, outs))

        def slot(key):
            v = m.get(key)
            if isinstance(v, str):
                k = names.setdefault(v, 0) if v in names else 0  # std::map operator[] default
                return _check_var(k, tv, what)
            if _is_int(v) and v != -1:
                return _check_var(v, tv, what)
            return -1

        mm = abi.Material()
        mm.defined = 1
        mm.prog_begin, mm.prog_end = begin, len(t.ops)
        mm.n_vars = tv
        mm.color_var, mm.dir_var = slot("color"), slot("dir")
        mm.inside_var, mm.hit_var = slot("inside"), slot("hit")
        compiled[mid] = mm
    t.materials = [compiled[j] for j in range(n)]


def compile_material_v2(t, m):
    """mat_func_<id> for RayMarch2.glsl, Graphics.cpp:705-739 + compileNode 412-463.

    Slots: 0 newDir, 1 reflectance, 2/3 mixDir[0]/mixRefl[0], 4/5 mixDir[1]/mixRefl[1], 6 mixFact.
    """
    consts = m.get("constants", [])
    nodes = m.get("nodes", [])
    what = "v2 material %r" % m.get("id")

    def const_ref(inp, want):
        if not (isinstance(inp, list) and len(inp) == 2 and inp[0] == -1):
            raise SceneError("%s: getInput() has no value for a node-linked input (Graphics.cpp:406)" % what)
        k = inp[1]
        if not (_is_int(k) and 0 <= k < len(consts)):
            raise SceneError("%s: constant %r missing" % (what, k))
        c = consts[k]
        if isinstance(c, list):
            if want == "scalar":
                raise SceneError("%s: vec3 constant where a float is required" % what)
            return t.const([f32(c[0]), f32(c[1]), f32(c[2])])
        if want == "vec3":
            raise SceneError("%s: float constant where a vec3 is required" % what)
        return t.const([f32(c), f32(c), f32(c)])

    def node(idx, out0, out1, depth, kind):
        if not (_is_int(idx) and 0 <= idx < len(nodes)):
            raise SceneError("%s: node %r missing" % (what, idx))
        nd = nodes[idx]
        name = nd.get("name")
        ins = nd.get("inputs", [])
        if name == "shader_diffuse":
            if kind != "vec":
                raise SceneError("%s: shader_diffuse feeds a float" % what)
            t.ops.append(_op("V2_DIFFUSE", [const_ref(ins[0], "vec3")], [out0, out1]))
        elif name == "shader_glossy":
            if kind != "vec":
                raise SceneError("%s: shader_glossy feeds a float" % what)
            col = const_ref(ins[0], "any")
            rough = const_ref(ins[1], "scalar")
            t.ops.append(_op("V2_GLOSSY", [col, rough], [out0, out1]))
        elif name == "shader_mix":
            if depth > 0 or kind != "vec":
                raise SceneError("%s: nested shader_mix does not compile (Graphics.cpp:428-430)" % what)
            for i, (o0, o1, k) in enumerate([(2, 3, "vec"), (4, 5, "vec"), (6, -1, "float")]):
                inp = ins[i] if i < len(ins) else [-1, 0]
                if inp[0] != -1:
                    node(inp[0], o0, o1, depth + 1, k)
            t.ops.append(_op("V2_MIX", [2, 3, 4, 5, 6], [out0, out1]))
        elif name == "misc_fresnel":
            if kind != "float":
                raise SceneError("%s: misc_fresnel output assigned to a vec3" % what)
            t.ops.append(_op("V2_FRESNEL", [], [out0]))
        # any other name: compileNode emits nothing (Graphics.cpp:412-463)

    begin = len(t.ops)
    node(m.get("output"), 0, 1, 0, "vec")
    return begin, len(t.ops)


RM2_BUILTIN_PRIMS = [("sphere", (0, 1, 0), (1, 1, 1), 1)]  # RayMarch2.glsl:139
RM3_BUILTIN_PRIMS = [("box", (0, -0.025, 0), (32, 0.05, 32), 1),  # RayMarch3.glsl:136
                     ("sphere", (0, 1, 0), (1, 1, 1), 2),  # RayMarch3.glsl:138
                     ("sphere", (6, 8, -4), (4, 4, 4), 0)]  # RayMarch3.glsl:140
RM3_SPECTRAL = [(1, 380, 780, f32(8.0), 1),    # mat_func_0, RayMarch3.glsl:251-281
                (1, 380, 780, f32(0.8), 0),    # mat_func_1, 283-313
                (1, 490, 590, f32(0.8), 0)]    # mat_func_2, 315-345
RM3_SKY = (1, 390, 830, f32(0.015), 0)         # RayMarch3.glsl:408-438


def _builtin_prims(t, lst):
    for kind, c, r, mat in lst:
        p = abi.Prim()
        p.type = abi.RMR_PRIM_SPHERE if kind == "sphere" else abi.RMR_PRIM_BOX
        p.mat_id = float(mat)
        p.c[:] = [f32(x) for x in c]
        p.r[:] = [f32(x) for x in r]
        p.dist_var = 0
        p.n_vars = 1
        t.prims.append(p)


def compile_scene(scene, variant):
    """scene: parsed JSON (dict) or JSON text; variant: 1/2/3 or 'rm1'/'rm2'/'rm3'."""
    if isinstance(variant, str):
        variant = abi.VARIANTS[variant]
    if isinstance(scene, (str, bytes)):
        scene = json.loads(scene)
    if scene is None:
        scene = {}
    t = Tables(variant)
    if variant == abi.RMR_VARIANT_RM1:
        compile_objects_v1(t, scene.get("objects", []))
        compile_materials_v1(t, scene.get("materials", []))
    elif variant == abi.RMR_VARIANT_RM2:
        _builtin_prims(t, RM2_BUILTIN_PRIMS)
        v2 = None
        for m in scene.get("materials", []):
            rng = compile_material_v2(t, m)
            if m.get("id") == 1:
                v2 = rng
        if v2 is None:
            raise SceneError("RayMarch2.glsl calls mat_func_1, which the scene does not define")
        t.v2 = (v2[0], v2[1], 7)
        t.rm2 = {"albedo": {0: (f32(0.8),) * 3, 1: (f32(0.8), f32(0.2), f32(0.2)), 2: (f32(0.2), f32(0.2), f32(0.8))},
                 "light_pos": [f32(2), f32(6), f32(-2)], "light_power": f32(50.0), "node_mat_id": 1}
    elif variant == abi.RMR_VARIANT_RM3:
        # RayMarch3.glsl has no insertion markers: the generated text is discarded (Graphics.cpp:742)
        _builtin_prims(t, RM3_BUILTIN_PRIMS)
        t.spectral = list(RM3_SPECTRAL)
        t.spectral_sky = RM3_SKY
    else:
        raise SceneError("unknown variant %r" % variant)
    if len(t.prims) > abi.RMR_MAX_PRIMS or len(t.ops) > abi.RMR_MAX_OPS or len(t.consts) > abi.RMR_MAX_CONSTS:
        raise SceneError("scene exceeds table limits")
    return t


def load_scene_file(path, variant):
    with open(path, "r") as f:
        return compile_scene(json.load(f), variant)


def flops_per_map(t):
    """Algorithmic flops of one map(): sphere 10, box 22, opU 2 per prim after the first;
    a Mandelbulb's fixed part 6 (its iterations are counted at run time, csrc/scene.cpp)."""
    f = 0
    for p in t.prims:
        f += {abi.RMR_PRIM_SPHERE: 10, abi.RMR_PRIM_BOX: 22, abi.RMR_PRIM_MANDELBULB: 6}.get(
            p.type, 10 * max(1, p.prog_end - p.prog_begin))
    return f + 2 * max(0, len(t.prims) - 1)


__all__ = ["SceneError", "Tables", "compile_scene", "load_scene_file", "flops_per_map", "quant_v1", "f32"]
_ = np  # numpy used by callers through Tables buffers
