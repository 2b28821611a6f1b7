"""Context-free access to librmr's scene compiler (rmr_scene_compile): reference scene JSON ->
rmr tables, on the CPU, without a GPU context."""
import ctypes as C
import json
import os

from . import abi
from ._lib import RMRError, lib


class CompiledScene:
    def __init__(self, scene, variant):
        if isinstance(variant, str):
            variant = abi.VARIANTS[variant]
        if isinstance(scene, dict):
            text = json.dumps(scene)
        elif isinstance(scene, str) and os.path.exists(scene):
            text = open(scene).read()
        else:
            text = scene or ""
        b = text.encode()
        self._h = C.c_void_p()
        # the library is chosen once per handle: free (and view) go to the library that compiled it
        self._L = lib()
        err = C.create_string_buffer(512)
        rc = self._L.rmr_scene_compile(variant, b, len(b), C.byref(self._h), err, len(err))
        if rc != abi.RMR_OK:
            raise RMRError(rc, err.value.decode(errors="replace"))
        self.variant = variant
        self.view = abi.Scene()
        self._L.rmr_scene_view(self._h, C.byref(self.view))

    def __del__(self):
        try:
            if self._h:
                self._L.rmr_scene_free(self._h)
        except Exception:
            pass

    def canonical(self):
        s = self.view
        prims = [(p.type, p.mat_id, p.prog_begin, p.prog_end, tuple(p.c), p.dist_var, tuple(p.r), p.n_vars)
                 for p in (s.prims[i] for i in range(s.n_prims))]
        ops = [(o.code, tuple(o.inp), tuple(o.out)) for o in (s.ops[i] for i in range(s.n_ops))]
        consts = [tuple(s.consts[3 * i:3 * i + 3]) for i in range(s.n_consts)]
        mats = []
        if s.variant != abi.RMR_VARIANT_RM3:
            mats = [(m.defined, m.prog_begin, m.prog_end, m.n_vars, m.color_var, m.dir_var, m.inside_var, m.hit_var)
                    for m in (s.materials[i] for i in range(s.n_materials))]
        return {"prims": prims, "ops": ops, "consts": consts, "materials": mats,
                "v2": (s.v2_prog_begin, s.v2_prog_end, s.v2_n_slots)}
