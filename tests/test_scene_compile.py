"""Scene compilation (the reference's GLSL code generator, Graphics.cpp:38-113 / 392-752, as table
compilers): the product compiler in librmr.so and the oracle's Python restatement must produce
identical tables, and must reject exactly the scenes whose generated GLSL does not compile."""
import glob
import json
import os

import pytest

from oracle import scene_compile
from raymarchrenderer_amd import abi
from raymarchrenderer_amd._lib import RMRError
from raymarchrenderer_amd.scene import CompiledScene

from .conftest import GOLDEN, SCENES

FILES = sorted(glob.glob(os.path.join(GOLDEN, "scenes", "*.scene")) + glob.glob(os.path.join(SCENES, "*.scene")))


@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f) for f in FILES])
@pytest.mark.parametrize("variant", ["rm1", "rm2", "rm3"])
def test_product_matches_oracle_compiler(path, variant):
    try:
        a = CompiledScene(path, variant).canonical()
    except RMRError as e:
        a = ("error", e.code)
    try:
        b = scene_compile.load_scene_file(path, variant).canonical()
    except scene_compile.SceneError:
        b = ("error", abi.ERRORS and -3)
    assert a == b


def test_stale_reference_scenes_fail_like_the_shader_compile():
    # material_test/object_test: shader_mix arity no longer matches RayMarch.glsl:346
    for name in ["material_test.scene", "object_test.scene"]:
        with pytest.raises(RMRError) as ei:
            CompiledScene(os.path.join(GOLDEN, "scenes", name), "rm1")
        assert ei.value.code == -3 and "shader_mix" in str(ei.value)


def test_v1_literal_quantisation():
    # std::to_string(float) keeps 6 decimals (Graphics.cpp:542,670)
    sc = {"materials": [{"id": 0, "total_vars": 2, "color": 0, "dir": 1,
                         "nodes": [{"name": "shader_diffuse", "inputs": [[0.1234567891, 1e-7, 2.5]], "outputs": [0, 1]}]}],
          "objects": [{"matID": 0, "total_vars": 1, "distance": 0,
                       "nodes": [{"name": "map_sphere", "inputs": [-1, [0.0000004, 1.0000004, 0], [1, 1, 1]], "outputs": [0]}]}]}
    t = CompiledScene(sc, "rm1").canonical()
    assert t["prims"][0][4] == (0.0, 1.0, 0.0)
    c = t["consts"][0]
    assert abs(c[0] - 0.123457) < 1e-7 and c[1] == 0.0 and c[2] == 2.5


def test_opu_order_and_program_objects():
    sc = {"materials": [{"id": 0, "total_vars": 1, "color": 0, "dir": -1,
                         "nodes": [{"name": "shader_emission", "inputs": [[1, 1, 1], [2, 2, 2]], "outputs": [0]}]}],
          "objects": [
              {"matID": 0, "total_vars": 3, "distance": 2,
               "nodes": [{"name": "domain_repeat", "inputs": [-1, [2, 0, 2]], "outputs": [0]},
                         {"name": "map_sphere", "inputs": [0, [0, 0.5, 0], [0.5, 0.5, 0.5]], "outputs": [1]},
                         {"name": "op_union", "inputs": [1, 1], "outputs": [2]}]},
              {"matID": 0, "total_vars": 1, "distance": 0,
               "nodes": [{"name": "map_box", "inputs": [-1, [0, -1, 0], [9, 0.1, 9]], "outputs": [0]}]}]}
    a = CompiledScene(sc, "rm1").canonical()
    b = scene_compile.compile_scene(sc, "rm1").canonical()
    assert a == b
    assert a["prims"][0][0] == abi.RMR_PRIM_PROGRAM and a["prims"][1][0] == abi.RMR_PRIM_BOX


@pytest.mark.parametrize("bad", [
    {"materials": [{"id": 1, "total_vars": 1, "nodes": []}]},                        # case 0 missing
    {"materials": [{"id": 0, "total_vars": 1, "nodes": [{"name": "nope", "inputs": [], "outputs": [0]}]}]},
    {"materials": [{"id": 0, "total_vars": 1, "color": 3, "nodes": []}]},           # vars[3] of vars[1]
    {"objects": [{"matID": 0, "total_vars": 1, "distance": 0,
                  "nodes": [{"name": "map_box", "inputs": [-1, [0, 0, 0]], "outputs": [0]}]}]},
])
def test_rejects_what_glsl_rejects(bad):
    with pytest.raises(RMRError):
        CompiledScene(bad, "rm1")
    with pytest.raises(scene_compile.SceneError):
        scene_compile.compile_scene(bad, "rm1")


def test_rm2_requires_mat_func_1_and_flattens_simple():
    t = CompiledScene(os.path.join(GOLDEN, "scenes", "simple.scene"), "rm2").canonical()
    codes = [o[0] for o in t["ops"]]
    assert codes == [abi.OP["V2_DIFFUSE"], abi.OP["V2_GLOSSY"], abi.OP["V2_FRESNEL"], abi.OP["V2_MIX"]]
    with pytest.raises(RMRError):
        CompiledScene(json.dumps({"materials": [{"id": 0, "constants": [[1, 1, 1]],
                                                  "nodes": [{"name": "shader_diffuse", "inputs": [[-1, 0]]}],
                                                  "output": 0}]}), "rm2")


def test_rm3_is_builtin_whatever_the_scene():
    a = CompiledScene(os.path.join(GOLDEN, "scenes", "default.scene"), "rm3").canonical()
    b = CompiledScene("", "rm3").canonical()
    assert a == b and len(a["prims"]) == 3
