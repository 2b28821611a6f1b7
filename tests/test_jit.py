"""hipRTC per-scene specialisation of the trace kernel (rmr_jit.cpp; the reference's per-scene
shader recompilation, Graphics::Reload). CPU: the generated source compiles for gfx950 for every
scene family. GPU: the specialised kernel is bitwise equal to the oracle and to the table-driven
kernels."""
import os

import numpy as np
import pytest

from oracle import camera, oracle, scene_compile
from oracle.envmap import synthetic_env
from raymarchrenderer_amd import abi, time_schedule
from raymarchrenderer_amd.renderer import jit_compile_scene

from .conftest import GOLDEN, SCENES

SCENE_CASES = [
    ("rm1_cornell5_b4", os.path.join(SCENES, "cornell5.scene"), "rm1", {"max_bounces": 4}),
    ("rm1_sphere1_b1", os.path.join(SCENES, "sphere1.scene"), "rm1", {"max_bounces": 1}),
    ("rm1_default", os.path.join(GOLDEN, "scenes", "default.scene"), "rm1", {}),
    ("rm1_glass", os.path.join(GOLDEN, "scenes", "glass_test.scene"), "rm1", {}),
    ("rm1_mandelbulb_b2", os.path.join(SCENES, "mandelbulb.scene"), "rm1", {"max_bounces": 2}),
    ("rm1_csg256_b4", os.path.join(SCENES, "csg256.scene"), "rm1", {"max_bounces": 4}),
    ("rm2_simple", os.path.join(GOLDEN, "scenes", "simple.scene"), "rm2", {}),
    ("rm3_builtin", None, "rm3", {}),
    ("rm1_sphere1_env", os.path.join(SCENES, "sphere1.scene"), "rm1", {"max_bounces": 4, "use_env_tex": 1}),
    ("rm1_csg_nodes_b4", os.path.join(SCENES, "csg_nodes.scene"), "rm1", {"max_bounces": 4}),
    ("rm1_csg64_b4", os.path.join(SCENES, "csg64.scene"), "rm1", {"max_bounces": 4}),
]
IDS = [c[0] for c in SCENE_CASES]


@pytest.mark.parametrize("name,path,variant,overrides", SCENE_CASES, ids=IDS)
def test_jit_source_compiles_for_gfx950(tmp_path, monkeypatch, name, path, variant, overrides):
    if name.endswith("_env"):
        pytest.skip("same generated source as the scene without the env map (the sky is a kernel parameter)")
    monkeypatch.setenv("RMR_JIT_CACHE", str(tmp_path))
    key = jit_compile_scene(path, variant)
    assert len(key) == 16
    blob = tmp_path / (key + ".hsaco")
    assert blob.exists() and blob.stat().st_size > 1000
    assert jit_compile_scene(path, variant) == key   # cached, same key


def test_jit_scheduler_directive(tmp_path, monkeypatch):
    """The inline approximate-map kernels (Cornell-5) carry an `//@opts` scheduler directive
    (rmr_jit.cpp): it reaches hipRTC (another code object under another key); RMR_JIT_SCHED=0 drops it
    in the diagnostic build."""
    path = os.path.join(SCENES, "cornell5.scene")
    monkeypatch.setenv("RMR_JIT_CACHE", str(tmp_path))
    k_on = jit_compile_scene(path, "rm1", diag=True)
    monkeypatch.setenv("RMR_JIT_SCHED", "0")
    k_off = jit_compile_scene(path, "rm1", diag=True)
    assert k_on != k_off
    on, off = (tmp_path / (k_on + ".hsaco")).read_bytes(), (tmp_path / (k_off + ".hsaco")).read_bytes()
    assert on != off


def test_release_library_ignores_environment(tmp_path, monkeypatch):
    """The release librmr.so reads no environment switch but RMR_JIT_CACHE: with the experiments'
    switches set (every one the diagnostic build reads), it compiles the same code object as without
    them, and their names are not in the binary; librmr_diag.so does read them."""
    from raymarchrenderer_amd._lib import LIB_DIAG_PATH, LIB_PATH
    path = os.path.join(SCENES, "cornell5.scene")
    monkeypatch.setenv("RMR_JIT_CACHE", str(tmp_path))
    k0 = jit_compile_scene(path, "rm1", diag=False)
    switches = {"RMR_JIT_SCHED": "0", "RMR_JIT_OPTS": "-DRMR_PROG_WAVES=7", "RMR_JIT_BAKE": "0", "RMR_JIT_CULL": "3",
                "RMR_JIT_STEP": "0", "RMR_JIT_BKEY": "0", "RMR_JIT_AMBCOUNT": "1", "RMR_ESC_BOXES": "4",
                "RMR_GRID": "0", "RMR_JIT": "0", "RMR_ESC": "0", "RMR_NPC": "0", "RMR_JIT_APPROX": "0", "RMR_EYE": "0"}
    for k, v in switches.items():
        monkeypatch.setenv(k, v)
    assert jit_compile_scene(path, "rm1", diag=False) == k0
    assert jit_compile_scene(path, "rm1", diag=True) != k0
    import re
    rel = set(m.decode() for m in re.findall(rb"(RMR_[A-Z0-9_]+)\x00", open(LIB_PATH, "rb").read()))
    dia = set(m.decode() for m in re.findall(rb"(RMR_[A-Z0-9_]+)\x00", open(LIB_DIAG_PATH, "rb").read()))
    env_names = set(switches) | {"RMR_SHADE_T", "RMR_REFILL_T", "RMR_FULL_T", "RMR_FULL_R", "RMR_NPC_KSEL",
                                 "RMR_BVH_LEAF", "RMR_GRID_CELLS", "RMR_GRID_PAD", "RMR_GRID_PER_CU", "RMR_JIT_DUMP"}
    assert not (rel & env_names), sorted(rel & env_names)
    assert env_names <= dia, sorted(env_names - dia)
    assert "RMR_JIT_CACHE" in rel


def _setup(r, path, variant, W, H, overrides):
    r.set_image_size(W, H)
    r.reload()
    if path is None:
        r.load_builtin(variant)
    else:
        r.load_scene(path, variant)
    prm = abi.default_params(**overrides)
    r.set_params(prm)
    view = camera.default_view(W, H)
    r.set_view(view)
    r.set_env_map(synthetic_env() if prm.use_env_tex else None)
    return prm, view


def _tables(path, variant):
    return scene_compile.compile_scene({}, variant) if path is None else scene_compile.load_scene_file(path, variant)


@pytest.mark.gpu
@pytest.mark.parametrize("name,path,variant,overrides", SCENE_CASES, ids=IDS)
def test_jit_samples_bitexact_vs_oracle(renderer, name, path, variant, overrides):
    W, H = 44, 36
    rect = (3, 2, 41, 35)
    prm, view = _setup(renderer, path, variant, W, H, overrides)
    renderer.set_jit(1)
    try:
        renderer.reset_stats()
        times = time_schedule(3, frame=1)
        gpu = renderer.trace_samples(times, rect)
        st = renderer.stats()
    finally:
        renderer.set_jit(2)
    assert st.jit_launches > 0
    env = synthetic_env() if prm.use_env_tex else None
    cpu = oracle.Oracle(_tables(path, variant), prm, view, W, H, env=env).trace_samples(times, rect)
    a, b = gpu[..., :3], cpu[..., :3]
    same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
    assert same.all(), "%s: %d samples differ" % (name, (~same.all(-1)).sum())


@pytest.mark.gpu
@pytest.mark.parametrize("rect,spp", [((0, 0, 8, 8), 1), ((0, 0, 40, 24), 2), ((0, 0, 40, 24), 3),
                                      ((0, 0, 64, 64), 9)])
def test_work_queue_partitions_cover_every_unit(renderer, rect, spp):
    """The trace kernel's work queue in 16 partitions of 128-unit chunks (rmr_trace.h trace_main:
    a wave starts on partition blockIdx % 16, walks on or scans the counters when its own is used up).
    Launches of 1, 15, 23 and 288 chunks — fewer, about as many and more chunks than partitions,
    partial last chunks, the small-launch scan and the walk — against the oracle, every sample."""
    W, H = 64, 64
    prm, view = _setup(renderer, os.path.join(SCENES, "cornell5.scene"), "rm1", W, H, {"max_bounces": 2})
    times = time_schedule(spp, frame=4)
    renderer.set_jit(1)
    try:
        renderer.reset_stats()
        gpu = renderer.trace_samples(times, rect)
        st = renderer.stats()
    finally:
        renderer.set_jit(2)
    assert st.jit_launches > 0
    cpu = oracle.Oracle(_tables(os.path.join(SCENES, "cornell5.scene"), "rm1"), prm, view, W, H).trace_samples(times, rect)
    a, b = gpu[..., :3], cpu[..., :3]
    same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
    assert same.all(), "%d samples differ" % (~same.all(-1)).sum()


@pytest.mark.gpu
def test_jit_matches_table_kernel_on_large_render(renderer):
    W, H = 256, 192
    _setup(renderer, os.path.join(SCENES, "cornell5.scene"), "rm1", W, H, {"max_bounces": 4})
    times = time_schedule(24)
    out = {}
    for mode in (0, 1):
        renderer.set_jit(mode)
        renderer.reload()
        renderer.reset_stats()
        renderer.render_spp(times)
        out[mode] = renderer.read_accum()
        assert (renderer.stats().jit_launches > 0) == (mode == 1)
    renderer.set_jit(2)
    assert np.array_equal(out[0].view(np.uint32), out[1].view(np.uint32))


@pytest.mark.gpu
def test_jit_animated_scene_bitexact(renderer):
    """C5-style animation: a reload that only moves a primitive switches the context to the
    structure-only kernel (no per-frame compile); every frame still equals the table kernel."""
    import json
    import math
    W, H = 64, 48
    with open(os.path.join(SCENES, "cornell5.scene")) as f:
        base = json.load(f)
    times = time_schedule(4)
    for frame in range(3):
        sc = json.loads(json.dumps(base))
        sc["objects"][3]["nodes"][0]["inputs"][1][1] = 0.5 * math.sin(2.0 * math.pi * frame / 120.0)
        out = {}
        for mode in (1, 0):
            renderer.set_jit(mode)
            _setup(renderer, sc, "rm1", W, H, {"max_bounces": 4})
            renderer.reset_stats()
            renderer.render_spp(times)
            out[mode] = renderer.read_accum()
            assert (renderer.stats().jit_launches > 0) == (mode == 1)
        assert np.array_equal(out[0].view(np.uint32), out[1].view(np.uint32)), "frame %d" % frame
    renderer.set_jit(2)


def _ties_scene():
    """Cornell-5 plus exact and near duplicates: a second copy of the sphere with another material
    (exact ties on its whole surface: the later object must win, RM1:219-222), a copy of the floor
    shifted by one float ulp, and a sphere whose surface touches the left wall. These drive the
    approximate-then-exact map (rmr_trace.h am_*) through its exact fallback on many lanes."""
    import json
    with open(os.path.join(SCENES, "cornell5.scene")) as f:
        sc = json.load(f)
    obj = sc["objects"]
    dup = json.loads(json.dumps(obj[3]))
    dup["matID"] = 1
    obj.append(dup)
    floor = json.loads(json.dumps(obj[0]))
    floor["matID"] = 2
    floor["nodes"][0]["inputs"][1][1] = float(np.nextafter(np.float32(-1.025), np.float32(0)))
    obj.append(floor)
    touch = json.loads(json.dumps(obj[3]))
    touch["nodes"][0]["inputs"][1] = [-2.45, 1.0, 1.5]
    touch["nodes"][0]["inputs"][2] = [0.5, 0.5, 0.5]
    obj.append(touch)
    return sc


@pytest.mark.gpu
def test_jit_approx_map_ties_bitexact(renderer):
    sc = _ties_scene()
    W, H = 48, 40
    rect = (0, 0, W, H)
    prm, view = _setup(renderer, sc, "rm1", W, H, {"max_bounces": 4})
    renderer.set_jit(1)
    try:
        times = time_schedule(3, frame=2)
        gpu = renderer.trace_samples(times, rect)
        assert renderer.stats().jit_launches > 0
    finally:
        renderer.set_jit(2)
    cpu = oracle.Oracle(scene_compile.compile_scene(sc, "rm1"), prm, view, W, H).trace_samples(times, rect)
    a, b = gpu[..., :3], cpu[..., :3]
    same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
    assert same.all(), "%d samples differ" % (~same.all(-1)).sum()


def _bvh_ties_scene():
    """_ties_scene padded past the inline-map limit (32 primitives) with small spheres above the
    box, so the BVH map with the nearest-primitive cache runs: its approximate traversal
    (rmr_trace.h map_bvh_npc) meets exact ties everywhere on the duplicated sphere and floor and has
    to take its exact fallback there."""
    import json
    sc = _ties_scene()
    ball = sc["objects"][3]
    for n in range(30):
        pad = json.loads(json.dumps(ball))
        pad["nodes"][0]["inputs"][1] = [-3.0 + 0.2 * n, 9.0 + 0.1 * (n % 3), -2.0 + 0.13 * n]
        pad["nodes"][0]["inputs"][2] = [0.05, 0.05, 0.05]
        sc["objects"].append(pad)
    assert len(sc["objects"]) > 32
    return sc


@pytest.mark.gpu
def test_jit_bvh_cache_ties_bitexact_vs_oracle(renderer):
    sc = _bvh_ties_scene()
    W, H = 48, 40
    rect = (0, 0, W, H)
    prm, view = _setup(renderer, sc, "rm1", W, H, {"max_bounces": 4})
    renderer.set_jit(1)
    try:
        times = time_schedule(3, frame=4)
        gpu = renderer.trace_samples(times, rect)
        assert renderer.stats().jit_launches > 0
    finally:
        renderer.set_jit(2)
    cpu = oracle.Oracle(scene_compile.compile_scene(sc, "rm1"), prm, view, W, H).trace_samples(times, rect)
    a, b = gpu[..., :3], cpu[..., :3]
    same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
    assert same.all(), "%d samples differ" % (~same.all(-1)).sum()


@pytest.mark.gpu
def test_jit_bvh_nearest_primitive_cache_matches_table_kernel(renderer):
    """csg256 (256 primitives, BVH map): the JIT kernel with the nearest-primitive cache (one
    primitive per map() while the Lipschitz bound proves it the unique minimiser, rmr_trace.h npc_*)
    equals the table-driven BVH kernel (no cache) bit for bit on a full render."""
    W, H = 160, 120
    _setup(renderer, os.path.join(SCENES, "csg256.scene"), "rm1", W, H, {"max_bounces": 4})
    times = time_schedule(6, frame=3)
    out = {}
    for mode in (0, 1):
        renderer.set_jit(mode)
        renderer.reload()
        renderer.reset_stats()
        renderer.render_spp(times)
        out[mode] = renderer.read_accum()
        assert (renderer.stats().jit_launches > 0) == (mode == 1)
    renderer.set_jit(2)
    assert np.array_equal(out[0].view(np.uint32), out[1].view(np.uint32))


def _shelf_scene():
    """Cornell-5 plus a diffuse shelf under the light: rays bouncing up from the floor hit its bottom
    face, whose getNormal is exactly (0,-1,0), where randHemisphere's frame is NaN (RM1:270-304) —
    NaN directions, which the reference's march turns into a t = 0 hit (opU NaN rule)."""
    import json
    with open(os.path.join(SCENES, "cornell5.scene")) as f:
        sc = json.load(f)
    shelf = json.loads(json.dumps(sc["objects"][0]))
    shelf["nodes"][0]["inputs"][1] = [0.0, 2.5, 0.0]
    shelf["nodes"][0]["inputs"][2] = [1.0, 0.05, 1.0]
    sc["objects"].append(shelf)
    return sc


@pytest.mark.gpu
def test_shelf_nan_directions_bitexact_vs_oracle(renderer):
    sc = _shelf_scene()
    W, H = 40, 32
    rect = (0, 0, W, H)
    prm, view = _setup(renderer, sc, "rm1", W, H, {"max_bounces": 4})
    times = time_schedule(4, frame=2)
    gpu = renderer.trace_samples(times, rect)
    cpu = oracle.Oracle(scene_compile.compile_scene(sc, "rm1"), prm, view, W, H).trace_samples(times, rect)
    a, b = gpu[..., :3], cpu[..., :3]
    same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
    assert same.all(), "%d samples differ" % (~same.all(-1)).sum()


def _bvh_cornell_scene():
    """Cornell-5 padded past the inline-map limit with 30 small spheres far above the box (no map()
    value changes: they never attain the minimum), so it runs through the BVH map with the
    nearest-primitive cache."""
    import json
    with open(os.path.join(SCENES, "cornell5.scene")) as f:
        sc = json.load(f)
    ball = sc["objects"][3]
    for n in range(30):
        pad = json.loads(json.dumps(ball))
        pad["nodes"][0]["inputs"][1] = [-3.0 + 0.2 * n, 9.0 + 0.1 * (n % 3), -2.0 + 0.13 * n]
        pad["nodes"][0]["inputs"][2] = [0.05, 0.05, 0.05]
        sc["objects"].append(pad)
    return sc


@pytest.mark.gpu
@pytest.mark.parametrize("jit", [1, 0])
def test_bvh_cache_nan_point_with_cached_sphere_bitexact(renderer, jit):
    """A NaN bounce direction (randHemisphere about a getNormal of exactly (0,-1,0), here the
    sphere's bottom) while the lane's cached primitive is the sphere: the cached distance at the NaN
    point is not NaN (prim_dist's box form drops NaN coordinates), so it must not seed the full map.
    Sample 3 of pixel (1441, 652) of the 1080p C2 view took that path (found at full frame: one
    sample in 8.3 M rendered the wrong path before the fix)."""
    sc = _bvh_cornell_scene()
    W, H = 1920, 1080
    rect = (1440, 648, 1448, 656)
    prm, view = _setup(renderer, sc, "rm1", W, H, {"max_bounces": 4})
    renderer.set_jit(jit)
    try:
        renderer.reset_stats()
        times = time_schedule(4)
        gpu = renderer.trace_samples(times, rect)
        assert (renderer.stats().jit_launches > 0) == (jit == 1)
    finally:
        renderer.set_jit(2)
    cpu = oracle.Oracle(scene_compile.compile_scene(sc, "rm1"), prm, view, W, H).trace_samples(times, rect)
    a, b = gpu[..., :3], cpu[..., :3]
    same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
    assert same.all(), "%d samples differ" % (~same.all(-1)).sum()


def _cull_scene(scene):
    """(path, variant) of a culling-switch case: "shelf" (NaN directions), "rm3" (built-in), "rm2:X"
    (RM2 on golden scene X), golden scenes by name (node-program materials) or scenes/ files."""
    if scene == "shelf":
        return _shelf_scene(), "rm1"
    if scene == "rm3":
        return None, "rm3"
    if scene.startswith("rm2:"):
        return os.path.join(GOLDEN, "scenes", scene[4:]), "rm2"
    g = os.path.join(GOLDEN, "scenes", scene)
    return (g if os.path.exists(g) and not os.path.exists(os.path.join(SCENES, scene)) else os.path.join(SCENES, scene)), "rm1"


@pytest.mark.gpu
@pytest.mark.parametrize("scene,bounces,spp", [("cornell5.scene", 4, 12), ("csg256.scene", 4, 4), ("shelf", 4, 12),
                                               ("mandelbulb.scene", 2, 2), ("rm3", 16, 8),
                                               ("rm2:simple.scene", 16, 8), ("default.scene", 8, 4),
                                               ("glass_test.scene", 8, 4)])
def test_culling_switches_bitexact(renderer, scene, bounces, spp):
    """The exact work-skipping paths (escape bound, nearest-primitive cache, approximate-then-exact
    map; rmr_set_culling) change only the number of map() calls: full renders with every switch
    on and with every switch off are bitwise equal, on the JIT and on the table-driven kernels.
    Since round 3 the escape bound covers every kernel class: RM2 (shadow rays included) and the
    node-program-material kernels (default, glass) as well."""
    W, H = 192, 128
    path, variant = _cull_scene(scene)
    _setup(renderer, path, variant, W, H, {"max_bounces": bounces})
    times = time_schedule(spp, frame=5)
    out, evals = {}, {}
    try:
        for jit in (1, 0):
            renderer.set_jit(jit)
            for flags in (abi.CULL_ALL, 0):
                renderer.set_culling(flags)
                renderer.reload()
                renderer.reset_stats()
                renderer.render_spp(times)
                out[(jit, flags)] = renderer.read_accum()
                evals[(jit, flags)] = renderer.stats().map_evals
    finally:
        renderer.set_culling(abi.CULL_ALL)
        renderer.set_jit(2)
    ref = out[(0, 0)].view(np.uint32)
    for k, img in out.items():
        assert np.array_equal(ref, img.view(np.uint32)), k
    assert evals[(1, abi.CULL_ALL)] < evals[(1, 0)] == evals[(0, 0)]


@pytest.mark.gpu
@pytest.mark.parametrize("step_mult", [1.5, 2.0])
def test_escape_bound_inside_rays_long_steps_bitexact(renderer, step_mult):
    """Inside marches (glass, distMult = -1, RM1:498-505) take no escape bound: a step longer than the
    distance to the surface (stepMultiply > 1, rmr_params.step_multiply) can carry an inside ray past
    its object's box in one step, where the reference's next map() is positive and -map < 0.001 is a
    hit, not a miss. Every switch on and off, JIT and table kernels, and the oracle agree bitwise."""
    W, H = 96, 64
    path = os.path.join(GOLDEN, "scenes", "glass_test.scene")
    prm, view = _setup(renderer, path, "rm1", W, H, {"max_bounces": 8, "step_multiply": step_mult})
    times = time_schedule(4, frame=2)
    out = {}
    try:
        for jit in (1, 0):
            renderer.set_jit(jit)
            for flags in (abi.CULL_ALL, 0):
                renderer.set_culling(flags)
                renderer.reload()
                out[(jit, flags)] = renderer.trace_samples(times, (0, 0, W, H))
    finally:
        renderer.set_culling(abi.CULL_ALL)
        renderer.set_jit(2)
    ref = out[(0, 0)]
    for k, img in out.items():
        same = (img.view(np.uint32) == ref.view(np.uint32)).all(-1) | (np.isnan(img).any(-1) & np.isnan(ref).any(-1))
        assert same.all(), "%s: %d samples differ" % (k, (~same).sum())
    rect = (20, 10, 60, 40)
    cpu = oracle.Oracle(_tables(path, "rm1"), prm, view, W, H).trace_samples(times, rect)
    a, b = out[(1, abi.CULL_ALL)][:, rect[1]:rect[3], rect[0]:rect[2], :3], cpu[..., :3]
    same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
    assert same.all(), "%d samples differ from the oracle" % (~same.all(-1)).sum()


@pytest.mark.gpu
@pytest.mark.parametrize("scene,max_dist", [("cornell5.scene", 6.0), ("rm3", 5.0), ("mandelbulb.scene", 2.5),
                                            ("csg64.scene", 12.0), ("default.scene", 6.0)])
def test_far_hits_take_the_miss_branch_bitexact(renderer, scene, max_dist):
    """march() returns a hit's t even when t >= maxDist (its hit test precedes the t >= maxDist test,
    RM1:240-251), and a step of stepMultiply > 1 can overshoot into an object there; trace() shades only
    `v.x < maxDist` (RM1:514, RM2:436, RM3:368) and runs its miss branch otherwise, with the point
    o + t d (RM3's rand seed). Every kernel class (approximate sphere/box map, RM3, stepped Mandelbulb,
    nearest-primitive cache, node-program materials) against the oracle, culling on and off."""
    W, H = 64, 48
    path, variant = _cull_scene(scene)
    prm, view = _setup(renderer, path, variant, W, H, {"max_bounces": 4, "max_dist": max_dist,
                                                        "step_multiply": 1.7})
    times = time_schedule(2, frame=5)
    out = {}
    renderer.set_jit(1)
    try:
        for flags in (abi.CULL_ALL, 0):
            renderer.set_culling(flags)
            renderer.reload()
            out[flags] = renderer.trace_samples(times, (0, 0, W, H))
    finally:
        renderer.set_culling(abi.CULL_ALL)
        renderer.set_jit(2)
    rect = (16, 12, 48, 36)
    cpu = oracle.Oracle(_tables(path, variant), prm, view, W, H).trace_samples(times, rect)
    for flags, img in out.items():
        a, b = img[:, rect[1]:rect[3], rect[0]:rect[2], :3], cpu[..., :3]
        same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
        assert same.all(), "culling %d: %d samples differ from the oracle" % (flags, (~same.all(-1)).sum())


@pytest.mark.gpu
@pytest.mark.parametrize("max_dist,step_mult", [(1000.0, 0.5), (7.0, 1.0), (4.0, 1.7)])
def test_rm2_shadow_light_bound_bitexact(renderer, max_dist, step_mult):
    """RM2's shadow rays end at the light distance (rmr_trace.h: the NEE step reads the shadow march
    only through sd >= length(lightPos - pos), RM2:481-482). With maxDist below some of the light
    distances (the bound is then off for those rays) and above, and stepMultiply up to 1.7: every switch
    on and off, JIT and table kernels, and the oracle agree bitwise."""
    W, H = 96, 64
    path = os.path.join(GOLDEN, "scenes", "simple.scene")
    prm, view = _setup(renderer, path, "rm2", W, H, {"max_bounces": 6, "max_dist": max_dist,
                                                      "step_multiply": step_mult})
    times = time_schedule(4, frame=3)
    out = {}
    try:
        for jit in (1, 0):
            renderer.set_jit(jit)
            for flags in (abi.CULL_ALL, 0):
                renderer.set_culling(flags)
                renderer.reload()
                out[(jit, flags)] = renderer.trace_samples(times, (0, 0, W, H))
    finally:
        renderer.set_culling(abi.CULL_ALL)
        renderer.set_jit(2)
    ref = out[(0, 0)]
    for k, img in out.items():
        same = (img.view(np.uint32) == ref.view(np.uint32)).all(-1) | (np.isnan(img).any(-1) & np.isnan(ref).any(-1))
        assert same.all(), "%s: %d samples differ" % (k, (~same).sum())
    rect = (24, 16, 56, 40)
    cpu = oracle.Oracle(_tables(path, "rm2"), prm, view, W, H).trace_samples(times, rect)
    a, b = out[(1, abi.CULL_ALL)][:, rect[1]:rect[3], rect[0]:rect[2], :3], cpu[..., :3]
    same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
    assert same.all(), "%d samples differ from the oracle" % (~same.all(-1)).sum()


@pytest.mark.gpu
@pytest.mark.parametrize("scene,W,H", [("cornell5.scene", 1920, 1080), ("csg256.scene", 960, 540),
                                       ("rm2:simple.scene", 1920, 1080), ("default.scene", 960, 540)])
def test_culling_switches_full_frame_bitexact(renderer, scene, W, H):
    """The same property at production frame sizes (rare events — NaN directions, near ties, cache
    bounds at grazing angles — show up only over millions of paths): every per-sample radiance of a
    2-spp frame is bitwise equal with the work-skipping paths on and off (round 3's full-frame sweep
    runs the other scene families)."""
    path, variant = _cull_scene(scene)
    _setup(renderer, path, variant, W, H, {"max_bounces": 4})
    times = time_schedule(2, frame=7)
    out = {}
    renderer.set_jit(1)
    try:
        for flags in (abi.CULL_ALL, 0):
            renderer.set_culling(flags)
            renderer.reload()
            out[flags] = renderer.trace_samples(times, (0, 0, W, H))
    finally:
        renderer.set_culling(abi.CULL_ALL)
        renderer.set_jit(2)
    a, b = out[abi.CULL_ALL], out[0]
    same = (a.view(np.uint32) == b.view(np.uint32)).all(-1) | (np.isnan(a).any(-1) & np.isnan(b).any(-1))
    assert same.all(), "%d of %d samples differ" % ((~same).sum(), same.size)


@pytest.mark.gpu
@pytest.mark.parametrize("scene", ["csg256.scene", "csg64.scene"])
def test_candidate_grid_full_frame_bitexact(monkeypatch, scene):
    """The nearest-primitive cache's full map() through the candidate grid (rmr_trace.h map_grid_npc,
    the default for BVH scenes) against the same cache over the BVH traversal (RMR_GRID=0, read at
    scene load by the diagnostic build): every sample of a 960x540 2-spp frame bitwise equal."""
    from raymarchrenderer_amd import Renderer
    W, H = 960, 540
    out = {}
    r = Renderer(0, 64, 64, diag=True)
    r.set_jit(1)
    try:
        for grid in ("1", "0"):
            monkeypatch.setenv("RMR_GRID", grid)
            _setup(r, os.path.join(SCENES, scene), "rm1", W, H, {"max_bounces": 4})
            out[grid] = r.trace_samples(time_schedule(2, frame=9), (0, 0, W, H))
    finally:
        monkeypatch.delenv("RMR_GRID")
        r.close()
    a, b = out["1"], out["0"]
    same = (a.view(np.uint32) == b.view(np.uint32)).all(-1) | (np.isnan(a).any(-1) & np.isnan(b).any(-1))
    assert same.all(), "%d of %d samples differ" % ((~same).sum(), same.size)


@pytest.mark.gpu
@pytest.mark.parametrize("scene", ["cornell5.scene", "csg256.scene"])
def test_scheduling_knobs_bitexact(scene):
    """Shading-batch size, refill threshold, persistent grid size (rmr_set_tuning) and the grid
    reserve (rmr_set_grid_reserve) decide only which lanes run which path when: the image is bitwise
    the same for every setting, including the per-kernel default (20-lane batches on Cornell-5, 16 on
    the cached BVH kernel)."""
    from raymarchrenderer_amd import Renderer
    W, H = 160, 96
    r = Renderer(0, 64, 64)   # own context: the settings below would outlive the test
    try:
        r.set_jit(1)
        _setup(r, os.path.join(SCENES, scene), "rm1", W, H, {"max_bounces": 4})
        times = time_schedule(6, frame=3)
        imgs = []
        for shade, grid in ((0, -1), (1, -1), (7 | (3 << 8), 2), (20, -1), (64 | (64 << 8), 1), (33, 5)):
            if shade:
                r.set_tuning(shade, grid)
            r.reload()
            r.render_spp(times)
            imgs.append(r.read_accum().view(np.uint32).copy())
        # a persistent grid of one workgroup (reserve beyond the occupancy grid), then 3 left free
        r.set_tuning(0, 0)   # (the occupancy grid again: a fixed grid per CU ignores the reserve)
        for reserve in (1 << 20, 3):
            r.set_grid_reserve(reserve)
            r.reload()
            r.render_spp(times)
            imgs.append(r.read_accum().view(np.uint32).copy())
        with pytest.raises(Exception):
            r.set_grid_reserve(-1)
    finally:
        r.close()
    for k, img in enumerate(imgs[1:], 1):
        assert np.array_equal(imgs[0], img), k


@pytest.mark.gpu
def test_mandelbulb_map_bitexact_vs_oracle(renderer):
    """The specialised kernel's Mandelbulb map (mb_iter8_poly, the whole estimator per map()) equals
    the oracle sample for sample."""
    path = os.path.join(SCENES, "mandelbulb.scene")
    W, H = 48, 40
    rect = (0, 0, W, H)
    prm, view = _setup(renderer, path, "rm1", W, H, {"max_bounces": 2})
    renderer.set_jit(1)
    try:
        times = time_schedule(2, frame=4)
        gpu = renderer.trace_samples(times, rect)
        assert renderer.stats().jit_launches > 0
    finally:
        renderer.set_jit(2)
    cpu = oracle.Oracle(_tables(path, "rm1"), prm, view, W, H).trace_samples(times, rect)
    a, b = gpu[..., :3], cpu[..., :3]
    same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
    assert same.all(), "%d samples differ" % (~same.all(-1)).sum()


def _rm2_variant(tmp_path, name, nodes, output, constants):
    """simple.scene's RM2 material (id 1, the built-in sphere's) with another v2 node program."""
    import json
    sc = {"materials": [{"id": 1, "constants": constants, "nodes": nodes, "output": output}], "objects": []}
    p = tmp_path / (name + ".scene")
    p.write_text(json.dumps(sc))
    return str(p)


# v2 programs (Graphics.cpp:405-463 compileNode) beyond simple.scene's diffuse/glossy/fresnel mix:
# one BSDF alone, a mirror (roughness 0: reflect), and a mix whose branches are swapped
RM2_PROGRAMS = {
    "diffuse": ([{"name": "shader_diffuse", "inputs": [[-1, 0]]}], 0, [[0.3, 0.6, 0.9]]),
    "glossy": ([{"name": "shader_glossy", "inputs": [[-1, 0], [-1, 1]]}], 0, [[0.9, 0.5, 0.1], 0.35]),
    "mirror": ([{"name": "shader_glossy", "inputs": [[-1, 0], [-1, 1]]}], 0, [[1.0, 1.0, 1.0], 0.0]),
    "mix_swapped": ([{"name": "shader_glossy", "inputs": [[-1, 1], [-1, 2]]}, {"name": "shader_diffuse", "inputs": [[-1, 0]]},
                     {"name": "shader_mix", "inputs": [[0, 0], [1, 0], [3, 0]]}, {"name": "misc_fresnel"}], 2,
                    [[0.2, 0.8, 0.2], [0.9, 0.9, 0.9], 0.05]),
}


@pytest.mark.parametrize("prog", sorted(RM2_PROGRAMS))
def test_jit_rm2_v2_program_compiles(tmp_path, monkeypatch, prog):
    """RM2's v2 material as generated straight-line code (JitV2Mats) compiles for every node form."""
    nodes, out, consts = RM2_PROGRAMS[prog]
    path = _rm2_variant(tmp_path, prog, nodes, out, consts)
    monkeypatch.setenv("RMR_JIT_CACHE", str(tmp_path))
    key = jit_compile_scene(path, "rm2")
    assert (tmp_path / (key + ".hsaco")).stat().st_size > 1000


@pytest.mark.gpu
@pytest.mark.parametrize("prog", sorted(RM2_PROGRAMS))
def test_jit_rm2_v2_program_bitexact_vs_oracle(renderer, tmp_path, prog):
    """The generated v2 material (JitV2Mats) against the oracle's table interpreter, bit for bit."""
    nodes, out, consts = RM2_PROGRAMS[prog]
    path = _rm2_variant(tmp_path, prog, nodes, out, consts)
    W, H = 40, 32
    rect = (0, 0, W, H)
    prm, view = _setup(renderer, path, "rm2", W, H, {"max_bounces": 6})
    renderer.set_jit(1)
    try:
        renderer.reset_stats()
        times = time_schedule(3, frame=2)
        gpu = renderer.trace_samples(times, rect)
        st = renderer.stats()
    finally:
        renderer.set_jit(2)
    assert st.jit_launches > 0
    cpu = oracle.Oracle(_tables(path, "rm2"), prm, view, W, H).trace_samples(times, rect)
    a, b = gpu[..., :3], cpu[..., :3]
    same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
    assert same.all(), "%s: %d samples differ" % (prog, (~same.all(-1)).sum())


def test_jit_stepped_mandelbulb_source(tmp_path, monkeypatch):
    """Scenes with one Mandelbulb get the stepped map (rmr_trace.h MBStep: begin / step / finish,
    finishing batches); RMR_JIT_STEP=0 keeps the whole map per pass (another code object; the
    diagnostic build, which also dumps the source with RMR_JIT_DUMP)."""
    path = os.path.join(SCENES, "mandelbulb.scene")
    monkeypatch.setenv("RMR_JIT_CACHE", str(tmp_path / "c"))
    (tmp_path / "d").mkdir()
    monkeypatch.setenv("RMR_JIT_DUMP", str(tmp_path / "d"))
    k_on = jit_compile_scene(path, "rm1", diag=True)
    assert jit_compile_scene(path, "rm1", diag=False) == k_on   # the release build's kernel
    src = (tmp_path / "d" / (k_on + ".hip")).read_text()
    assert "kStepped = RMR_MB_STEPPED" in src and "mb_step(s, " in src and "mb_de(s.r, s.dr)" in src
    monkeypatch.setenv("RMR_JIT_STEP", "0")
    k_off = jit_compile_scene(path, "rm1", diag=True)
    assert k_off != k_on
    assert "kStepped = false" in (tmp_path / "d" / (k_off + ".hip")).read_text()
    # a sphere/box scene has no stepped map
    k_c5 = jit_compile_scene(os.path.join(SCENES, "cornell5.scene"), "rm1", diag=True)
    assert "kStepped = false" in (tmp_path / "d" / (k_c5 + ".hip")).read_text()


def _csg64_unpackable(tmp_path):
    """csg64 with one object's material id out of am_pack's range (|id| >= 2^15, no such material:
    the path ends black, as in the reference): the cache kernel then keeps the LDS table unpacked."""
    import json
    s = json.load(open(os.path.join(SCENES, "csg64.scene")))
    s["objects"][5]["matID"] = 40000
    p = tmp_path / "csg64_unpackable.scene"
    p.write_text(json.dumps(s))
    return str(p)


@pytest.mark.parametrize("unpackable", [False, True])
def test_cache_kernel_packed_table_only_for_packable_ids(tmp_path, monkeypatch, unpackable):
    """rmr_jit.cpp emits RMR_NPC_PACKED (the select-free LDS primitive table, rmr_trace.h
    npc_pack_entry) for a cache scene only when every material id can carry a scene index."""
    path = _csg64_unpackable(tmp_path) if unpackable else os.path.join(SCENES, "csg64.scene")
    dump = tmp_path / "dump"
    dump.mkdir()
    monkeypatch.setenv("RMR_JIT_CACHE", str(tmp_path / "cache"))
    monkeypatch.setenv("RMR_JIT_DUMP", str(dump))
    key = jit_compile_scene(path, "rm1", diag=True)
    src = (dump / (key + ".hip")).read_text()
    assert "#define RMR_NPC_DP_LDS 1" in src
    assert ("#define RMR_NPC_PACKED 1" in src) == (not unpackable)


@pytest.mark.gpu
def test_cache_kernel_unpacked_table_bitexact_vs_oracle(renderer, tmp_path):
    """The cache kernel on the unpacked LDS table (a material id am_pack cannot carry) against the
    oracle, every sample of a small frame (the packed table: rm1_csg64_b4 above)."""
    path = _csg64_unpackable(tmp_path)
    W, H = 44, 36
    rect = (3, 2, 41, 35)
    prm, view = _setup(renderer, path, "rm1", W, H, {"max_bounces": 4})
    renderer.set_jit(1)
    try:
        times = time_schedule(3, frame=2)
        gpu = renderer.trace_samples(times, rect)
    finally:
        renderer.set_jit(2)
    cpu = oracle.Oracle(_tables(path, "rm1"), prm, view, W, H).trace_samples(times, rect)
    a, b = gpu[..., :3], cpu[..., :3]
    same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
    assert same.all(), "%d samples differ" % (~same.all(-1)).sum()
