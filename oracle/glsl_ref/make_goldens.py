"""oracle/glsl_ref/make_goldens.py — TEST INFRASTRUCTURE: generate tests/golden/ fixtures by running
the reference GLSL (RayMarch*.glsl from /root/reference) on Mesa llvmpipe in this container.

    python -m oracle.glsl_ref.make_goldens [--only NAME] [--conv-spp N]

Fixtures are data (inputs + reference outputs); the reference source itself is not stored.
  kat_<scene>.npz   function-level known answers: map / march / getNormal / rand chain /
                    randHemisphere on fixed input sets (+ wavelengthToColor for RM3)
  img_<name>.npz    low-spp renders (4 spp) and converged renders (--conv-spp) of 64x48 images
  display_ref.npz   Graphics::Display (FullQuad.vs / .fs, GL_FRAMEBUFFER_SRGB, blend) drawn screens
MANIFEST.json records every configuration, the camera, the seed schedule and the GL driver.
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import camera  # noqa: E402
from oracle.envmap import synthetic_env  # noqa: E402
from oracle.glsl_ref import ref_run, shader_build  # noqa: E402
from raymarchrenderer_amd import abi, parity_schedule, time_schedule  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")
GS = os.path.join(GOLDEN, "scenes")
W, H = 64, 48

# name: (scene file or None, variant, params overrides, converged spp)
IMAGES = {
    "rm3_builtin": (None, 3, {}, 262144),
    "rm1_cornell5_b4": (os.path.join(ROOT, "scenes", "cornell5.scene"), 1, {"max_bounces": 4}, 262144),
    "rm1_sphere1_b1": (os.path.join(ROOT, "scenes", "sphere1.scene"), 1, {"max_bounces": 1}, 16384),
    "rm2_simple": (os.path.join(GS, "simple.scene"), 2, {}, 65536),
    "rm1_default": (os.path.join(GS, "default.scene"), 1, {}, 131072),
    "rm1_glass": (os.path.join(GS, "glass_test.scene"), 1, {}, 65536),
    "rm1_multilight": (os.path.join(GS, "multilight.scene"), 1, {}, 65536),
    # env-map sky (useEnvTex = 1, synthetic_env): RM1:78-113 / RM2:84-107
    "rm1_sphere1_env": (os.path.join(ROOT, "scenes", "sphere1.scene"), 1, {"max_bounces": 4, "use_env_tex": 1}, 16384),
    "rm2_simple_env": (os.path.join(GS, "simple.scene"), 2, {"use_env_tex": 1}, 16384),
    # RM1 object node set (op_union / op_subtract / op_intersect / domain_repeat / math / misc)
    "rm1_csg_nodes_b4": (os.path.join(ROOT, "scenes", "csg_nodes.scene"), 1, {"max_bounces": 4}, 131072),
    # C3's Mandelbulb node added to the reference path (shader_build X1), 2 bounces as C3
    "rm1_mandelbulb_b2": (os.path.join(ROOT, "scenes", "mandelbulb.scene"), 1, {"max_bounces": 2}, 65536),
    # C4's generator cut to 64 primitives (the reference codegen compiles it; 256 does not finish)
    "rm1_csg64_b4": (os.path.join(ROOT, "scenes", "csg64.scene"), 1, {"max_bounces": 4}, 32768),
}
KATS = {
    "rm3": (None, 3),
    "cornell5": (os.path.join(ROOT, "scenes", "cornell5.scene"), 1),
    "default": (os.path.join(GS, "default.scene"), 1),
    "csg_nodes": (os.path.join(ROOT, "scenes", "csg_nodes.scene"), 1),
    "mandelbulb": (os.path.join(ROOT, "scenes", "mandelbulb.scene"), 1),
    "csg64": (os.path.join(ROOT, "scenes", "csg64.scene"), 1),
}


def _scene(path):
    return shader_build.load_scene(path) if path else None


def make_kat(name, path, variant, rng):
    scene = _scene(path)
    prm = abi.default_params()
    n = 512
    pts = rng.uniform([-5, -1.5, -5], [5, 5, 5], size=(n, 3)).astype(np.float32)
    m = ref_run.probe(variant, scene, 0, pts, n, 2, prm)
    eye = np.array([0, 4, -6], np.float32)
    o = (eye + rng.normal(0, 0.3, size=(n, 3))).astype(np.float32)
    d = rng.normal(0, 1, size=(n, 3))
    d[:, 1] = -np.abs(d[:, 1])
    d[:, 2] = np.abs(d[:, 2])
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    march = ref_run.probe(variant, scene, 1, np.concatenate([o, d], 1), n, 2, prm)
    # normals at march hit points
    hits = (o + d * march[:, :1]).astype(np.float32)
    nrm = ref_run.probe(variant, scene, 2, hits, n, 3, prm)
    seeds = rng.uniform(-50, 1500, size=(n, 8)).astype(np.float32)
    t = 0.512
    rnd = ref_run.probe(variant, scene, 3, seeds, n, 4, prm, time=t)
    hin = np.concatenate([rng.uniform(-5, 5, size=(n, 4)), rng.normal(0, 1, size=(n, 3)),
                          np.zeros((n, 1)), rng.uniform(0, 1, size=(n, 1))], 1).astype(np.float32)
    hin[:, 4:7] /= np.linalg.norm(hin[:, 4:7], axis=1, keepdims=True)
    hemi = ref_run.probe(variant, scene, 4, hin, n, 3, prm, time=t)
    out = dict(map_in=pts, map_out=m, march_in=np.concatenate([o, d], 1), march_out=march, normal_in=hits,
               normal_out=nrm, rand_in=seeds, rand_out=rnd, rand_time=np.float32(t), hemi_in=hin, hemi_out=hemi,
               probe_width=np.int32(64))
    if variant == 3:
        wls = np.arange(360, 860, dtype=np.float32)
        out["wl_in"] = wls
        out["wl_out"] = ref_run.wl2rgb_probe(wls)
    np.savez_compressed(os.path.join(GOLDEN, "kat_%s.npz" % name), **out)


NAN_MAIN = r"""
layout(std430, binding = 2) readonly buffer ProbeIn { float pin[]; };
layout(std430, binding = 3) writeonly buffer ProbeOut { float pout[]; };
uniform int probeCount;
void main()
{
    uint gw = gl_NumWorkGroups.x * gl_WorkGroupSize.x;
    uint i = gl_GlobalInvocationID.y * gw + gl_GlobalInvocationID.x;
    if (i >= uint(probeCount)) return;
    channels = vec3(1, 1, 1);
    vec3 nanv = normalize(vec3(pin[4 * i + 3]));      // pin = 0: normalize(vec3(0)) = NaN
    vec3 o = vec3(pin[4 * i], pin[4 * i + 1], pin[4 * i + 2]);
    vec2 m = map(nanv);
    vec2 a = march(o, nanv, 1.0);
    vec2 b = march(o, nanv, -1.0);
    pout[6 * i] = m.x; pout[6 * i + 1] = m.y;
    pout[6 * i + 2] = a.x; pout[6 * i + 3] = a.y;
    pout[6 * i + 4] = b.x; pout[6 * i + 5] = b.y;
}
"""


def make_kat_nan(rng):
    """NaN ray directions (normalize(vec3(0)) after total internal reflection in shader_refraction):
    map(NaN) and march(o, NaN, +-1) of the reference on llvmpipe, per scene."""
    import math
    out = {}
    for name, (path, variant) in KATS.items():
        if variant != 1:
            continue
        n = 64
        o = rng.uniform([-5, -1, -5], [5, 5, 5], size=(n, 3)).astype(np.float32)
        pin = np.concatenate([o, np.zeros((n, 1), np.float32)], 1)
        src = shader_build.build(variant, _scene(path), probe_main=NAN_MAIN)
        lx, ly = shader_build.LOCAL[variant]
        prm = abi.default_params()
        lines = ["image 8 8"] + ref_run._uniform_lines(prm, np.zeros(15, np.float32))
        lines += ["ui probeCount %d" % n, "run 0 0 0 0 0 0 %d %d" % (64 // lx, int(math.ceil(n / 64.0 / ly)))]
        _, so = ref_run.run_job(src, lines, None, ssbo_in=pin.ravel(), ssbo_out_n=6 * n)
        out["%s_origin" % name] = o
        out["%s_out" % name] = so.reshape(n, 6)
    np.savez_compressed(os.path.join(GOLDEN, "kat_nan.npz"), **out)


def make_image(name, path, variant, kw, conv_spp, threads):
    scene = _scene(path)
    prm = abi.default_params(**kw)
    view = camera.default_view(W, H)
    env = synthetic_env() if kw.get("use_env_tex") else None
    lo = ref_run.render(variant, scene, W, H, time_schedule(4), prm, view, threads=threads, env=env)
    t0 = time.time()
    # converged reference on the parity schedule (small seeds, see raymarchrenderer_amd.parity_schedule)
    conv = ref_run.render(variant, scene, W, H, parity_schedule(conv_spp), prm, view, threads=threads, env=env)
    dt = time.time() - t0
    extra = {"env": env} if env is not None else {}
    np.savez_compressed(os.path.join(GOLDEN, "img_%s.npz" % name), lo=lo, conv=conv, view=view,
                        spp_lo=np.int32(4), spp_conv=np.int32(conv_spp), conv_schedule="parity", **extra)
    return dt


# Graphics::Display cases on a 96x72 accumulator: centre, zoom, bounds min / max, screen (w, h)
DISPLAY_CASES = [
    ((64.0, 48.0), 1.0, (0, 0), (128, 96), (128, 96)),              # 1:1, texel centres on pixel centres
    ((64.0, 48.0), 0.5, (1, 1), (127, 95), (128, 96)),              # the GUI's start zoom (GUI.cpp:187)
    ((50.3, 40.9), 2.7, (20.5, 10.0), (110.0, 80.25), (128, 96)),   # magnified, clipped by the bounds
    ((-20.0, 130.0), 1.3, (0, 0), (500, 500), (128, 96)),           # quad partly off screen
    ((64.0, 48.0), 0.37, (0, 0), (1000, 1000), (131, 97)),          # minified, ragged screen
    ((64.5, 48.5), 1.0, (0, 0), (500, 500), (128, 96)),             # quad edges through pixel centres
    ((65.0, 49.0), 1.0, (10.5, 5.5), (100.5, 70.5), (128, 96)),     # bounds through pixel centres
    ((60.25, 45.75), 3.0, (0, 0), (500, 500), (128, 96)),
    ((64.0, 48.0), 0.25, (0, 0), (500, 500), (128, 96)),
]


def display_background(w, h):
    """The screen content behind the quad (the GUI): a fixed pattern, alpha 7."""
    y, x = np.mgrid[0:h, 0:w]
    bg = np.stack([(7 * x + 13 * y) % 256, (11 * x + 3 * y + 50) % 256, (5 * x + 17 * y + 99) % 256,
                   np.full_like(x, 7)], -1)
    return bg.astype(np.uint8)


def make_display():
    """Graphics::Display (Graphics.cpp:356-390, FullQuad.vs / .fs) on llvmpipe over DISPLAY_CASES:
    tests/golden/display_ref.npz holds the accumulator and every case's drawn screen."""
    rng = np.random.default_rng(2024)
    acc = rng.uniform(-0.2, 1.3, size=(72, 96, 4)).astype(np.float32)
    acc[rng.random((72, 96)) < 0.01, 0] = np.nan
    acc[rng.random((72, 96)) < 0.005, 2] = np.inf
    acc[..., 1] = np.where(rng.random((72, 96)) < 0.3, rng.uniform(0, 0.004, (72, 96)), acc[..., 1]).astype(np.float32)
    out = {"accum": acc}
    for k, (centre, zoom, vmin, vmax, size) in enumerate(DISPLAY_CASES):
        bg = display_background(*size)
        out["case%d" % k] = np.array(list(centre) + [zoom] + list(vmin) + list(vmax) + list(size), np.float64)
        out["out%d" % k] = ref_run.display(acc, centre, zoom, vmin, vmax, bg)
    np.savez_compressed(os.path.join(GOLDEN, "display_ref.npz"), **out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="", help="comma-separated fixture names (kat_<scene>, kat_nan, <image>)")
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--conv-scale", type=float, default=1.0)
    args = ap.parse_args()
    if not ref_run.available():
        sys.exit("reference or Mesa swrast driver not available")
    ref_run.ensure_built()
    os.makedirs(GOLDEN, exist_ok=True)
    man_path = os.path.join(GOLDEN, "MANIFEST.json")
    man = json.load(open(man_path)) if os.path.exists(man_path) else {}
    gl = subprocess.run(["bash", "-c", "RMR_VERBOSE=1 true"], capture_output=True, text=True)
    _ = gl
    man["generator"] = "oracle/glsl_ref/make_goldens.py (reference GLSL on Mesa llvmpipe via oracle/glsl_ref/harness.c)"
    man["driver"] = "Mesa 23.2.1 llvmpipe (swrast_dri.so), GL 4.5 core"
    man["image_size"] = [W, H]
    man["camera"] = "Program.cpp:102 default camera, aspect W/H"
    man["time_schedule"] = ("lo: time(f=0, s) = 0.016 * s; conv: parity_schedule(n) = s * 0.016 / 256 "
                            "(small seeds keep the sin-hash out of its float32-quantised regime), float32")
    man.setdefault("kat", {})
    man.setdefault("images", {})
    rng = np.random.default_rng(20251015)
    for name, (path, variant) in KATS.items():
        if args.only and "kat_" + name not in args.only.split(","):
            continue
        make_kat(name, path, variant, rng)
        man["kat"][name] = {"scene": os.path.relpath(path, ROOT) if path else "builtin", "variant": variant}
        print("kat", name, flush=True)
    if not args.only or "display" in args.only.split(","):
        make_display()
        man["display"] = {"fixture": "display_ref.npz", "shaders": "FullQuad.vs / FullQuad.fs",
                          "harness": "oracle/glsl_ref/display_harness.c (compat 4.3, sRGB8_ALPHA8 target)",
                          "cases": len(DISPLAY_CASES)}
        print("display", flush=True)
    if not args.only or "kat_nan" in args.only.split(","):
        make_kat_nan(np.random.default_rng(7))
        man["kat"]["nan"] = {"scenes": [k for k, v in KATS.items() if v[1] == 1], "probe": "map/march with NaN dir"}
        print("kat nan", flush=True)
    for name, (path, variant, kw, spp) in IMAGES.items():
        if args.only and name not in args.only.split(","):
            continue
        spp = int(spp * args.conv_scale)
        dt = make_image(name, path, variant, kw, spp, args.threads)
        man["images"][name] = {"scene": os.path.relpath(path, ROOT) if path else "builtin", "variant": variant,
                               "params": kw, "spp_lo": 4, "spp_conv": spp, "seconds": round(dt, 1)}
        print("image", name, spp, "spp", round(dt, 1), "s", flush=True)
        with open(man_path, "w") as f:
            json.dump(man, f, indent=1, sort_keys=True)
    with open(man_path, "w") as f:
        json.dump(man, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
