"""oracle/glsl_ref/ref_run.py — TEST INFRASTRUCTURE: run the reference GLSL on llvmpipe.

Only usable where /root/reference and Mesa's swrast driver exist (this container); outputs are
committed as fixtures by make_goldens.py, never regenerated on the GPU box.
"""
import hashlib
import math
import os
import subprocess
import tempfile

import numpy as np

from . import shader_build

HERE = os.path.dirname(os.path.abspath(__file__))
REF_OUT = os.path.join(os.path.dirname(HERE), "_ref")
HARNESS = os.path.join(REF_OUT, "glsl_harness")


def available():
    return os.path.isdir(shader_build.REF) and os.path.exists("/usr/lib/x86_64-linux-gnu/dri/swrast_dri.so")


def ensure_built():
    if not os.path.exists(HARNESS):
        subprocess.check_call(["make", "-s", "-C", HERE])


SHADER_CACHE = os.path.join(tempfile.gettempdir(), "rmr_glsl_ref")  # outside the repo: never shipped


def _write_shader(src):
    os.makedirs(SHADER_CACHE, exist_ok=True)
    h = hashlib.sha1(src.encode()).hexdigest()[:16]
    p = os.path.join(SHADER_CACHE, "shader_%s.glsl" % h)
    if not os.path.exists(p):
        with open(p, "w") as f:
            f.write(src)
    return p


def _uniform_lines(params, view):
    v = np.asarray(view, np.float32).reshape(5, 3)
    lines = ["uf maxDist %r" % float(params.max_dist), "ui maxSteps %d" % params.max_steps,
             "ui maxBounces %d" % params.max_bounces, "uf stepMultiply %r" % float(params.step_multiply),
             "ui useEnvTex %d" % params.use_env_tex, "ui separateChannels %d" % params.separate_channels,
             "ui envTex 0"]
    for name, row in zip(["eye", "ray00", "ray01", "ray10", "ray11"], v):
        lines.append("u3f %s %.9g %.9g %.9g" % (name, row[0], row[1], row[2]))
    return lines


def run_job(src, job_lines, out_floats_shape, ssbo_in=None, ssbo_out_n=0, threads=None, timeout=3600, env=None):
    ensure_built()
    shader = _write_shader(src)
    with tempfile.TemporaryDirectory() as td:
        job = os.path.join(td, "job.txt")
        lines = list(job_lines)
        if ssbo_in is not None:
            pin = os.path.join(td, "in.f32")
            np.ascontiguousarray(ssbo_in, np.float32).tofile(pin)
            lines.insert(1, "ssbo_in %s" % pin)
        if ssbo_out_n:
            lines.insert(1, "ssbo_out %d" % ssbo_out_n)
        if env is not None:  # after the "image" line, which binds the accumulator on unit 0
            pe = os.path.join(td, "env.rgba8")
            np.ascontiguousarray(env, np.uint8).tofile(pe)
            lines.insert(1, "envtex %s %d %d" % (pe, env.shape[1], env.shape[0]))
        with open(job, "w") as f:
            f.write("\n".join(lines) + "\n")
        out = os.path.join(td, "out.f32")
        sout = os.path.join(td, "sout.f32")
        env = dict(os.environ)
        if threads:
            env["LP_NUM_THREADS"] = str(threads)
        r = subprocess.run([HARNESS, shader, job, out, sout], env=env, capture_output=True, text=True, timeout=timeout)
        if r.returncode != 0:
            raise RuntimeError("harness failed (%d): %s" % (r.returncode, r.stderr[-4000:]))
        img = np.fromfile(out, np.float32)
        so = np.fromfile(sout, np.float32) if ssbo_out_n else None
    if out_floats_shape is not None:
        img = img.reshape(out_floats_shape)
    return img, so


def render(variant, scene, W, H, times, params, view, rect=None, first_sample=0, threads=None, env=None):
    """nspp Graphics::Render calls (one per entry of `times`, currentSample = first_sample + k) over
    `rect` (x0, y0, x1, y1) of a W x H accumulator that starts at 0. Returns (H, W, 4) float32."""
    src = shader_build.build(variant, scene)
    lx, ly = shader_build.LOCAL[variant]
    x0, y0, x1, y1 = rect if rect is not None else (0, 0, W, H)
    gx, gy = int(math.ceil(x1 / lx)), int(math.ceil(y1 / ly))
    lines = ["image %d %d" % (W, H)] + _uniform_lines(params, view)
    for k, t in enumerate(times):
        lines.append("run %.9g %d %d %d %d %d %d %d" % (float(t), first_sample + k, x0, y0, x1, y1, gx, gy))
    img, _ = run_job(src, lines, (H, W, 4), threads=threads, env=env)
    return img


PROBE_MAIN = r"""
layout(std430, binding = 2) readonly buffer ProbeIn { float pin[]; };
layout(std430, binding = 3) writeonly buffer ProbeOut { float pout[]; };
uniform int probeMode;
uniform int probeCount;
void main()
{
    uint gw = gl_NumWorkGroups.x * gl_WorkGroupSize.x;
    uint i = gl_GlobalInvocationID.y * gw + gl_GlobalInvocationID.x;
    if (i >= uint(probeCount)) return;
    channels = vec3(1, 1, 1);
    if (probeMode == 0) {            // map(p)
        vec3 p = vec3(pin[3 * i], pin[3 * i + 1], pin[3 * i + 2]);
        vec2 d = map(p);
        pout[2 * i] = d.x; pout[2 * i + 1] = d.y;
    } else if (probeMode == 1) {     // march(o, d, 1)
        vec3 o = vec3(pin[6 * i], pin[6 * i + 1], pin[6 * i + 2]);
        vec3 dd = vec3(pin[6 * i + 3], pin[6 * i + 4], pin[6 * i + 5]);
        vec2 v = march(o, dd, 1);
        pout[2 * i] = v.x; pout[2 * i + 1] = v.y;
    } else if (probeMode == 2) {     // getNormal(p)
        vec3 p = vec3(pin[3 * i], pin[3 * i + 1], pin[3 * i + 2]);
        vec3 n = getNormal(p);
        pout[3 * i] = n.x; pout[3 * i + 1] = n.y; pout[3 * i + 2] = n.z;
    } else if (probeMode == 3) {     // rand chain of 4 calls with seeds pin[8i..8i+7]
        for (int k = 0; k < 4; k++) pout[4 * i + k] = rand(vec2(pin[8 * i + 2 * k], pin[8 * i + 2 * k + 1]));
    } else if (probeMode == 4) {     // randHemisphere(s1, s2, n) from randChange = pin[9i+8]
        randChange = pin[9 * i + 8];
        vec3 b = randHemisphere(vec2(pin[9 * i], pin[9 * i + 1]), vec2(pin[9 * i + 2], pin[9 * i + 3]),
                                vec3(pin[9 * i + 4], pin[9 * i + 5], pin[9 * i + 6]));
        pout[3 * i] = b.x; pout[3 * i + 1] = b.y; pout[3 * i + 2] = b.z;
    }
}
"""
PROBE_WL = r"""
void main() {}
"""


def probe(variant, scene, mode, inputs, n, out_per, params, time=0.0, width=64):
    """Evaluate a reference function on n inputs (invocation i at gid (i % width, i / width))."""
    src = shader_build.build(variant, scene, probe_main=PROBE_MAIN)
    lx, ly = shader_build.LOCAL[variant]
    gx = width // lx
    gy = int(math.ceil(n / float(width) / ly))
    lines = ["image 8 8"] + _uniform_lines(params, np.zeros(15, np.float32))
    lines += ["ui probeMode %d" % mode, "ui probeCount %d" % n]
    lines.append("run %.9g 0 0 0 0 0 %d %d" % (time, gx, gy))
    _, so = run_job(src, lines, None, ssbo_in=np.asarray(inputs, np.float32).ravel(), ssbo_out_n=n * out_per)
    return so.reshape(n, out_per)


def wl2rgb_probe(wls):
    """wavelengthToColor(uint) of RayMarch3.glsl on a list of wavelengths."""
    main = r"""
layout(std430, binding = 2) readonly buffer ProbeIn { float pin[]; };
layout(std430, binding = 3) writeonly buffer ProbeOut { float pout[]; };
uniform int probeCount;
void main()
{
    uint i = gl_GlobalInvocationID.y * gl_NumWorkGroups.x * gl_WorkGroupSize.x + gl_GlobalInvocationID.x;
    if (i >= uint(probeCount)) return;
    vec3 c = wavelengthToColor(uint(pin[i]));
    pout[3 * i] = c.r; pout[3 * i + 1] = c.g; pout[3 * i + 2] = c.b;
}
"""
    src = shader_build.build(3, None, probe_main=main)
    n = len(wls)
    gy = int(math.ceil(n / 64.0 / 16))
    lines = ["image 8 8", "ui probeCount %d" % n, "run 0 0 0 0 0 0 4 %d" % gy]
    _, so = run_job(src, lines, None, ssbo_in=np.asarray(wls, np.float32), ssbo_out_n=3 * n)
    return so.reshape(n, 3)


DISPLAY_HARNESS = os.path.join(REF_OUT, "display_harness")


def display(accum, centre, zoom, vmin, vmax, screen):
    """Graphics::Display (Graphics.cpp:356-390) with the reference's FullQuad.vs / FullQuad.fs on
    llvmpipe: accum (H, W, 4) float32 (row 0 = the texture's first row), screen (h, w, 4) uint8 with
    row 0 = top (the window's coordinates). Returns the drawn screen, row 0 = top."""
    if not os.path.exists(DISPLAY_HARNESS):
        subprocess.check_call(["make", "-s", "-C", HERE])
    acc = np.ascontiguousarray(accum, np.float32)
    H, W = acc.shape[:2]
    scr = np.ascontiguousarray(screen, np.uint8)
    sh, sw = scr.shape[:2]
    with tempfile.TemporaryDirectory() as td:
        pa, pb, po = (os.path.join(td, n) for n in ("acc.f32", "bg.rgba8", "out.rgba8"))
        acc.tofile(pa)
        scr[::-1].tofile(pb)   # GL rows bottom-up
        args = [DISPLAY_HARNESS, os.path.join(shader_build.REF, "FullQuad.vs"), os.path.join(shader_build.REF, "FullQuad.fs"),
                pa, str(W), str(H), pb, str(sw), str(sh)]
        args += ["%.9g" % float(v) for v in (centre[0], centre[1], zoom, vmin[0], vmin[1], vmax[0], vmax[1])]
        args.append(po)
        r = subprocess.run(args, capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            raise RuntimeError("display harness failed (%d): %s" % (r.returncode, r.stderr[-4000:]))
        out = np.fromfile(po, np.uint8).reshape(sh, sw, 4)[::-1].copy()
    return out
