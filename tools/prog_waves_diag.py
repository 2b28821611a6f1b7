"""Diagnostics for the node-program-material kernel built at a forced wave target (RMR_PROG_WAVES):
renders per-sample planes of a scene with the default build and with each -DRMR_PROG_WAVES=N build
(RMR_JIT_OPTS, diagnostic library), counts the samples that differ bitwise from the default build and
saves every plane to an .npz for offline analysis against the CPU oracle (tools/prog_waves_cmp.py).

    python tools/prog_waves_diag.py --scene tests/golden/scenes/glass_test.scene --waves 6,7 --out gpurun_out/pw.npz
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("RMR_LIB", "diag")   # tools run against the diagnostic build (env switches)
import numpy as np  # noqa: E402
from raymarchrenderer_amd import Renderer, abi, time_schedule  # noqa: E402
from oracle import camera  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scene", default=os.path.join(ROOT, "tests", "golden", "scenes", "glass_test.scene"))
ap.add_argument("--waves", default="7")
ap.add_argument("--extra", default="", help="further RMR_JIT_OPTS words for the forced builds")
ap.add_argument("--spp", type=int, default=4)
ap.add_argument("--bounces", type=int, default=16)
ap.add_argument("--W", type=int, default=256)
ap.add_argument("--H", type=int, default=96)
ap.add_argument("--out", default="")
a = ap.parse_args()

prm = abi.default_params(max_bounces=a.bounces)
view = camera.default_view(a.W, a.H)
times = time_schedule(a.spp)
r = Renderer(0, a.W, a.H)
r.set_jit(1)
planes = {}
for w in ["default"] + a.waves.split(","):
    if w == "default":
        os.environ.pop("RMR_JIT_OPTS", None)
    else:
        os.environ["RMR_JIT_OPTS"] = ("-DRMR_PROG_WAVES=%s %s" % (w, a.extra)).strip()
    r.load_scene(a.scene, "rm1")
    r.set_params(prm)
    r.set_view(view)
    r.reload()
    planes[w] = r.trace_samples(times, (0, 0, a.W, a.H))
    d = planes[w].view(np.uint32) != planes["default"].view(np.uint32)
    print("waves %s: %d of %d samples differ from the default build" % (w, int(np.any(d, -1).sum()), d.shape[0] * d.shape[1] * d.shape[2]),
          flush=True)
r.close()
if a.out:
    np.savez_compressed(a.out, times=times, W=a.W, H=a.H, bounces=a.bounces, scene=a.scene,
                        **{"w_" + k: v for k, v in planes.items()})
