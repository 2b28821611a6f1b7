"""GPU renders of the converged-parity cases on parity_schedule, saved for offline analysis:
gpurun_out/diag_psnr.npz (one HxWx4 image per case)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("RMR_LIB", "diag")   # tools run against the diagnostic build (env switches)
import numpy as np  # noqa: E402

from raymarchrenderer_amd import Renderer, abi, parity_schedule  # noqa: E402
from tests.test_gpu_reference_psnr import CASES  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")
out = {}
r = Renderer(0, 64, 48)
for name, (path, variant, kw, _floor) in sorted(CASES.items()):
    g = np.load(os.path.join(GOLDEN, "img_%s.npz" % name))
    H, W = g["conv"].shape[:2]
    n = int(g["spp_conv"]) * int(os.environ.get("DIAG_MULT", "1"))
    r.set_image_size(W, H)
    r.reload()
    if path is None:
        r.load_builtin(variant)
    else:
        r.load_scene(path, variant)
    r.set_params(abi.default_params(**kw))
    r.set_view(g["view"])
    r.render_spp(parity_schedule(n))
    out[name] = r.read_accum()
    print(name, n, float(out[name][..., :3].mean()), float(g["conv"][..., :3].mean()), flush=True)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", "diag_psnr.npz"), **out)
