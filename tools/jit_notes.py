"""Registers, spills and scratch of the hipRTC code object of every kernel class, read
from the code objects hipRTC writes (the compiler the product runs; a hipcc build of the same source
allocates differently). CPU only.   python tools/jit_notes.py [OUT]"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
S, G = os.path.join(ROOT, "scenes"), os.path.join(ROOT, "tests", "golden", "scenes")
CLASSES = [("C1 sphere", os.path.join(S, "sphere1.scene"), "rm1"),
           ("C2 / C5 Cornell-5 (approximate map, certified probes)", os.path.join(S, "cornell5.scene"), "rm1"),
           ("C3 Mandelbulb (stepped map)", os.path.join(S, "mandelbulb.scene"), "rm1"),
           ("C4 csg256 (cache + grid)", os.path.join(S, "csg256.scene"), "rm1"),
           ("RM3 built-in", None, "rm3"),
           ("RM2 simple.scene", os.path.join(G, "simple.scene"), "rm2"),
           ("glass_test (node-program materials)", os.path.join(G, "glass_test.scene"), "rm1"),
           ("default.scene (node-program materials)", os.path.join(G, "default.scene"), "rm1"),
           ("multilight (node-program materials)", os.path.join(G, "multilight.scene"), "rm1"),
           ("csg_nodes (node-program objects)", os.path.join(S, "csg_nodes.scene"), "rm1")]
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def notes(path):
    text = subprocess.run([READELF, "--notes", path], capture_output=True, text=True, check=True).stdout
    out = {}
    for key in ("vgpr_count", "vgpr_spill_count", "sgpr_count", "private_segment_fixed_size"):
        m = re.search(r"\.%s:\s+(\d+)" % key, text)
        out[key] = int(m.group(1)) if m else None
    return out


def main(out=None):
    d = tempfile.mkdtemp()
    os.environ["RMR_JIT_CACHE"] = d
    from raymarchrenderer_amd.renderer import jit_compile_scene
    lines = ["| kernel class | VGPRs | spilled VGPRs | SGPRs | private segment (B) |", "|---|---|---|---|---|"]
    for name, path, variant in CLASSES:
        key = jit_compile_scene(path, variant)
        n = notes(os.path.join(d, key + ".hsaco"))
        lines.append("| %s | %d | %d | %d | %d |" % (name, n["vgpr_count"], n["vgpr_spill_count"], n["sgpr_count"],
                                                     n["private_segment_fixed_size"]))
    text = "\n".join(lines)
    print(text)
    if out:
        open(out, "w").write(text + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
