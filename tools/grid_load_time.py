"""Scene-load time of csg256 per candidate-grid size (RMR_GRID_CELLS), and without the grid."""
import os, sys, time
sys.path.insert(0, os.getcwd())
os.environ.setdefault("RMR_LIB", "diag")   # tools run against the diagnostic build (env switches)
from raymarchrenderer_amd import Renderer
r = Renderer(0, 256, 256)
for cells in ("65536", "131072", "262144", "524288", "1048576"):
    os.environ["RMR_GRID_CELLS"] = cells
    t = time.time(); r.load_scene("scenes/csg256.scene", "rm1"); print("cells", cells, "load_scene s", round(time.time() - t, 3), flush=True)
os.environ["RMR_GRID"] = "0"
t = time.time(); r.load_scene("scenes/csg256.scene", "rm1"); print("no grid load_scene s", round(time.time() - t, 3))
