#!/bin/bash
# csg256 (C4's scene) sweeps of load-time knobs: grid cell count and region pad
export RMR_LIB=diag   # tools run against the diagnostic build (env switches)
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 400 python tools/env_ab.py RMR_GRID_CELLS 1048576 2097152 4194304 8388608 --scenes csg256 --spp 8 --rounds 3 > gpurun_out/c4_cells.log 2>&1 || exit $?
cat gpurun_out/c4_cells.log
timeout -k 10 400 python tools/env_ab.py RMR_GRID_PAD 0.5 0.25 1.0 --scenes csg256 --spp 8 --rounds 3 > gpurun_out/c4_pad.log 2>&1 || exit $?
cat gpurun_out/c4_pad.log
timeout -k 10 60 python -c "
import time, os, sys
sys.path.insert(0, '.')
from raymarchrenderer_amd import Renderer
r = Renderer(0, 64, 64)
for cells in ('262144', '1048576', '2097152', '4194304'):
    os.environ['RMR_GRID_CELLS'] = cells
    t0 = time.perf_counter(); r.load_scene('scenes/csg256.scene', 'rm1'); print('grid', cells, 'load ms', round((time.perf_counter() - t0) * 1e3, 1))
" > gpurun_out/c4_gridtime.log 2>&1 || exit $?
cat gpurun_out/c4_gridtime.log
