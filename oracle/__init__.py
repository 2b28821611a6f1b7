"""oracle — TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference hot path (liboracle.so + scene_compile.py + camera.py) and the
llvmpipe harness that pins it to the reference GLSL. Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import it; the product (raymarchrenderer_amd, librmr.so) never does.
"""
