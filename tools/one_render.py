import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from raymarchrenderer_amd import Renderer, abi, time_schedule
r = Renderer(0, 1920, 1080); r.set_jit(1)
r.set_schedule(int(sys.argv[1])); r.set_tuning(20, -1, -1)
r.load_scene(os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "scenes/cornell5.scene"), "rm1")
r.set_params(abi.default_params(max_bounces=4)); r.reload()
for _ in range(2): r.render_spp(time_schedule(16))
print(r.stats().trace_ms); r.close()
