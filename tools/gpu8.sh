cd $GRAFT_REPO_ROOT
timeout -k 10 400 python tools/ab.py raymarchrenderer_amd/librmr_x.so raymarchrenderer_amd/librmr_a.so raymarchrenderer_amd/librmr_b.so raymarchrenderer_amd/librmr_c.so --rounds 6 > gpurun_out/ab2.log 2>&1
