cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/ab.py raymarchrenderer_amd/librmr.so raymarchrenderer_amd/librmr_x.so raymarchrenderer_amd/librmr_y.so --rounds 6 > gpurun_out/ab1.log 2>&1
