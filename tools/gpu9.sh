cd $GRAFT_REPO_ROOT
timeout -k 10 400 python tools/ab.py raymarchrenderer_amd/librmr_a.so raymarchrenderer_amd/librmr_d.so raymarchrenderer_amd/librmr_e.so raymarchrenderer_amd/librmr_f.so --rounds 6 > gpurun_out/ab3.log 2>&1
