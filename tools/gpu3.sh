cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 tools/probes/sqrt_exhaustive > gpurun_out/sqrt_exhaustive.log 2>&1 || exit $?
bash tools/pmc.sh pmc1
