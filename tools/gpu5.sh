cd $GRAFT_REPO_ROOT
bash tools/pmc.sh pmc2 --spp 16 --steps 1 --warmup 0 --no-cpu-baseline
