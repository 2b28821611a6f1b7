export RMR_LIB=diag   # tools run against the diagnostic build (env switches)
cd /root/repo
for o in -O3 -DRMR_CHUNK=64 -DRMR_CHUNK=32; do
  for spp in 4 16 64; do
    RMR_JIT_OPTS="$o" timeout -k 10 100 python tools/stats_run.py --spp $spp 2>&1 | grep -v amdgpu.ids | cut -c1-75 | sed "s/^/[$o spp=$spp] /" || exit 1
  done
done
