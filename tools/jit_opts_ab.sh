export RMR_LIB=diag   # tools run against the diagnostic build (env switches)
cd /root/repo
for o in "" "-mllvm -amdgpu-early-ifcvt=1" "-mllvm -amdgpu-sched-strategy=max-ilp" "-mllvm -amdgpu-schedule-metric-bias=0" "-mllvm -amdgpu-sched-strategy=iterative-ilp"; do
  RMR_JIT_OPTS="$o" timeout -k 10 200 python tools/stats_run.py --spp 32 2>&1 | grep -v amdgpu.ids | sed "s|^|[$o] |" || exit 1
done
