export RMR_LIB=diag   # tools run against the diagnostic build (env switches)
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_ANY -d gpurun_out/pmcab -o run --output-format csv -- python3 tools/env_ab.py RMR_JIT_APPROX 1 0 --scenes cornell5 --rounds 1 > gpurun_out/pmcab.log 2>&1
