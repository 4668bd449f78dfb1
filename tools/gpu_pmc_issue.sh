# PMC issue probe of the replay kernels: instructions per op by class and
# active-issue cycles (is pass 1 issue-bound or latency-bound?).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --ops ${OPS:-2000}"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAVES --kernel-trace -d gpurun_out/pmci1 -o run --output-format csv -- $B > gpurun_out/pmci1.log 2>&1 || { echo PMCI1FAIL; tail gpurun_out/pmci1.log; exit 1; }
echo ALLOK
# second pass: scalar / LDS issue and stalls
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAVES --kernel-trace -d gpurun_out/pmci2 -o run --output-format csv -- $B > gpurun_out/pmci2.log 2>&1 || { echo PMCI2FAIL; tail gpurun_out/pmci2.log; exit 1; }
echo ALLOK2
