cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python3 -u tools/varbench.py $VARIANTS > gpurun_out/var.log 2>&1 || { echo VARFAIL; tail gpurun_out/var.log; exit 1; }
cat gpurun_out/var.log
