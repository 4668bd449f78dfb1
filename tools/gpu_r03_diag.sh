set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03diag
MTE_WAVE_CLOCK=/tmp/wclock.bin timeout -k 10 300 python -u tools/rsmall_diag.py 1250 > gpurun_out/r03diag/diag.json 2> gpurun_out/r03diag/diag.err
