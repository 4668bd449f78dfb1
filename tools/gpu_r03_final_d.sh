# small-batch round phases (opt-in) A/B, then the final-library validation (C)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 bash tools/gpu_r03_rsmall.sh || exit 1
timeout -k 10 1000 bash tools/gpu_r03_final_c.sh || exit 1
