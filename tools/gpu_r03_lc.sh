set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03lc
timeout -k 10 400 python -u tools/lc_probe.py > gpurun_out/r03lc/probe.jsonl 2> gpurun_out/r03lc/probe.err
