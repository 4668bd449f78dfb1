# round 4: the HBM tree pass on the GPU (local-client and long legacy documents)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_htree.py tests/test_reconnect.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/htree.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
