set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06wtt
mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -v --timeout 170 --timeout-method thread tests/test_gpu_parity.py tests/test_abi.py -m gpu -k "write_through or abi or golden" > $o/tests.log 2>&1
tail -3 $o/tests.log
