set -e
python tools/dump_matrix.py 289 /tmp/kbench_mat
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gap -o run -- tools/kbench /tmp/kbench_mat gap
