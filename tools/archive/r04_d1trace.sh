set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${1:-gpurun_out/r04d1}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 -u bench.py --force-distributed --steps 10 --warmup 2 --no-cpu-baseline > $O/d1.json 2> $O/d1.err
f=$(find $O/prof -name '*kernel_trace.csv' | head -n 1); cp "$f" $O/trace.csv
python tools/trace_gaps.py $O/trace.csv > $O/gaps.txt
