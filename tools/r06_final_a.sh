# Round 6 final check, part A (one box): the full GPU suite, smoke, the rocprofv3 kernel trace of the
# C3 bench (stats CSV + timeline), PMC traffic at HEAD for C3, C2 and C4 (tools/r06_pmc.sh)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06fa
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > $o/tests.log 2>&1
tail -2 $o/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1
tail -1 $o/smoke.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-wrapper --no-cold > $o/prof_bench.json 2> $o/prof_bench.err
python3 tools/rocpd_stats.py $o/prof/run_results.db $o/c3_kernel_stats.csv
python3 tools/rocpd_timeline.py $o/prof/run_results.db 1 --iters > $o/c3_timeline.txt
head -14 $o/c3_timeline.txt
for cfg in c3 c2 c4; do
  bash tools/r06_pmc.sh $cfg
  cp gpurun_out/pmc_$cfg/r06_traffic_$cfg.json $o/
done
echo done
