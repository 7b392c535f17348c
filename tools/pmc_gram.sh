cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "bm|200|python bench.py --gram mfma --no-cpu-baseline" \
 "f_m|120|timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_gm -o fetch -- python3 bench.py --gram mfma --no-cpu-baseline --steps 2 --warmup 1" \
 "h_m|120|timeout -s KILL 100 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc_gm -o hit -- python3 bench.py --gram mfma --no-cpu-baseline --steps 2 --warmup 1" \
 "f_e|120|timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_ge -o fetch -- python3 bench.py --gram ell --no-cpu-baseline --steps 2 --warmup 1" \
 "h_e|120|timeout -s KILL 100 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc_ge -o hit -- python3 bench.py --gram ell --no-cpu-baseline --steps 2 --warmup 1"
