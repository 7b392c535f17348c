set -e
mkdir -p gpurun_out/r06spawn
timeout -k 10 200 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_multirank.py -k bench_spawns -m gpu > gpurun_out/r06spawn/test.log 2>&1
SPIS_DEVICE=0 SPIS_TRANSPORT=host timeout -k 10 200 python -u bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r06spawn/c3_2rank_full.json 2> gpurun_out/r06spawn/c3_2rank_full.err
cat gpurun_out/r06spawn/c3_2rank_full.json
