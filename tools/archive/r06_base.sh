set -e
mkdir -p gpurun_out/r06base
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r06base/c3.json 2> gpurun_out/r06base/c3.err
cat gpurun_out/r06base/c3.json
