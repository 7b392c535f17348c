set -e
for r in 1 2 3; do
  for opt in "" "--graphs" "--no-fuse"; do
    v=$(python bench.py --no-cpu-baseline --steps 20 $opt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']), round(d['kernels']['iteration_us'],1))")
    echo "run$r [$opt] $v"
  done
done
