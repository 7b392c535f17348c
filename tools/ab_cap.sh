set -e
mkdir -p gpurun_out/cap2
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/cap2/t.log 2>&1
for r in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export SPIS_LIBRARY=$PWD/ab_old_libspis.so; else unset SPIS_LIBRARY; fi
    timeout -k 10 150 python -u bench.py --no-cpu-baseline > gpurun_out/cap2/c3_${v}_$r.log 2>&1
    echo "c3 $v $r $(tail -1 gpurun_out/cap2/c3_${v}_$r.log | cut -c100-140)"
  done
done
for cfg in c5 c4 c2; do
  for v in new old; do
    if [ $v = old ]; then export SPIS_LIBRARY=$PWD/ab_old_libspis.so; else unset SPIS_LIBRARY; fi
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --config $cfg > gpurun_out/cap2/${cfg}_${v}.log 2>&1
    echo "$cfg $v $(tail -1 gpurun_out/cap2/${cfg}_${v}.log | cut -c100-140)"
  done
done
