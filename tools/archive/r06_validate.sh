# Round 6 measurement set on one box: rocprofv3 kernel stats of the C3 bench, PMC traffic (two
# passes), the C3 line as the driver runs it, and the other configurations' lines.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06v
mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-wrapper --no-cold > $o/prof_bench.json 2> $o/prof_bench.err
echo "rocprof done"
bash tools/r06_pmc.sh c3
echo "pmc done"
timeout -k 10 400 python3 bench.py > $o/c3_default.json 2> $o/c3_default.err
python3 -c "import json;d=json.load(open('$o/c3_default.json'));print('c3', d['value'], d['roofline']['frac'], d['roofline']['traffic'], d['wrapper']['frac_of_value'], d['cpu_baseline']['value'])"
for cfg in c2 c4; do
  timeout -k 10 300 python3 bench.py --config $cfg --no-cpu-baseline --no-cold > $o/${cfg}.json 2> $o/${cfg}.err
  python3 -c "import json;d=json.load(open('$o/${cfg}.json'));print('$cfg', d['value'], d['roofline']['frac'])"
done
timeout -k 10 300 python3 bench.py --tol 1e-7 --no-cpu-baseline --no-cold --no-wrapper > $o/c3_tol7.json 2> $o/c3_tol7.err
timeout -k 10 300 python3 bench.py --method cgmres_p --no-cpu-baseline --no-cold --no-wrapper > $o/c3_p.json 2> $o/c3_p.err
timeout -k 10 300 python3 bench.py --force-distributed --steps 20 --no-cpu-baseline > $o/dist1.json 2> $o/dist1.err
python3 -c "
import json
for f in ('c3_tol7','c3_p','dist1'):
    d=json.load(open('$o/'+f+'.json')); print(f, d['value'])"
timeout -k 10 600 python3 bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-cold > $o/c5.json 2> $o/c5.err
python3 -c "import json;d=json.load(open('$o/c5.json'));print('c5', d['value'], d['roofline']['frac'])"
