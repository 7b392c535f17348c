# HEAD re-check: full GPU suite, smoke, the C3 line
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06rc
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > $o/tests.log 2>&1
tail -2 $o/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1
tail -1 $o/smoke.log
timeout -k 10 400 python3 bench.py > $o/c3.json 2> $o/c3.err
python3 -c "import json;d=json.load(open('$o/c3.json'));print('c3', d['value'], d['roofline']['frac'], d['roofline']['traffic'], d['wrapper']['frac_of_value'], d['cpu_baseline']['value'])"
