#!/bin/bash
# one line per bench JSON: file, it/s, dominant launch us, iteration us
for f in "$@"; do
  [ -f "$f" ] || { echo "$f missing"; continue; }
  python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); k=d.get('kernels',{}); print('$f', round(d['value']), round(d['roofline']['avg_launch_us'],1), 'iter', round(k.get('iteration_us',0),1))"
done
