#!/bin/bash
# Headline warm-up A/B (bench.py --settle self|gen), fresh processes
# alternating, the driver's command shape otherwise (--steps 20 --warmup 5).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r7n}
mkdir -p $O
for i in 1 2 3 4; do
  for m in self gen; do
    timeout -k 10 120 python3 $R/bench.py --steps 20 --warmup 5 --no-extras --no-cpu --no-gather --settle $m > $O/h_${m}_$i.json 2>/dev/null || exit 1
    python3 -c "import json,sys; j=json.load(open('$O/h_${m}_$i.json')); print('$m', j['value'], j['roofline']['frac'], j['roofline']['clock']['clock_GHz'])"
  done
done
