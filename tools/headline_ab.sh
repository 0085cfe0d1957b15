#!/bin/bash
# headline A/B: bench.py's headline leg only, alternating the given extra-argument sets
# usage: bash tools/headline_ab.sh "<args A>" "<args B>" ...
for rep in 1 2; do
  for args in "$@"; do
    timeout -k 10 120 python3 bench.py --steps 200 --no-cpu --no-host-inclusive --no-echo --no-other-configs --no-config3 $args > /tmp/hl.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open('/tmp/hl.json').read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['kernel_ms']['unmask'])" "$args"
  done
done
