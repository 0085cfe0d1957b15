#!/bin/bash
# configs[3] dealt-leg A/B: the split pipeline at several walk CU counts vs serial decodes
for rep in 1 2; do
  for v in "" "WSC_C3_WALK_CUS=16" "WSC_C3_WALK_CUS=48" "WSC_C3_SERIAL=1"; do
    env $v timeout -k 10 200 python3 bench.py --steps 30 --no-cpu --no-host-inclusive --no-echo --no-other-configs > /tmp/c3.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open('/tmp/c3.json').read().strip().splitlines()[-1]); c=d['configs3_dealt']; print(sys.argv[1] or 'default', c['gib_s'], c['ms_per_step'], c['parity_ok'])" "$v"
  done
done
