set -o pipefail
mkdir -p gpurun_out
for v in "WSC_U8_CHAINS=1" "WSC_U8_CHAINS=4" "WSC_U8_GRID=512" "WSC_U8_GRID=2048"; do
  echo "== $v"
  env $v timeout -k 10 200 python3 tools/cfg_bench.py "TEXT 262144" > gpurun_out/p.json 2>gpurun_out/p.err || { tail -5 gpurun_out/p.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/p.json'))
for k,v in d.items(): print(k[:20], {x: v.get(x) for x in ('ms','gib_s','walk_ms','unmask_ms','u8_ms','device_errors')})"
done
