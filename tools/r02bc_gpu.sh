set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 4 2; do
  echo "== chains $v"
  WSC_U8_CHAINS=$v timeout -k 10 200 python3 tools/cfg_bench.py TEXT > gpurun_out/p$v.json 2>gpurun_out/p.err || { tail -5 gpurun_out/p.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/p$v.json'))
for k,v in d.items(): print(k[:20], {x: v.get(x) for x in ('ms','gib_s','walk_ms','unmask_ms','u8_ms','device_errors')})"
done
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2>gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bench.json'))
print(d['value'], d['ms_per_step'], d['roofline'])
for k,v in d.get('other_configs',{}).items(): print(k[:44], v.get('ms'), v.get('gib_s'), v.get('pipelined_gib_s'), v.get('device_errors'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_bench -o kt -- python3 bench.py --steps 20 --no-cpu --no-host-inclusive --no-echo --no-other-configs --no-config3 > gpurun_out/kt_bench.log 2>&1 || { tail -20 gpurun_out/kt_bench.log; exit 1; }
tail -1 gpurun_out/kt_bench.log
