set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for v in 2 4; do
WSC_U8_CHAINS=$v timeout -k 10 300 python3 tools/cfg_bench.py TEXT "configs[2]" > gpurun_out/cfg_t.json 2>gpurun_out/cfg.err || { tail -20 gpurun_out/cfg.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/cfg_t.json'))
for k,v in d.items(): print('$v', k[:44], {x: v.get(x) for x in ('ms','gib_s','walk_ms','unmask_ms','u8_ms','pipelined_ms_per_batch','device_errors')})"
done
