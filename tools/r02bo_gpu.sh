set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_utf8.py > gpurun_out/pytest_u8.log 2>&1 || { tail -40 gpurun_out/pytest_u8.log; exit 1; }
tail -1 gpurun_out/pytest_u8.log
for i in 1 2; do
timeout -k 10 300 python3 tools/cfg_bench.py TEXT > gpurun_out/cfg_t.json 2>gpurun_out/cfg.err || { tail -20 gpurun_out/cfg.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/cfg_t.json'))
for k,v in d.items(): print(k[:44], {x: v.get(x) for x in ('ms','gib_s','walk_ms','unmask_ms','u8_ms','device_errors')})"
done
