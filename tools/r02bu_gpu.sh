set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python3 tools/cfg_bench.py TEXT "configs[1] 1M x 1 KiB BIN, 16" "configs[2] 256k mixed 125" > gpurun_out/cfg_t.json 2>gpurun_out/cfg.err || { tail -20 gpurun_out/cfg.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/cfg_t.json'))
for k,v in d.items(): print(k[:44], {x: v.get(x) for x in ('ms','gib_s','walk_ms','unmask_ms','u8_ms','device_errors')})"
