set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_session.py tests/test_gpu_utf8.py > gpurun_out/pytest_s.log 2>&1 || { tail -40 gpurun_out/pytest_s.log; exit 1; }
tail -2 gpurun_out/pytest_s.log
timeout -k 10 300 python -u tools/cfg_bench.py TEXT > gpurun_out/cfg_text.json 2>gpurun_out/cfg.err || { tail -20 gpurun_out/cfg.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/cfg_text.json'))
for k,v in d.items(): print(k[:40], {x: v.get(x) for x in ('ms','gib_s','walk_ms','unmask_ms','u8_ms','pipelined_ms_per_batch','device_errors')})"
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
