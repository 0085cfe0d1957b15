set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_session.py tests/test_gpu_utf8.py > gpurun_out/pytest_s.log 2>&1 || { tail -40 gpurun_out/pytest_s.log; exit 1; }
tail -1 gpurun_out/pytest_s.log
timeout -k 10 300 python3 tools/cfg_bench.py TEXT > gpurun_out/cfg_text_noprof.json 2>gpurun_out/cfg2.err || { tail -20 gpurun_out/cfg2.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/cfg_text_noprof.json'))
for k,v in d.items(): print(k[:40], {x: v.get(x) for x in ('ms','gib_s','frac','walk_ms','unmask_ms','u8_ms','device_errors')})"
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
