set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/pytest_p.log 2>&1 || { tail -40 gpurun_out/pytest_p.log; exit 1; }
tail -1 gpurun_out/pytest_p.log
timeout -k 10 500 python3 tools/cfg_bench.py "configs[1]" "configs[2]" "configs[4]" TEXT > gpurun_out/cfg_all.json 2>gpurun_out/cfg.err || { tail -20 gpurun_out/cfg.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/cfg_all.json'))
for k,v in d.items(): print(k[:44], {x: v.get(x) for x in ('ms','gib_s','walk_ms','unmask_ms','u8_ms','pipelined_ms_per_batch','device_errors')})"
