set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "split or staged or geometr" > gpurun_out/pytest_geo.log 2>&1 || { tail -30 gpurun_out/pytest_geo.log; exit 1; }
tail -1 gpurun_out/pytest_geo.log
timeout -k 10 200 python -u bench.py --no-echo --no-cpu --no-host-inclusive --no-other-configs --no-config3 > gpurun_out/hb.json 2>gpurun_out/hb.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/hb.json')); print('head', d['value'], d['ms_per_step'])"
timeout -k 10 400 python -u tools/cfg_bench.py > gpurun_out/cfg.json 2>gpurun_out/cfg.err || { tail -20 gpurun_out/cfg.err; exit 1; }
python - <<'PY'
import json
d=json.load(open('gpurun_out/cfg.json'))
for k,v in d.items(): print(k[:40], {x: v[x] for x in ('ms','gib_s','pipelined_ms_per_batch','pipelined_gib_s','pipelined_walk_cus','pipelined_unmask_cus','device_errors')})
PY
