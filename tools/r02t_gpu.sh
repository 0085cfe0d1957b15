set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/cfg_bench.py > gpurun_out/cfg.json 2>gpurun_out/cfg.err || { tail -20 gpurun_out/cfg.err; exit 1; }
python - <<'PY'
import json
d=json.load(open('gpurun_out/cfg.json'))
for k,v in d.items(): print(k[:40], {x: v[x] for x in ('ms','gib_s','frac','walk_ms','unmask_ms','pipelined_ms_per_batch','pipelined_gib_s','device_errors')})
PY
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_cfg -- python3 tools/cfg_bench.py "configs[1] 1M x 1 KiB BIN, 16" "configs[2]" > gpurun_out/kt_cfg.log 2>&1 || exit 1
