set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2>gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bench.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac'])
for k,v in d.get('other_configs',{}).items(): print(k[:44], v.get('ms'), v.get('gib_s'), v.get('pipelined_ms_per_batch'), v.get('device_errors'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_bench -o kt -- python3 bench.py --steps 20 --no-cpu --no-host-inclusive --no-echo --no-other-configs --no-config3 > gpurun_out/kt_bench.log 2>&1 || { tail -20 gpurun_out/kt_bench.log; exit 1; }
echo prof done
