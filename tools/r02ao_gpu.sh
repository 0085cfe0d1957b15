set -o pipefail
mkdir -p gpurun_out
for m in 0 64; do for rep in 1 2; do
  WSC_WALK_MODE=$m timeout -k 10 200 python -u bench.py --no-echo --no-cpu --no-host-inclusive --no-other-configs --no-config3 > gpurun_out/hb.json 2>gpurun_out/hb.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/hb.json')); print('mode $m head', d['value'], d['ms_per_step'])"
done; done
timeout -k 10 120 python -u tools/staged_probe.py c3 128 0 || exit 1
timeout -k 10 120 python -u tools/staged_probe.py c3 16 0 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_c3 -- python3 tools/staged_probe.py c3 128 0 20 > /dev/null 2>&1 || exit 1
