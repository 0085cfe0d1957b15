set -o pipefail
mkdir -p gpurun_out
B="bench.py --no-echo --no-cpu --no-host-inclusive --no-other-configs --no-config3 --steps 100"
for v in 0 1; do
  WSC_STAGE_VARIANT=$v timeout -k 10 200 python -u $B > gpurun_out/v$v.json 2>gpurun_out/v.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/v$v.json')); print('v$v', d['value'], d['ms_per_step'], d['parity_ok'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_q -- python3 $B > gpurun_out/kt_q.log 2>&1 || exit 1
WSC_STAGE_VARIANT=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_q1 -- python3 $B > gpurun_out/kt_q.log 2>&1 || exit 1
