set -o pipefail
mkdir -p gpurun_out
B="bench.py --no-echo --no-cpu --no-host-inclusive --no-other-configs --no-config3 --steps 100"
for rep in 1 2; do for u in 0 1 2 3; do
  WSC_UNMASK_BUF=$u timeout -k 10 200 python -u $B > gpurun_out/u$u.json 2>gpurun_out/v.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/u$u.json')); print('buf$u', d['value'], d['ms_per_step'], d['single_batch'], d['parity_ok'])"
done; done
WSC_UNMASK_BUF=2 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/pytest_buf.log 2>&1 || { tail -30 gpurun_out/pytest_buf.log; exit 1; }
tail -2 gpurun_out/pytest_buf.log
