set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for f in 0 1 2; do
  WSC_EVENT_FENCE=$f timeout -k 10 200 python -u bench.py --no-echo --no-cpu --no-host-inclusive --no-other-configs --no-config3 > gpurun_out/bench_f$f.json 2>/dev/null || exit 1
done
WSC_EVENT_FENCE=2 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "split" > gpurun_out/pytest_split.log 2>&1 || exit 1
