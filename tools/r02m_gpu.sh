set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "split_pipeline or staged" > gpurun_out/pytest_staged.log 2>&1 || { tail -30 gpurun_out/pytest_staged.log; exit 1; }
tail -3 gpurun_out/pytest_staged.log
for st in 1 0 1; do
  timeout -k 10 200 python -u bench.py --no-echo --no-cpu --no-host-inclusive --no-other-configs --no-config3 --staged $st > gpurun_out/bench_st$st.json 2>gpurun_out/bench_st.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/bench_st$st.json')); print($st, d['value'], d['ms_per_step'], d['single_batch'], d['parity_ok'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_staged2 -- python3 bench.py --no-echo --no-cpu --no-host-inclusive --no-other-configs --no-config3 --steps 40 > gpurun_out/kt_staged.log 2>&1 || exit 1
