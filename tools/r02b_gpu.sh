set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_run.sh "pytest_gpu:600:python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" || exit 1
for wl in 1k mixed 1k1 mixed1 frag; do
  timeout -k 10 120 python -u tools/walk_stamps.py $wl > gpurun_out/stamps_$wl.log 2>&1 || exit 1
done
for wl in 1k mixed; do
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_${wl}_fetch -- python3 tools/decode_loop.py $wl 20 > gpurun_out/pmc_${wl}_fetch.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_${wl}_write -- python3 tools/decode_loop.py $wl 20 > gpurun_out/pmc_${wl}_write.log 2>&1 || exit 1
done
timeout -k 10 400 python -u bench.py --no-echo > gpurun_out/bench_b.json 2> gpurun_out/bench_b.err || exit 1
