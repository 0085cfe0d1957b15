set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for wl in 64k 1k 1k1 mixed mixed1 frag; do
  timeout -k 10 120 python -u tools/decode_loop.py $wl 20 --time > gpurun_out/loop_$wl.log 2>&1 || exit 1
  WSC_U8_GRID=1 timeout -k 10 120 python -u tools/decode_loop.py $wl 20 --time > gpurun_out/loop_${wl}_u8g1.log 2>&1 || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_mixed -- python3 tools/decode_loop.py mixed 50 > gpurun_out/kt_mixed.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_1k -- python3 tools/decode_loop.py 1k 50 > gpurun_out/kt_1k.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
