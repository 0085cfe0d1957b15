set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_utf8.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_walk.log 2>&1 || exit 1
for wl in 64k 1k 1k1 mixed mixed1 frag; do
  timeout -k 10 120 python -u tools/decode_loop.py $wl 20 --time > gpurun_out/loop_$wl.log 2>&1 || exit 1
done
for wl in mixed 1k; do
  timeout -k 10 120 python -u tools/walk_stamps.py $wl > gpurun_out/stamps_$wl.log 2>&1 || exit 1
done
