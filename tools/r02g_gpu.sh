set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for wl in 64k 1k mixed mixed1 1k1; do
  timeout -k 10 120 python -u tools/decode_loop.py $wl 20 --time > gpurun_out/loop_$wl.log 2>&1 || exit 1
done
timeout -k 10 120 python -u tools/walk_stamps.py mixed > gpurun_out/stamps_mixed.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_1k1 -- python3 tools/decode_loop.py 1k1 30 > gpurun_out/kt_1k1.log 2>&1 || exit 1
