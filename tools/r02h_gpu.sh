set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for g in 1280 256 64; do
  WSC_U8_GRID=$g timeout -k 10 120 python -u tools/decode_loop.py mixed 20 --time > gpurun_out/loop_mixed_g$g.log 2>&1 || exit 1
done
timeout -k 10 400 python -u bench.py --no-echo --no-cpu --no-host-inclusive > gpurun_out/bench_h.json 2> gpurun_out/bench_h.err || exit 1
