set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/gap_probe.py > gpurun_out/gap_probe.log 2>&1 || exit 1
for g in 64 1280; do
  WSC_U8_GRID=$g timeout -k 10 200 python -u bench.py --no-echo --no-cpu --no-host-inclusive --no-other-configs --no-config3 > gpurun_out/bench_u8g$g.json 2>/dev/null || exit 1
done
