set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_bench -- python3 bench.py --no-echo --no-cpu --no-host-inclusive --no-other-configs --no-config3 --steps 40 > gpurun_out/kt_bench.log 2>&1 || exit 1
