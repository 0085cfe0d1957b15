set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/full_bench.json 2>gpurun_out/full_bench.err || { tail -20 gpurun_out/full_bench.err; exit 1; }
tail -c 3000 gpurun_out/full_bench.json
