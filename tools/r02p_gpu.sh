set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/hbm_ceiling 1073741824 sweep > gpurun_out/hbm_policy.log 2>&1 || exit 1
cat gpurun_out/hbm_policy.log
