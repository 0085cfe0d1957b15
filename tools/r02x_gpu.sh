set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/walk_stamps.py 1k > gpurun_out/stamps_1k.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/walk_stamps.py mixed > gpurun_out/stamps_mixed.log 2>&1 || exit 1
tail -4 gpurun_out/stamps_1k.log; tail -4 gpurun_out/stamps_mixed.log
for w in c1 c2 head; do
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_$w -- python3 tools/single_loop.py $w 3 > /dev/null 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_$w -- python3 tools/single_loop.py $w 3 > /dev/null 2>&1 || exit 1
done
