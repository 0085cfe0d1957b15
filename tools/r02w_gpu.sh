set -o pipefail
mkdir -p gpurun_out
for w in c1 head c2; do timeout -k 10 120 python -u tools/single_loop.py $w 50 || exit 1; done
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "fuzz or edge or tiny or config1 or config2 or golden or split" > gpurun_out/pytest_lanes.log 2>&1 || { tail -30 gpurun_out/pytest_lanes.log; exit 1; }
tail -2 gpurun_out/pytest_lanes.log
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU --output-format csv -d gpurun_out/pmc_c1_sq2 -- python3 tools/single_loop.py c1 5 > gpurun_out/pmc_c1_sq2.log 2>&1 || exit 1
