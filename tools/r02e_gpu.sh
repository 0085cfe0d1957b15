set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for wl in mixed 1k 1k1; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d gpurun_out/sq_$wl -- python3 tools/decode_loop.py $wl 10 > gpurun_out/sq_$wl.log 2>&1 || exit 1
done
