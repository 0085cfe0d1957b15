set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in t64 t1; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_$w -o kt -- python3 tools/single_loop.py $w 20 > gpurun_out/$w.log 2>&1 || { tail -20 gpurun_out/$w.log; exit 1; }
grep "$w:" gpurun_out/$w.log
f=$(find gpurun_out/kt_$w -name '*kernel_stats.csv' | head -1); cut -d, -f1-4 "$f" | grep wsc
done
