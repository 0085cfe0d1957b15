set -o pipefail
mkdir -p gpurun_out
for w in c2 c1; do for wc in 16 32 64 128; do for rest in 0 1; do
  timeout -k 10 120 python -u tools/staged_probe.py $w $wc $rest || exit 1
done; done; done
for rest in 0 1; do timeout -k 10 120 python -u tools/staged_probe.py head 16 $rest || exit 1; done
