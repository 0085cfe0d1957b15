set -o pipefail
mkdir -p gpurun_out
for pat in range stride; do for w in 64 96 128; do
  PATTERN=$pat timeout -k 10 120 python -u tools/staged_probe.py c2 $w 1 100 || exit 1
done; done
