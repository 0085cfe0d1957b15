set -o pipefail
mkdir -p gpurun_out
B="python -u bench.py --no-echo --no-cpu --no-host-inclusive --no-other-configs --no-config3"
run() { tag=$1; shift; timeout -k 10 200 $B "$@" > gpurun_out/ab_$tag.json 2>gpurun_out/ab.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab_$tag.json')); print('$tag', d['value'], d['ms_per_step'], d['parity_ok'])"; }
for rep in 1 2; do
run base$rep --steps 100
run us2_$rep --steps 100 --unmask-streams 2
run wc8_$rep --steps 100 --walk-cus 8
run p3_$rep --steps 100 --pipeline 3
run p3us2_$rep --steps 100 --pipeline 3 --unmask-streams 2
run st0_$rep --steps 100 --staged 0
done
