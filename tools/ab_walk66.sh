# Walk geometry A/B: the 64 walking columns of a 256-lane block spread 16 per wave (mode 66) vs one
# walking wave (mode 65), same blocks and look-back; geometry tests first
set -e
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q -k walk_geometries --timeout 120 --timeout-method thread -p no:cacheprovider
for r in 1 2; do
  for c in c2 t1 t64; do
    for m in 65 66; do
      echo "== $c mode $m"; WSC_WALK_MODE=$m timeout -k 10 120 python3 tools/single_loop.py $c 200
    done
  done
done
for m in 65 66; do echo "== stamps mode $m"; WSC_WALK_MODE=$m timeout -k 10 120 python3 tools/walk_stamps.py mixed; done
