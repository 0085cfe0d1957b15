# Walk geometry A/B: 64-lane blocks whose first 16 / 32 lanes walk (modes 16, 32) vs one walking
# wave per CU (mode 65), on the configs with up to 64 segments per CU; geometry tests first
set -e
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q -k walk_geometries --timeout 120 --timeout-method thread -p no:cacheprovider
for r in 1 2; do
  for c in c2 t1 t64; do
    for m in 65 16 32; do
      echo "== $c mode $m"; WSC_WALK_MODE=$m timeout -k 10 120 python3 tools/single_loop.py $c 200
    done
  done
done
