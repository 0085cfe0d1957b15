# A/B of the walk for many short segments: tiled (default) vs the three-launch walk (WSC_WALK_TILED=0)
for c in c11 c21; do
  python tools/single_loop.py $c 200
  WSC_WALK_TILED=0 python tools/single_loop.py $c 200
done
