# A/B of the walk's speculation depth (headers fetched per memory round trip): libraries built with
# -DWSC_WALK_SPEC=4/8/16 into abl/, alternated twice on one box over the many-frame configs
set -e
for r in 1 2; do
  for d in 4 8 16; do
    echo "spec$d $(timeout -k 10 120 python3 tools/lib_ab.py abl/spec$d.so configs 'configs[2]' 'configs[1] 1M x 1 KiB BIN, 16' 'configs[4]')"
  done
done
