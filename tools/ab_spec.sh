# A/B of the walk's speculation depth (headers fetched per memory round trip): libraries built with
# -DWSC_WALK_SPEC=N into abl/ (SPECS="4 8 16" by default; EXTRA adds config name fragments), alternated twice on one box over the many-frame configs
set -e
for r in 1 2; do
  for d in ${SPECS:-4 8 16}; do
    echo "spec$d $(timeout -k 10 120 python3 tools/lib_ab.py abl/spec$d.so configs 'configs[2]' 'configs[1] 1M x 1 KiB BIN, 16' 'configs[4]' ${EXTRA:-})"
  done
done
