set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do for lib in head cur; do
  if [ $lib = head ]; then export WSC_LIB=$PWD/netman_amd/libwscodec_head.so; else unset WSC_LIB; fi
  for w in c1 head; do echo -n "$lib "; timeout -k 10 120 python -u tools/single_loop.py $w 30 || exit 1; done
done; done
