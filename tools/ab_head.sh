#!/bin/bash
# headline unmask geometry: window 4 / 8 KiB x XCD run length, 200 steps each, twice
HL="--steps 200 --warmup 10 --no-cpu --no-host-inclusive --no-echo --no-other-configs --no-config3"
for rep in 1 2; do
  for w in 4096 8192; do
    for x in 4 8 16; do
      echo "=== window $w WSC_XCD_RUN=$x rep $rep"
      WSC_XCD_RUN=$x timeout -k 10 120 python3 bench.py $HL --window $w || exit $?
    done
  done
done
