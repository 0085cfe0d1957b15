#!/bin/bash
# encode copy: XCD runs (WSC_XCD_RUN=1 / 8), twice each, same box
for rep in 1 2; do
  for x in 1 8; do
    echo "=== WSC_XCD_RUN=$x rep $rep"
    WSC_XCD_RUN=$x timeout -k 10 200 python3 tools/enc_only.py || exit $?
  done
done
