for c in c1 c2 c11 c4 head; do
  python tools/single_loop.py $c 200
  WSC_AB_NO_U8=1 python tools/single_loop.py $c 200
done
