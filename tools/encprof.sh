# Encode kernels alone (tools/enc_one.py), in-tree library vs an A/B build (tools/build_variant.sh): kernel trace + SQ
# instruction / wave-cycle counters, one pass each.   bash tools/encprof.sh <lib_b.so> [1k|64k]
set -e
cd /tmp; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; o=$R/gpurun_out/encprof; rm -rf $o; mkdir -p $o
for v in a b; do
  if [ $v = a ]; then L=$R/netman_amd/libwscodec.so; else L=$R/$1; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $o/t_$v -o run -- python3 $R/tools/enc_one.py $L $2 > $o/t_$v.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAVES -d $o/p_$v -o run --output-format csv -- python3 $R/tools/enc_one.py $L $2 > $o/p_$v.log 2>&1
done
echo done
