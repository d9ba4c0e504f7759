# Stripe-stride sweeps through tools/layout_ab.py (4 KiB vects unless SIZE
# says otherwise).  Output: gpurun_out/r02_layout_*.log
set -e
run() { CODEC=$1 CASE=$2 SIZE=${4:-4096} LAYOUTS=$3 ROUNDS=11 timeout -k 10 200 python tools/layout_ab.py 2>/dev/null >> gpurun_out/${OUT:-r02_layout_4k}.log; }
k16() { local lo=$1 hi=$2 s=rec; for ((k=lo; k<=hi; k++)); do s="$s,${3:-4096}:$((k*16384))"; done; echo $s; }
[ -z "$DENSE" ] && for c in reconst_one encode; do
run 12,3 $c $(k16 4 10)
run 10,4 $c $(k16 4 10)
run 16,4 $c $(k16 5 12)
done
[ -z "$DENSE" ] && for c in reconst_one encode; do
run 12,3 $c rec,16384:262144,16384:327680,16384:393216,16384:524288 16384
run 12,3 $c rec,65536:1048576,65536:1310720,65536:1572864 65536
done
if [ -n "$DENSE" ]; then
  k8() { local lo=$1 hi=$2 s=rec; for ((k=lo; k<=hi; k++)); do s="$s,4096:$((k*8192))"; done; echo $s; }
  for c in reconst_one encode; do
    OUT=r02_layout_dense run 6,3 $c $(k8 5 32)
    OUT=r02_layout_dense run 10,4 $c $(k8 7 32)
    OUT=r02_layout_dense run 12,3 $c rec,1048576:16777216,1048576:20971520,1048576:25165824 1048576
    OUT=r02_layout_dense run 16,4 $c rec,1048576:25165824,1048576:33554432 1048576
  done
fi
if [ -n "$VERIFY" ]; then
  for c in reconst_one encode; do
    OUT=r02_layout_verify run 10,4 $c rec,1048576:16777216 1048576
    OUT=r02_layout_verify run 12,3 $c rec,8192:131072 8192
    OUT=r02_layout_verify run 12,4 $c rec,4000:65536 4000
    OUT=r02_layout_verify run 13,2 $c rec,4096:65536
    OUT=r02_layout_verify run 12,3 $c rec,4198656:67108864 4194304
    OUT=r02_layout_verify run 10,4 $c rec,65536:1048576 65536
  done
fi
if [ -n "$ODD" ]; then
  for c in reconst_one encode; do
    OUT=r02_layout_odd run 12,3 $c 4100:61500,4100:65536 4100
    OUT=r02_layout_odd run 10,4 $c 4100:57400,4100:65536 4100
    OUT=r02_layout_odd run 12,3 $c 1026:15390,1026:16384 1026
    OUT=r02_layout_odd run 12,3 $c 12304:184560,12304:196608 12304
  done
fi
if [ -n "$SM" ]; then
  for c in reconst_one encode; do
    OUT=r02_layout_sm run 12,4 $c rec,sm,sm:4352 4096
    OUT=r02_layout_sm run 12,4 $c rec,sm,sm:4352 4100
    OUT=r02_layout_sm run 12,4 $c rec,sm,sm:4352 1048578
    OUT=r02_layout_sm run 12,4 $c rec,sm,sm:4352 1048576
    OUT=r02_layout_sm run 12,3 $c rec,sm,sm:4352 4096
    OUT=r02_layout_sm run 16,4 $c rec,sm,sm:4352 4096
  done
fi
if [ -n "$STAGED" ]; then
  for c in reconst_2 reconst_4; do
    OUT=r02_layout_staged run 12,4 $c rec,1052672:16842752,1048832:16781312,1114112:17825792,1048576:20971520,1048576:33554432 1048576
    OUT=r02_layout_staged run 12,4 $c rec,4352:69632,4096:98304,4096:131072 4096
    OUT=r02_layout_staged run 12,4 $c rec,sm 1048576
    OUT=r02_layout_staged run 12,4 $c rec,65792:1052672 65536
  done
fi
if [ -n "$DELTA" ]; then
  for c in reconst_one encode; do
    OUT=r02_layout_delta run 12,4 $c rec,4096:65552,4096:65600,4096:65792,4096:66560,4096:69632,4096:73728,4096:98304,4096:131072 4096
    OUT=r02_layout_delta run 12,4 $c 4100:65600,4100:65792,4100:66560,4100:69632,4100:81920,4100:98304,4100:131072 4100
  done
fi
if [ -n "$ALIGN" ]; then
  for c in reconst_one encode; do
    OUT=r02_layout_align run 12,4 $c 4096:65536,4096:65536@16,4096:65536@64,4096:65536@128,4096:65536@256,4096:65536@1024,4096:65536@2048 4096
    OUT=r02_layout_align run 12,4 $c 4100:65600,8192:131072,8192:131072@2046,4100:65600@2046 4100
    OUT=r02_layout_align run 12,4 $c 1048576:16777216,1048576:16777216@16,1048576:16777216@256,1048576:16777216@2048 1048576
  done
fi
