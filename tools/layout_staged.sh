export TMPDIR=/tmp
M=1048576
L="rec,$((M+256)):$((16*(M+256))),$((M+4096)):$((16*(M+4096))),$((M+4352)):$((16*(M+4352))),$((M+65536)):$((16*(M+65536))),$M:$((16*M+4096))"
for c in reconst_2 reconst_4 encode reconst_one; do
  CODEC=12,4 SIZE=$M CASE=$c LAYOUTS=$L ROUNDS=9 GIB=4 timeout -k 10 120 python tools/layout_ab.py || exit $?
done
L4="rec,4352:69632,4096:69632,4096:65792,4224:67584"
for c in reconst_2 reconst_4 encode reconst_one; do
  CODEC=12,4 SIZE=4096 CASE=$c LAYOUTS=$L4 ROUNDS=9 GIB=4 timeout -k 10 120 python tools/layout_ab.py || exit $?
done
