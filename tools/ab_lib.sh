# A/B of two builds of the native library on one box: the command "$@" runs alternately with
# $AB_OLD (another build, via MX_GOSSIP_LIB) and with the current build, 3 times each; outputs in
# gpurun_out/ab_old.log / ab_new.log.  Usage on the GPU box:
#   AB_OLD=_ab/lib_head.so bash tools/ab_lib.sh python -u tools/chocobench.py
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
for i in 1 2 3; do
  MX_GOSSIP_LIB=$AB_OLD timeout -k 10 200 "$@" >> gpurun_out/ab_old.log 2>&1 || exit 1
  timeout -k 10 200 "$@" >> gpurun_out/ab_new.log 2>&1 || exit 1
done
