# A/B of two builds of the native library on one box: Choco GPU tests on the current build, then
# tools/chocobench.py alternating between $AB_OLD (another build, via MX_GOSSIP_LIB) and the
# current one.  Usage on the GPU box: AB_OLD=<path to .so> bash tools/ab_choco.sh
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gossip.py -m gpu -x -q --timeout 120 --timeout-method thread -k "choco or topk" > gpurun_out/ab_tests.log 2>&1 || exit 1
for i in 1 2 3; do
  MX_GOSSIP_LIB=$AB_OLD timeout -k 10 120 python -u tools/chocobench.py >> gpurun_out/ab_old.log 2>&1 || exit 1
  timeout -k 10 120 python -u tools/chocobench.py >> gpurun_out/ab_new.log 2>&1 || exit 1
done
