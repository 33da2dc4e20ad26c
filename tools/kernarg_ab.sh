set -u
mkdir -p gpurun_out/r6l
B="python -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 --staged 0 --configs 0 --choco 0 --allreduce 0 --er 0"
export TMPDIR=/tmp
for rep in 1 2; do
  timeout -k 10 120 $B > gpurun_out/r6l/plain_$rep.json 2>/dev/null || exit 1
  HIP_FORCE_DEV_KERNARG=1 timeout -k 10 120 $B > gpurun_out/r6l/devkarg_$rep.json 2>/dev/null || exit 1
  HIP_FORCE_DEV_KERNARG=0 timeout -k 10 120 $B > gpurun_out/r6l/hostkarg_$rep.json 2>/dev/null || exit 1
  timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6l/trace_$rep -o trace -- $B > gpurun_out/r6l/rocprof_$rep.log 2>&1 || exit 1
done
