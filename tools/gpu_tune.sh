set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/mixtune.py > gpurun_out/mixtune.log 2>&1 &&
timeout -k 10 300 python -u tools/chocobench.py > gpurun_out/choco.log 2>&1 &&
timeout -k 10 -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/chocoprof -o choco -- python -u tools/chocobench.py > gpurun_out/chocoprof.log 2>&1
