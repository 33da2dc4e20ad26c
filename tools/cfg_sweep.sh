set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u bench.py --params 181668 --budget 0.5 --steps 2000 --warmup 50 --choco 0 --cpu-seconds 0 > gpurun_out/cfg2.json
timeout -k 10 200 python -u bench.py --params 181668 --budget 1.0 --steps 2000 --warmup 50 --choco 0 --cpu-seconds 0 > gpurun_out/cfg2_full.json
timeout -k 10 200 python -u bench.py --params 36546980 --budget 0.5 --steps 50 --warmup 10 --choco 0 --cpu-seconds 0 > gpurun_out/cfg3.json
timeout -k 10 200 python -u bench.py --params 36546980 --budget 1.0 --steps 50 --warmup 10 --choco 0 --cpu-seconds 0 > gpurun_out/cfg3_full.json
