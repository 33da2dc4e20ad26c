#!/bin/bash
set -u
mkdir -p gpurun_out/r2s13; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/choco_long.py > gpurun_out/r2s13/long.log 2>&1; echo rc=$?; cat gpurun_out/r2s13/long.log | grep drift
