#!/bin/bash
# MATCHA communication-budget sweep of the headline shape (graph 0, 8 workers x 25.6M, one GPU):
# one bench.py line per budget (schedule from solver.py's probabilities, numpy seed 1234).
set -u
mkdir -p gpurun_out
for b in 0.1 0.2 0.3 0.4 0.5 0.6 0.7 0.8 0.9 1.0; do
  timeout -k 10 120 python -u bench.py --budget $b --steps 100 --warmup 10 --choco 0 --cpu-seconds 0 \
      > gpurun_out/budget_$b.json 2> gpurun_out/budget_$b.err || exit $?
done
