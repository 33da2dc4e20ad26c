#!/bin/bash
# profile_round.sh with the headline launches only (r02b: the WRN figure's launches had skewed it).
set -u
export TMPDIR=/tmp
bash tools/profile_round.sh r02c > gpurun_out/profile_r02c.log 2>&1; rc=$?; tail -3 gpurun_out/profile_r02c.log; exit $rc
