#!/bin/bash
# A/B of a k_step_n launch option selected by an environment variable (read once per process):
# the step_n parity tests with the option on, then tools/exp_stepn_ab.py in alternating processes.
# usage: bash tools/gpurun/stepn_env_ab.sh VAR OUTDIR [values...]   (default values: 0 1 0 1)
set -o pipefail
VAR=$1; O=gpurun_out/$2; shift 2
VALS=${@:-0 1 0 1}
mkdir -p $O
env $VAR=${TEST_VAL:-1} timeout -k 10 300 python -u -m pytest tests/test_env_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "step_n or fingerprint or philox" > $O/pytest_$VAR.log 2>&1; rc=$?; tail -2 $O/pytest_$VAR.log; [ $rc -eq 0 ] || exit $rc
for v in $VALS; do echo "== $VAR=$v" >> $O/ab.txt; env $VAR=$v timeout -k 10 120 python tools/exp_stepn_ab.py 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || exit 1; done
cat $O/ab.txt
