#!/bin/bash
# A/B of the non-temporal k_step variant at 2^26 boards (R48_STEP_NT), processes alternated, after the
# single-step parity tests with the option on.
set -o pipefail
O=gpurun_out/${1:-r04_nt}; mkdir -p $O
R48_STEP_NT=1 timeout -k 10 300 python -u -m pytest tests/test_env_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "philox or step_n_equals or past_the" > $O/pytest_nt.log 2>&1; rc=$?; tail -2 $O/pytest_nt.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1 0 1; do R48_STEP_NT=$v timeout -k 10 120 python tools/exp_kstep_ab.py 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || exit 1; done
cat $O/ab.txt
