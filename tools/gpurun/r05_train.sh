#!/bin/bash
# Round-5 k_cnn_train session: the CNN update tests on the first library, kernel-only timings of every
# library at 2^24 rows (tools/exp_train.py, one process, libraries alternated), per-phase stamps of
# the stamp builds given in STAMPS, then the SQ counter passes of the first library.
# usage: STAMPS="a.so b.so" bash tools/gpurun/r05_train.sh OUTDIR lib.so [lib.so ...]
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; shift; mkdir -p $O
R48_LIB=$1 timeout -k 10 600 python -u -m pytest tests/test_a3c_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "fused_cnn or trainer_fused_update or rollout" > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do timeout -k 10 300 python -u tools/exp_train.py 16777216 "$@" 2>&1 | grep -v amdgpu.ids >> $O/timing.txt || exit 1; done
cat $O/timing.txt
for S in $STAMPS; do echo "== $S" >> $O/stamps.txt; timeout -k 10 300 python -u tools/exp_train_stamps.py $S 2>&1 | grep -v amdgpu.ids >> $O/stamps.txt || exit 1; done
cat $O/stamps.txt
R48_LIB=$1 bash tools/gpurun/pmc_train.sh $O/pmc
