#!/bin/bash
# GPU job: A3C GPU tests (fused update parity), k_cnn_train timing and its PMC MFMA-busy pass, and the
# config-5 conv timings incl. the fused-epilogue variants.  usage: bash tools/gpurun/train_conv_check.sh
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/tcc; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_a3c_gpu.py > $O/pytest_a3c.txt 2>&1 && tail -2 $O/pytest_a3c.txt \
&& timeout -k 10 300 python -u tools/exp_train.py 16777216 > $O/train.txt 2>&1 && cat $O/train.txt \
&& timeout -k 10 300 python -u tools/exp_conv.py > $O/conv.txt 2>&1 && cat $O/conv.txt \
&& timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES --output-format csv -d $O/pmc -o pmc -- python3 tools/exp_train.py 16777216 > $O/pmc.log 2>&1 && echo pmc ok
