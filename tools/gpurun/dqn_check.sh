set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_dqn_gpu.py -k "train_step or pack or conv" > gpurun_out/ts.txt 2>&1; rc=$?; tail -3 gpurun_out/ts.txt; [ $rc -eq 0 ] && bash tools/gpurun/dqn_prof.sh
