set -o pipefail
O=gpurun_out/g42; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_a3c_gpu.py > $O/pytest_a3c.txt 2>&1
echo rc=$?
