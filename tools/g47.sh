set -o pipefail
O=gpurun_out/g47; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_a3c_gpu.py -k "tiling or policy" > $O/pytest.txt 2>&1
echo rc=$?
