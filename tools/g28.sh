# final check of the round's tree: GPU suite, smoke, driver bench, profiles of the shipped build
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/g28; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 \
&& timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
&& timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err \
&& bash tools/prof_r02.sh > $O/prof.txt 2>&1
echo rc=$?
