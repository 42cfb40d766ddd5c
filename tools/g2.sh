# GPU check: instruction rates, env parity tests, step_n sweep, driver-shaped bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/g2; mkdir -p $O
timeout -k 10 120 build/instr_rate > $O/instr_rate.txt 2>&1 \
&& timeout -k 10 400 python -u -m pytest tests/test_env_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest_env.txt 2>&1 \
&& timeout -k 10 200 python tools/exp_stepn.py orient > $O/exp.txt 2>&1 \
&& timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
echo rc=$?
