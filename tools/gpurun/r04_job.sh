set -o pipefail
O=gpurun_out/r04a; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_checkpoint_gpu.py tests/test_env_gpu.py tests/test_dqn_gpu.py tests/test_a3c_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "resume or without_auto_reset or bench_size or fused_cnn_update_gradients or train_step_matches_autograd or step_n" > $O/pytest.log 2>&1; rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
R48_STEPN_LANE_BOARDS=1 timeout -k 10 300 python -u -m pytest tests/test_env_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "step_n or fingerprint or philox" > $O/pytest_lane1.log 2>&1; rc=$?; tail -3 $O/pytest_lane1.log; [ $rc -eq 0 ] || exit $rc
for v in 2 1 2 1; do R48_STEPN_LANE_BOARDS=$v timeout -k 10 120 python tools/exp_stepn_ab.py >> $O/ab_lane.txt 2>&1 || exit 1; echo "lane=$v" >> $O/ab_lane.txt; done
cat $O/ab_lane.txt
