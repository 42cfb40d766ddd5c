set -o pipefail
bash tools/gpurun/pmc_train.sh gpurun_out/pmc_train_r06 > /dev/null 2>&1; r1=$?; echo train rc=$r1
[ $r1 -eq 0 ] && bash tools/gpurun/pmc_rollout.sh gpurun_out/pmc_rollout_r06 > /dev/null 2>&1; r2=$?; echo rollout rc=$r2
[ $r1 -eq 0 ] && [ $r2 -eq 0 ] && bash tools/gpurun/prof_env.sh r06
