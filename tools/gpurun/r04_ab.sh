#!/bin/bash
# Round-4 env A/Bs: k_step_n fairness variants, non-temporal k_step, device kernargs.
set -o pipefail
TEST_VAL=2 bash tools/gpurun/stepn_env_ab.sh R48_STEPN_FAIR r04_fair2 0 4 2 3 0 4 2 3 || exit 1
bash tools/gpurun/kstep_nt_ab.sh r04_nt || exit 1
bash tools/gpurun/stepn_env_ab.sh HIP_FORCE_DEV_KERNARG r04_kernarg 0 1 0 1
