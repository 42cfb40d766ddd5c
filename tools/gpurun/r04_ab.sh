#!/bin/bash
# Round-4 env A/Bs: non-temporal k_step at 2^26 boards, device-memory kernel arguments at K = 20.
set -o pipefail
bash tools/gpurun/kstep_nt_ab.sh r04_nt || exit 1
bash tools/gpurun/stepn_env_ab.sh HIP_FORCE_DEV_KERNARG r04_kernarg 0 1 0 1
