#!/bin/bash
# Per-kernel clocks (GRBM_GUI_ACTIVE pass) of the config-5 step loop, current tree and an older tree,
# alternated twice. usage: bash tools/gpurun/dqn_step_clocks.sh OUT OLD_DIR
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/$1; OLD=$2; mkdir -p $O
for i in 1 2; do for arm in new old; do
  D=.; [ $arm = old ] && D=$OLD
  (cd $D && timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE --output-format csv -d $O/${arm}_$i -o clk -- python3 tools/prof_dqn_step.py > $O/${arm}_$i.log 2>&1) || exit 1
  python3 tools/kernel_clocks.py $O/${arm}_$i 200 > $O/${arm}_$i.json || exit 1
  python3 -c "
import json; k = json.load(open('$O/${arm}_$i.json'))['kernels']
print('$arm $i', open('$O/${arm}_$i.log').read().strip().splitlines()[-1], ' | ', '; '.join('%s %.2f GHz %.3f ms' % (n[:28], v['clock_ghz'], v['mean_dispatch_ms']) for n, v in list(k.items())[:6]))"
done; done
