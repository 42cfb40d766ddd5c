#!/bin/bash
# Config-5 whole step (act + env step/store + update) of the current tree vs an older tree, one
# process per arm, alternated N times (order reversed every other round): act, update and the step.
# usage: N=8 bash tools/gpurun/dqn_step_ab.sh OUT OLD_DIR
set -o pipefail
O=gpurun_out/$1; OLD=$2; mkdir -p $O
T="import torch, bench; r = bench.dqn_config5(torch.device('cuda', 0), 0x20485EED, 1 << 21); print('act %.3f ms update %.3f ms env %.3f ms step %.3f ms' % (r['act_ms'], r['update_ms'], r['env_step_store_ms'], r['act_ms'] + r['update_ms'] + r['env_step_store_ms']), flush=True)"
N=${N:-8} bash tools/gpurun/tree_ab.sh $1 $OLD "python -u -c \"$T\"" > /dev/null || exit 1
python3 - $O/timing.txt <<'PY'
import sys, re, statistics as S
rows = [l.split() for l in open(sys.argv[1]) if l.startswith(("old", "new"))]
for arm in ("old", "new"):
    v = [(float(r[2]), float(r[5]), float(r[11])) for r in rows if r[0] == arm]
    print(arm, "n %d  act %.3f  update %.3f  step %.3f ms (means; step min %.3f max %.3f)" % (
        len(v), S.mean(x[0] for x in v), S.mean(x[1] for x in v), S.mean(x[2] for x in v),
        min(x[2] for x in v), max(x[2] for x in v)))
PY
