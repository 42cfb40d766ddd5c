#!/bin/bash
# GPU job: kernel trace + stats of A3C config-3 train steps in both loss modes (tools/prof_a3c.py).
# usage: bash tools/gpurun/a3c_prof.sh
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/a3c_prof; mkdir -p $O
for m in textbook reference; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$m -o a3c -- python3 tools/prof_a3c.py 2 $m > $O/$m.log 2>&1 || exit 1
done
echo done
