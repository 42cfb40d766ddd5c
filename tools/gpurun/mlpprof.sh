#!/bin/bash
# kernel trace of the reference-MLP A3C train step (both loss modes)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_mlpprof}; mkdir -p $O
for m in textbook reference; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$m -o kt -- python3 tools/prof_mlp.py $m 2 > $O/$m.log 2>&1 || exit 1
f=$(find $O/$m -name "kt_kernel_stats.csv" | head -1); echo "== $m"; python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
rows.sort(key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:10]: print('%-60s %6s calls %10.3f ms avg %8.3f ms' % (r['Name'][:60], r['Calls'], float(r['TotalDurationNs'])/1e6, float(r['AverageNs'])/1e6))"
done
