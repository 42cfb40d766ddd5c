#!/bin/bash
# GPU job: FETCH_SIZE and WRITE_SIZE passes (separate runs, --pmc only) over two config-5 updates
# (tools/prof_dqn.py 2), summarised by tools/dqn_traffic.py.  usage: bash tools/gpurun/dqn_traffic.sh
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/dqn_traffic}; mkdir -p $O
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o pmc -- python3 tools/prof_dqn.py 2 > $O/fetch.log 2>&1 \
&& timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o pmc -- python3 tools/prof_dqn.py 2 > $O/write.log 2>&1 \
&& python3 tools/dqn_traffic.py $O 3 | tee $O/traffic.txt
