#!/bin/bash
# PMC passes for k_step (separate passes, --pmc only, no trace domains) at 2^20 and 2^26 boards.
set -o pipefail
OUT=gpurun_out/pmc
mkdir -p $OUT
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --no-extras"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/n20/fetch -o pmc -- $B --steps 200 --warmup 20 > $OUT/n20_fetch.log 2>&1 \
&& timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/n20/write -o pmc -- $B --steps 200 --warmup 20 > $OUT/n20_write.log 2>&1 \
&& timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/n26/fetch -o pmc -- $B --boards 67108864 --steps 20 --warmup 4 > $OUT/n26_fetch.log 2>&1 \
&& timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/n26/write -o pmc -- $B --boards 67108864 --steps 20 --warmup 4 > $OUT/n26_write.log 2>&1 \
&& python tools/pmc_traffic.py $OUT/n20 1048576 $OUT/pmc_n20.json && python tools/pmc_traffic.py $OUT/n26 67108864 $OUT/pmc_n26.json \
&& echo "== bench" && timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && cat gpurun_out/bench.json
