#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration of the config-5 conv's access patterns: build/probe_conv_io in
# calibration mode (chain 0) under two separate --pmc passes, then its timing sweep.
# usage: bash tools/gpurun/probe_conv_pmc.sh OUT
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o pmc -- build/probe_conv_io cal > $O/fetch.log 2>&1 \
&& timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o pmc -- build/probe_conv_io cal > $O/write.log 2>&1 \
&& timeout -k 10 240 build/probe_conv_io > $O/timing.txt 2>&1 && cat $O/timing.txt
