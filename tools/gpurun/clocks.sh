#!/bin/bash
# Per-kernel average clocks of the CNN / MLP / ResNet kernels: one rocprofv3
# --pmc GRBM_GUI_ACTIVE pass over tools/prof_clocks.py.  usage: bash tools/gpurun/clocks.sh OUTDIR
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE --output-format csv -d $O/pmc -o clk -- python3 tools/prof_clocks.py > $O/prof_clocks.log 2>&1 \
&& python3 tools/kernel_clocks.py $O/pmc > $O/kernel_clocks.json && cat $O/prof_clocks.log | grep -v amdgpu.ids && cat $O/kernel_clocks.json
