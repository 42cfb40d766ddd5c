#!/bin/bash
# k_conv_wgrad timing probes (round 6): the product vs builds with the MFMAs compiled out, the DMAs
# compiled out (stale LDS: timing only) and a 4-buffer ring at 32 input channels, one process per
# library, twice; then SQ counters of the product's wgrad dispatches (two --pmc passes).
# usage: bash tools/gpurun/wgrad_probe.sh OUT
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
P=rein48_amd/lib/librein48.so
for i in 1 2; do
  for l in $P varlib/wg_nomfma.so varlib/wg_nodma.so varlib/wg_ring4.so; do
    CASES=wgrad64,wgrad32 timeout -k 10 300 python -u tools/exp_conv.py 65536 $l 2>&1 | grep -v amdgpu.ids >> $O/probe.txt || exit 1
  done
done
cat $O/probe.txt
export CASES=wgrad64,wgrad32
X="python3 tools/exp_conv.py 65536"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC --output-format csv -d $O/p1 -o pmc -- $X > $O/p1.log 2>&1 \
&& timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o pmc -- $X > $O/p2.log 2>&1 \
&& for k in k_conv_wgradILi64 k_conv_wgradILi32; do python3 tools/pmc_summary.py $k 131072 $O/p1 $O/p2 > $O/$k.json; done && cat $O/k_conv_wgradILi64.json
