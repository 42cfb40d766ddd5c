set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_fwd; mkdir -p $O
P="python3 tools/exp_policy.py 8388608"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o pmc -- $P > $O/p1.log 2>&1 \
&& timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o pmc -- $P > $O/p2.log 2>&1 \
&& timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- $P > $O/kt.log 2>&1
echo rc=$?
