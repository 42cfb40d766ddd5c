# PMC of the shipped k_cnn_forward (grouped conv2, desync priority) at 2^23 boards: two --pmc passes
set -o pipefail
O=gpurun_out/g40; mkdir -p $O
export TMPDIR=/tmp
P="python3 tools/exp_policy.py 8388608"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o pmc -- $P > $O/p1.log 2>&1 \
&& timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --output-format csv -d $O/p2 -o pmc -- $P > $O/p2.log 2>&1 \
&& python3 tools/pmc_summary.py k_cnn_forward 131072 $O/p1 $O/p2 > $O/pmc_k_cnn_forward.json
echo rc=$?
