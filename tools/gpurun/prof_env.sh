# Profiles of the shipped env path (tools/make_profiles.py turns them into profiles/<round>/):
# kernel trace + stats of the driver's bench command, then PMC passes (one counter group per
# run, --pmc only) for k_step_n (K = 20, 2^20 boards, the bench's dispatch) and for k_step
# (single-step HBM kernel) at 2^20 and 2^26 boards.  usage: bash tools/gpurun/prof_env.sh r03
set -o pipefail
export TMPDIR=/tmp
R=${1:-r03}
O=gpurun_out/prof_$R; mkdir -p $O
KS="python3 tools/prof_stepn.py 20 300"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/kt_bench.json 2> $O/kt.log \
&& timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LEVEL_WAVES SQ_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/sqa -o pmc -- $KS > $O/sqa.log 2>&1 \
&& timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $O/sqb -o pmc -- $KS > $O/sqb.log 2>&1 \
&& timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/stepn_fetch -o pmc -- $KS > $O/f1.log 2>&1 \
&& timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/stepn_write -o pmc -- $KS > $O/w1.log 2>&1 \
&& timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/k20_fetch -o pmc -- python3 tools/prof_kstep.py 1048576 400 > $O/f2.log 2>&1 \
&& timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/k20_write -o pmc -- python3 tools/prof_kstep.py 1048576 400 > $O/w2.log 2>&1 \
&& timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/k26_fetch -o pmc -- python3 tools/prof_kstep.py 67108864 30 > $O/f3.log 2>&1 \
&& timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/k26_write -o pmc -- python3 tools/prof_kstep.py 67108864 30 > $O/w3.log 2>&1
echo rc=$?
