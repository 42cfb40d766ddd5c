set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/g1
cd $GRAFT_REPO_ROOT
timeout -k 10 60 rocprofv3 -L > gpurun_out/g1/counters.txt 2>&1 || true
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/g1/sq -o pmc -- python3 tools/prof_stepn.py 20 200 > gpurun_out/g1/sq.log 2>&1 \
&& timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/g1/kt -o kt -- python3 tools/prof_stepn.py 20 200 > gpurun_out/g1/kt.log 2>&1 \
&& timeout -k 10 200 python3 tools/exp_stepn.py base > gpurun_out/g1/exp.txt 2>&1
echo rc=$?
