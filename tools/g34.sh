set -o pipefail
O=gpurun_out/g34; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o dqn -- python3 tools/prof_dqn.py > $O/prof_dqn.txt 2>&1
echo rc=$?
find $O/prof -name "*kernel_stats.csv" | head -3
