set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_train; mkdir -p $O
bash tools/pmc_train.sh \
&& timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python tools/prof_train.py 16777216 5 > $O/kt.log 2>&1
echo rc=$?
