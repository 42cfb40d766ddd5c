set -o pipefail
O=gpurun_out/g24; mkdir -p $O
for v in q246 q147 q357 q247 q136 q246b; do
  L=build/lib_$v.so; [ $v = q246 ] || [ $v = q246b ] && L=rein48_amd/lib/librein48.so
  R48_LIB=$L timeout -k 10 200 python tools/exp_stepn.py $v > $O/exp_$v.txt 2>&1 || exit 1
done
echo rc=$?
