set -o pipefail
O=gpurun_out/g25; mkdir -p $O
for v in q246 q136 q357 q246b q136b q357b; do
  b=${v%b}; L=build/lib_$b.so; [ $b = q246 ] && L=rein48_amd/lib/librein48.so
  R48_LIB=$L timeout -k 10 200 python tools/exp_stepn.py $v > $O/exp_$v.txt 2>&1 || exit 1
done
echo rc=$?
