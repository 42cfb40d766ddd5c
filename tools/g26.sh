set -o pipefail
O=gpurun_out/g26; mkdir -p $O
for v in q136 q125 q135 q146 q137 q236 q136b; do
  b=${v%b}; L=build/lib_$b.so; [ $b = q136 ] && L=rein48_amd/lib/librein48.so
  R48_LIB=$L timeout -k 10 200 python tools/exp_stepn.py $v > $O/exp_$v.txt 2>&1 || exit 1
done
echo rc=$?
