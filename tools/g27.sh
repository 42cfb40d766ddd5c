set -o pipefail
O=gpurun_out/g27; mkdir -p $O
for v in base al64 al128 al256 q125 base2 al64b; do
  b=${v%b}; b=${b%2}; L=build/lib_$b.so; [ $b = base ] && L=rein48_amd/lib/librein48.so
  R48_LIB=$L timeout -k 10 200 python tools/exp_stepn.py $v > $O/exp_$v.txt 2>&1 || exit 1
done
echo rc=$?
