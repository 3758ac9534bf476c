set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r02z2_pc_rows.txt
: > $out
for shape in "--K 4096 --N 16384" "--K 1024 --N 4096" "--K 4096 --N 4096"; do
  echo "# TSG_ELL_VARIANT=0 $shape" >> $out
  TSG_ELL_VARIANT=0 timeout -k 10 200 python scripts/small_m_sweep.py $shape --M 1,2,3,4 >> $out 2>&1 || exit 1
done
