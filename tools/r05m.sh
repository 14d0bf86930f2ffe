set -o pipefail
O=gpurun_out/r05m; mkdir -p $O
for v in prod abA abB abC abE; do
  L=cmvs-pmvs_amd/libpmvs_amd_$v.so; [ $v = prod ] && L=cmvs-pmvs_amd/libpmvs_amd.so
  PMVS_AMD_LIB=$L timeout -k 10 200 python3 -u tools/refine_sizes.py 226014,228010,246014 10000,80000 > $O/sizes_$v.jsonl 2> $O/sizes_$v.err || exit 1
done
echo "rc=$?"
