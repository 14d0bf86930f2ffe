set -o pipefail
O=gpurun_out/r05c; mkdir -p $O
PMVS_AMD_LIB=cmvs-pmvs_amd/libpmvs_amd_prof.so timeout -k 10 300 python3 -u tools/refine_sizes.py 1206,202032,204016 10000,80000 > $O/sizes_prof.jsonl 2> $O/sizes_prof.err && \
bash tools/gpu_round.sh check r05c
echo "rc=$?"
