set -o pipefail
O=gpurun_out/r05e; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "configs or refine_batch or c2" > $O/parity.log 2>&1 && \
PMVS_AMD_LIB=cmvs-pmvs_amd/libpmvs_amd_prof.so timeout -k 10 400 python3 -u tools/refine_sizes.py 225016,226014,227012,228010,245016,246014,247012,248010 10000,80000 > $O/sizes_prof.jsonl 2> $O/sizes_prof.err && \
timeout -k 10 400 python3 -u tools/refine_sizes.py 1206,132042,225016,226014,227012,228010,246014,248010 2000,5000,10000,40000,80000,120000 > $O/sizes.jsonl 2> $O/sizes.err
echo "rc=$?"
