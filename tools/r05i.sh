set -o pipefail
O=gpurun_out/r05i; mkdir -p $O
S=1000,2000,3000,5000,10000,80000
timeout -k 10 400 python3 -u tools/refine_sizes.py 132042,226014,228010,248010,288010 $S > $O/sizes.jsonl 2> $O/sizes.err && \
PMVS_AMD_LIB=cmvs-pmvs_amd/libpmvs_amd_w1.so timeout -k 10 300 python3 -u tools/refine_sizes.py 224020,244020,284020,222040 $S > $O/sizes_w1.jsonl 2> $O/sizes_w1.err && \
PMVS_AMD_LIB=cmvs-pmvs_amd/libpmvs_amd_w1r.so timeout -k 10 300 python3 -u tools/refine_sizes.py 244020,284020 $S > $O/sizes_w1r.jsonl 2> $O/sizes_w1r.err
echo "rc=$?"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_c3_full.py -m gpu -x -v --timeout 600 --timeout-method thread -k step_and_first > gpurun_out/r05i/c3test.log 2>&1 && \
timeout -k 10 500 python3 -u bench.py > gpurun_out/r05i/bench.json 2> gpurun_out/r05i/bench.err
echo "rc2=$?"
