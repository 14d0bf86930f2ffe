#!/bin/bash
# the 1920x1080 C5-shaped exchange test under three refine layouts for the small batches
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06r; mkdir -p $O
cd $R
T="tests/test_gpu_c5_exchange.py::test_c5_shaped_two_clusters_exchange_small"
for V in default 132042 226014; do
  if [ $V = default ]; then E=""; else E="PMVS_REFINE_SMALL_CONFIG=$V"; fi
  env $E timeout -k 10 200 python3 -u -m pytest "$T" -m gpu -x -v -s --timeout 180 --timeout-method thread > $O/pytest_$V.log 2>&1; rc=$?
  echo "== $V rc=$rc"; grep -E "C5 cluster" $O/pytest_$V.log | sed -E "s/checks \{.*sphere_residual_p99': ([0-9.e-]+).*/p99 \1/" | cut -c1-300
  [ $rc -le 1 ] || exit $rc
done
