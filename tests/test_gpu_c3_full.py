"""The headline configuration at full size (BASELINE.json configs[2], C3: 50 views 3840x2160,
level 0): one bench.py loop step on the device, its model checked by the bench's size-independent
invariants, and the first expansion waves of loop iteration 1 compared record for record with the
CPU oracle on the same scene and seeds (bench.py loop_samples -> parity_c3_first_waves; bench.py
exits 3 on a mismatch)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(900)
def test_c3_full_size_first_waves_match_oracle(gpu_available):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "0", "--no-c2",
           "--cpu-iterations", "1", "--cpu-waves", "2", "--cpu-seconds", "1"]
    pr = subprocess.run(cmd, capture_output=True, text=True, timeout=800)
    assert pr.returncode == 0, pr.stderr[-3000:]
    line = json.loads(pr.stdout.strip().splitlines()[-1])
    assert line["config"]["width"] == 3840 and line["config"]["height"] == 2160 and line["config"]["views"] == 50
    assert line["parity_c3_first_waves"] is True, line.get("parity_c3_detail")
    detail = line["parity_c3_detail"][0]
    assert detail["mismatched_records"] == 0 and detail["stats_equal"] and detail["added"] > 10000, detail
    assert line["checks"]["ok"], line["checks"]
    assert line["value"] > 0
