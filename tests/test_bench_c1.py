"""CPU: BASELINE config 1 as a timed line (bench.py --config c1_java_cpu_64x64).

Config 1 is the reference's own CPU-runnable case, the Java Encoder path on one 64x64 8-frame stack
(Encoder.java:47-89).  The line must carry the driver contract's fields with n_gpus 0, and the step's
output must be the committed golden fixture (tests/golden/c1_64x64x8.npz), so the number is the time of
the right computation.
"""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_c1_line_parses_and_matches_golden():
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--config", "c1_java_cpu_64x64",
                        "--steps", "3", "--warmup", "1"], capture_output=True, text=True, timeout=300, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "dtype", "data", "config", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 0 and d["steps"] == 3 and d["unit"] == "cubes/s" and d["value"] > 0
    assert d["config"]["cubes_per_step"] == 64
    cb = d["cpu_baseline"]
    assert cb["kind"] == "port" and cb["cores"] >= 1 and "availableProcessors()" in cb["pool_rule"]
    gold = np.load(os.path.join(REPO, "tests", "golden", "c1_64x64x8.npz"))["q"]
    assert d["output_sha256"] == hashlib.sha256(np.ascontiguousarray(gold, dtype=np.int32).tobytes()).hexdigest()
