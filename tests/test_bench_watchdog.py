"""bench.py never leaves the driver without a JSON line: a stage that overruns its deadline (a
hang in RCCL on a first multi-GPU run, for instance) makes rank 0 print the contract's line with
"value": null and an "error" naming the stage, and the process exit non-zero.
The stall is simulated before any GPU work, so this runs on CPU."""
import json
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("stage", ["attach", "timed"])
def test_stalled_stage_prints_error_line_within_deadline(stage):
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--simulate-stall", stage,
                        "--stage-timeout", "2"], capture_output=True, text=True, timeout=120, env=env)
    dt = time.monotonic() - t0
    assert p.returncode == 3, p.stderr
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["value"] is None and stage in d["error"] and "deadline" in d["error"]
    assert d["metric"].startswith("PageRank GTEPS") and d["unit"] == "GTEPS"
    assert dt < 60, dt


def test_non_zero_rank_prints_no_line():
    env = dict(os.environ, RANK="1", WORLD_SIZE="2", LOCAL_RANK="1")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--simulate-stall", "attach",
                        "--stage-timeout", "1"], capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode == 3
    assert p.stdout.strip() == ""
    assert "attach" in p.stderr
