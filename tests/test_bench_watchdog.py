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


# ---- --gpus N: never a 1-GPU number for an N-GPU request ----------------------

def _env_without_launcher(**extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    env.update(extra)
    return env


def test_world_size_mismatch_is_an_error_line():
    env = _env_without_launcher(RANK="0", WORLD_SIZE="3", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], capture_output=True,
                       text=True, timeout=120, env=env)
    assert p.returncode != 0
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["value"] is None and "WORLD_SIZE=3" in d["error"] and d["n_gpus"] == 2


def test_plain_gpus_n_launches_n_ranks():
    """Without WORLD_SIZE, `bench.py --gpus 2` starts two ranks under torch.distributed.run as a child
    and relays rank 0's line.  Here (no GPU) the ranks find no device and say so: the relayed line is
    an error line for n_gpus 2 and the status is non-zero -- never a line with n_gpus 1."""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0"],
                       capture_output=True, text=True, timeout=240, env=_env_without_launcher())
    assert p.returncode != 0, p.stdout
    lines = [json.loads(l) for l in p.stdout.splitlines() if l.lstrip().startswith("{")]
    assert len(lines) == 1, (p.stdout, p.stderr[-3000:])
    d = lines[0]
    assert d["n_gpus"] == 2 and d["value"] is None and "GPU" in d["error"], d
    assert "starting 2 ranks" in p.stderr


def test_gather_roofline_block():
    """roofline.gather: cold gathers / the measured L2-resident gather rate and
    LDS-served entries / the measured LDS rate, against the pass time (profiles/rates.json)."""
    sys.path.insert(0, ROOT)
    import bench

    rates = bench.gather_rates()
    assert rates is not None and rates["l2_gather_per_s"] > 1e11 and rates["lds_read_per_s"] > 1e12
    g = bench.gather_roofline({"local_edges": 1_000_000_000, "hot_cover_ppm": 750_000}, 2.0)
    assert g["cold_gathers"] == 250_000_000 and g["lds_entries"] == 750_000_000
    assert abs(g["cold_floor_ms"] - 250e6 / rates["l2_gather_per_s"] * 1e3) < 1e-3
    assert abs(g["frac_cold"] - g["cold_floor_ms"] / 2.0) < 1e-3
    assert bench.gather_roofline({"local_edges": 10, "hot_cover_ppm": 0}, 0.0) is None
