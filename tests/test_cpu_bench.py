"""CPU tests of bench.py's contract plumbing: `python bench.py --gpus N` starts N ranks itself (the driver's
scaling runs call it that way) and the process group it builds has exactly N ranks; the algorithmic work per
utterance reproduces SURVEY §8(d)'s flop-counter figures for the configs BASELINE.json names."""
import json
import os
import subprocess
import sys

from conftest import ROOT


def test_bench_gpus_flag_spawns_that_many_ranks():
    env = dict(os.environ, FDDM_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"], env=env,
                         capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1]
    rec = json.loads(line)
    assert rec["n_gpus"] == 2 and rec["parallelism"] == "dp2" and rec["global_batch"] == 64


def test_bench_rejects_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"], env=env,
                         capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert out.returncode != 0 and "--gpus is 2" in out.stderr


def test_gflop_per_utt_matches_survey():
    sys.argv = ["bench.py"]
    import bench
    a = bench.parse()
    assert abs(bench.gflop_per_utt(a) - 193.87) < 0.05                     # C2
    a.layers, a.d_model, a.heads, a.seq_len, a.batch = 12, 768, 12, 512, 16
    assert abs(bench.gflop_per_utt(a) - 491.68) < 0.05                     # C4
    assert bench.config_tag(a).startswith("C4")
    a.layers, a.d_model, a.heads, a.seq_len, a.batch, a.seconds = 2, 128, 4, 32, 4, 1.0
    assert abs(bench.gflop_per_utt(a) - 14.32) < 0.05                      # C1
