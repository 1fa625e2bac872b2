"""The bench.py driver contract: one JSON line on rank 0 with the required keys,
for one process and for a 2-rank torch.distributed.run launch (gloo on one
GPU: the rehearsal of the RCCL path the driver runs on 2/4/8 GPUs)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}
SMALL = ["--steps", "2", "--warmup", "1", "--batch", "1", "--height", "128", "--width", "256", "--iters", "3"]


def _json_lines(out: str):
    return [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]


def _env():
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


@pytest.mark.gpu
def test_bench_single_process_json():
    r = subprocess.run([sys.executable, "bench.py"] + SMALL, cwd=ROOT, env=_env(), capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1, r.stdout
    rec = recs[0]
    assert KEYS <= set(rec), set(KEYS) - set(rec)
    assert rec["n_gpus"] == 1 and rec["steps"] == 2 and rec["value"] > 0
    assert rec["config"]["global_batch"] == 1 and rec["config"]["model"] == "raft_large"


@pytest.mark.gpu
def test_bench_two_ranks_gloo_one_json_line():
    port = 29500 + os.getpid() % 1000
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2", "--dist-backend", "gloo"] + SMALL
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=115)
    assert r.returncode == 0, r.stderr[-2000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1, r.stdout  # rank 0 only
    rec = recs[0]
    assert rec["n_gpus"] == 2 and rec["config"]["global_batch"] == 2 and rec["config"]["parallelism"] == "dp2"
    # the communication of the DP path: world check, per-rank step times, the final-flow gather
    assert rec["rccl_world"] == 2 and len(rec["per_rank_ms_per_step"]) == 2
    assert rec["gather_ms"] is not None and rec["gather_ms"] > 0 and rec["config"]["result_gather"]


@pytest.mark.gpu
def test_bench_extras_keys():
    """--extras on: the secondary configs land in the same JSON line (each a
    record or null), here at a small size so the test stays short."""
    r = subprocess.run([sys.executable, "bench.py", "--extras", "on", "--extra-steps", "2", "--train-batch", "1",
                        "--train-size", "128", "256"] + SMALL, cwd=ROOT,
                       env=_env(), capture_output=True, text=True, timeout=115)
    assert r.returncode == 0, r.stderr[-2000:]
    rec = _json_lines(r.stdout)[0]
    ex = rec["extras"]
    assert set(ex) >= {"b1_fps", "small_b1_fps_32it", "small_b1_fps_12it", "fp32_b1_fps", "train_pairs_per_s",
                       "extras_wall_s"}
    assert ex["fp32_b1_fps"]["config"]["dtype"] == "fp32"
    for k in ("b1_fps", "small_b1_fps_32it", "small_b1_fps_12it", "fp32_b1_fps", "train_pairs_per_s"):
        assert ex[k] is not None and ex[k]["value"] > 0, (k, r.stderr[-1500:])
    # single GPU: the training extra runs in a fresh child process (bench.py:run_training_child)
    assert ex["train_pairs_per_s"]["process"].startswith("fresh child"), ex["train_pairs_per_s"]
    assert ex["train_pairs_per_s"]["config"]["image_size"] == [128, 256]
