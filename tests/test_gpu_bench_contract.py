"""bench.py keeps the driver contract: one JSON line with BASELINE.json's metric, the
roofline object and the CPU baseline (short run, GPU box)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_json_line():
    out = subprocess.run([sys.executable, "bench.py", "--steps", "5", "--warmup", "2",
                          "--cpu-seconds", "1"], cwd=REPO, capture_output=True, text=True,
                         timeout=200)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    with open(os.path.join(REPO, "BASELINE.json")) as f:
        assert r["metric"] == json.load(f)["metric"]
    assert r["value"] > 0 and r["unit"] == "env_steps/s" and r["n_gpus"] == 1
    assert r["steps"] == 5 and r["warmup"] == 2 and r["higher_is_better"] is True
    assert r["scaling"] == "strong" and r["vs_baseline"] is None and r["dtype"] == "f64"
    assert r["config"]["envs_total"] == 4096
    rf = r["roofline"]
    assert rf["bound"] == "valu-latency" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    assert rf["achieved"] > 0 and abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-12
    # the kernel time comes from events bracketing the timed region: never above the wall
    # time per step, and the post-region sampled event pairs hold >= 10 launches
    assert 0 < rf["kernel_avg_ms"] <= r["ms_per_step"] * 1.001
    assert "launch, 10 samples" in rf["sampled_launch_timing"]
    cb = r["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] in ("port", "reference")
    assert cb["per_env"]["value"] > 0
    assert "workload" in r["config"]
    # the short C5 leg (BASELINE configs[4]) rides along in the default line
    c5 = r["c5"]
    assert c5["env_only"]["value"] > 0 and c5["env_policy"]["value"] > 0
    assert c5["env_policy"]["value"] <= c5["env_only"]["value"] * 1.05
    # ... and its learner-in-the-loop leg (the whole SAC iteration as one HIP graph)
    ln = c5["env_policy_learner"]
    assert 0 < ln["value"] <= c5["env_policy"]["value"] * 1.05
    assert ln["critic_loss"] == ln["critic_loss"] and ln["actor_loss"] == ln["actor_loss"]
    assert rf["scope"].startswith("per GPU") and rf["step_avg_ms"] == rf["kernel_avg_ms"]


def test_bench_two_rank_rehearsal_checks_rows():
    """The multi-rank bench path on one GPU (2 ranks over gloo, BENCH_BACKEND=gloo: the
    gather goes through the host, so the rate measures nothing): barriers, max-over-ranks
    timing, the per-step gather and, after the timed region, the cross-rank row check -- every
    rank's gathered rows against every rank's own rows, bitwise -- recorded in the line."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, BENCH_BACKEND="gloo")
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                          "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                          str(port), "bench.py", "--gpus", "2", "--steps", "5", "--warmup", "2",
                          "--gather-block", "0"], cwd=REPO, capture_output=True, text=True,
                         timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["config"]["envs_total"] == 4096
    cfg = r["config"]
    assert cfg["gather_transport"] == "torch" and cfg["rccl"] is None
    rc = cfg["row_check"]
    assert rc["ok"] is True and rc["bad_rows"] == 0 and rc["bad_rows_by_source_rank"] == [0, 0]


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_bench_descent_sac_two_rank_rehearsal():
    """BASELINE configs[4]'s multi-GPU path on one GPU (2 ranks over gloo): each rank steps
    its 2,048-env shard with the fused actor and runs FusedSAC on its shard's buffer, the
    gradients all-reduced before each Adam launch; one JSON line, finite losses."""
    env = dict(os.environ, BENCH_BACKEND="gloo")
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                          "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                          str(_free_port()), "bench.py", "--workload", "descent-sac", "--gpus", "2",
                          "--steps", "4", "--warmup", "2"], cwd=REPO, capture_output=True, text=True,
                         timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["config"]["envs_total"] == 4096 and r["config"]["envs_per_gpu"] == 2048
    # (gloo ranks: the torch.distributed reduce, eager; RCCL cannot put two ranks on one GPU)
    assert r["config"]["update"] == "FusedSAC" and r["config"]["hip_graph"] is False
    assert r["config"]["learner_reduce"].startswith("torch.distributed")
    ln = r["env_policy_learner"]
    assert ln["value"] > 0 and ln["critic_loss"] == ln["critic_loss"] and ln["actor_loss"] == ln["actor_loss"]


def test_bench_descent_sac_one_rank_rccl_reduce_in_graph():
    """the C5 iteration with the learner's gradient all-reduce over
    libbsg's RCCL communicator (a one-rank communicator here) stays one HIP graph, and the
    reduce calls were issued (captured, then replayed)."""
    out = subprocess.run([sys.executable, "bench.py", "--workload", "descent-sac", "--steps", "10",
                          "--warmup", "3"], cwd=REPO, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    assert r["config"]["hip_graph"] is True
    assert r["config"]["learner_reduce"].startswith("rccl")
    ln = r["env_policy_learner"]
    assert ln["value"] > 0 and ln["critic_loss"] == ln["critic_loss"]
