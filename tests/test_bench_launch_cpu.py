"""bench.py --gpus N self-launch (parallel.launch): N rank processes, whole-job
aggregation, global p50, failure propagation.  CPU ranks over gloo."""
import json
import os
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mcp_amd.parallel.launch import spawn_ranks  # noqa: E402


def _run_bench(*extra, timeout=600):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    env["OMP_NUM_THREADS"] = "2"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu",
                        "--model", "tiny", "--batch", "2", "--steps", "1", "--warmup", "0",
                        "--services", "3", "--min-nodes", "2", "--max-nodes", "2", *extra],
                       capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout        # rank 0 prints ONE JSON line
    return json.loads(lines[0]), r.stderr


def test_bench_self_launch_two_ranks():
    out, err = _run_bench("--gpus", "2")
    assert out["n_gpus"] == 2
    assert out["config"]["parallelism"] == "dp2"
    assert out["config"]["global_batch"] == 4
    # both ranks ran (each logs its own steps)
    assert "[rank 0] step 0" in err and "[rank 1] step 0" in err
    # whole-job value = all plans / the slowest rank's timed span
    span_s = out["ms_per_step"] * out["steps"] / 1e3
    assert abs(out["value"] - 4 / span_s) <= 0.01 * out["value"] + 1e-3
    assert out["p50_latency_ms"] > 0 and out["p99_latency_ms"] >= out["p50_latency_ms"]


def test_bench_single_rank_unchanged():
    out, err = _run_bench("--gpus", "1")
    assert out["n_gpus"] == 1 and out["config"]["parallelism"] == "dp1"
    assert out["config"]["global_batch"] == 2


def test_spawn_ranks_propagates_failure(tmp_path):
    script = tmp_path / "child.py"
    script.write_text(textwrap.dedent("""
        import os, sys, time
        if os.environ["RANK"] == "1":
            sys.exit(5)
        time.sleep(60)          # rank 0 would hang: the launcher must stop it
    """))
    assert spawn_ranks(str(script), [], 2) == 5


def test_spawn_ranks_env(tmp_path):
    script = tmp_path / "child.py"
    out = tmp_path / "out"
    out.mkdir()
    script.write_text(textwrap.dedent(f"""
        import os
        keys = ["RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR"]
        open(os.path.join({str(out)!r}, os.environ["RANK"]), "w").write(
            ",".join(os.environ[k] for k in keys))
    """))
    assert spawn_ranks(str(script), [], 3) == 0
    got = sorted(p.read_text() for p in out.iterdir())
    assert got == [f"{r},{r},3,3,127.0.0.1" for r in range(3)]
