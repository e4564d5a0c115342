"""bench.py as its own launcher: `python bench.py --gpus N` with no
torchrun around it starts N rank processes itself (bench.self_launch). These
CPU tests drive the launcher with a stand-in rank program (a few lines of
Python that report their environment) and check the rank environment, the
re-printed line, the worst-exit-status rule and the grace-period kill; one
runs the real bench.py path on this GPU-less container, where the ranks must
fail loudly and the launcher must say so. The GPU test in tests/test_gpu.py
runs the real thing at N=2 on one shared device."""
import io
import json
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

RANK_PROG = r"""
import json, os, sys, time
r = int(os.environ["RANK"])
mode = os.environ.get("FAKE_MODE", "ok")
if r == 0:
    print("a progress line that is not the result", flush=True)
    print(json.dumps({"metric": "m", "value": 1.0, "env": {k: os.environ[k] for k in
          ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}, "argv": sys.argv[1:]}), flush=True)
if mode == "rank1_fails" and r == 1:
    sys.exit(5)
if mode == "rank1_hangs" and r == 1:
    time.sleep(600)
if mode in ("rank0_fails", "rank0_fails_rank1_hangs") and r == 0:
    sys.exit(7)
if mode == "rank0_fails_rank1_hangs" and r == 1:
    time.sleep(600)
if mode == "rank1_signal" and r == 1:
    os.kill(os.getpid(), 9)
"""


def _run(tmp_path, mode, n=3, grace_s=60.0, timeout_s=None):
    import bench

    prog = tmp_path / "rank.py"
    prog.write_text(RANK_PROG)
    os.environ["FAKE_MODE"] = mode
    try:
        buf = io.StringIO()
        t0 = time.monotonic()
        code = bench.self_launch(["--gpus", str(n), "--steps", "1"], n, cmd=[sys.executable, str(prog)],
                                 grace_s=grace_s, timeout_s=timeout_s, out=buf)
        el = time.monotonic() - t0
    finally:
        del os.environ["FAKE_MODE"]
    lines = [l for l in buf.getvalue().splitlines() if l.strip()]
    return code, [json.loads(l) for l in lines], el


def test_self_launch_sets_rank_env_and_reprints_rank0_line(tmp_path):
    code, lines, _ = _run(tmp_path, "ok", n=3)
    assert code == 0
    assert len(lines) == 1  # one line on stdout: rank 0's result, nothing else
    ln = lines[0]
    assert ln["env"]["RANK"] == "0" and ln["env"]["LOCAL_RANK"] == "0" and ln["env"]["WORLD_SIZE"] == "3"
    assert ln["env"]["MASTER_ADDR"] == "127.0.0.1" and int(ln["env"]["MASTER_PORT"]) > 0
    assert ln["argv"] == ["--gpus", "3", "--steps", "1"]
    assert "self-launch" in ln["launcher"]


def test_self_launch_returns_the_worst_status(tmp_path):
    code, lines, _ = _run(tmp_path, "rank1_fails")
    assert code == 5 and len(lines) == 1  # rank 0's line still printed
    code, lines, _ = _run(tmp_path, "rank0_fails")
    assert code == 7
    code, lines, _ = _run(tmp_path, "rank1_signal")
    assert code == 128 + 9


def test_self_launch_kills_a_hung_rank_after_a_failure(tmp_path):
    # rank 0 fails at once, rank 1 would sleep 10 minutes (a rank that lost
    # its peer in a collective): killed once the grace period is over
    code, lines, el = _run(tmp_path, "rank0_fails_rank1_hangs", n=2, grace_s=0.5)
    assert el < 30, el
    assert code == 128 + 9  # the killed rank's status is the worst one


def test_self_launch_bounds_the_whole_job(tmp_path):
    code, lines, el = _run(tmp_path, "rank1_hangs", n=2, timeout_s=2.0)
    assert el < 30, el
    assert code == 128 + 9 and len(lines) == 1


def test_launcher_parent_never_imports_torch():
    # the parent must not initialise HIP before its ranks start: run the
    # launcher in a fresh interpreter and check torch never entered it
    code = ("import sys, io; sys.path.insert(0, %r); import bench; "
            "rc = bench.self_launch([], 2, cmd=[sys.executable, '-c', 'pass'], out=io.StringIO()); "
            "print('torch' in sys.modules, rc)" % ROOT)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == ["False", "1"]  # ranks exited 0 but printed no line -> 1


def test_bench_self_launch_without_gpu_fails_loudly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present (tests/test_gpu.py runs the real N=2 launch)")
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["HCLIB_BENCH_LAUNCH_TIMEOUT_S"] = "200"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--share-device", "--no-extras", "--steps", "1", "--warmup", "0"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode != 0
    assert r.stdout.strip() == ""  # no result line without a GPU
