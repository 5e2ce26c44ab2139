"""bench.py's multi-rank launcher (`python bench.py --gpus N` without a
torchrun environment): child environment, argv, exit-code propagation and the
WORLD_SIZE / --gpus consistency check.  CPU only; the workers are stubs."""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

STUB = ("import os, sys, time\n"
        "r = os.environ['RANK']\n"
        "print('rank', r, os.environ['LOCAL_RANK'], os.environ['WORLD_SIZE'], os.environ['MASTER_ADDR'],"
        " os.environ['MASTER_PORT'], ' '.join(sys.argv[1:]), flush=True)\n"
        "if os.environ.get('SLEEP_RANK') == r: time.sleep(60)\n"
        "sys.exit(3 if os.environ.get('FAIL_RANK') == r else 0)\n")


def _env(**kw):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    e.update(kw)
    return e


def test_spawn_ranks_env_and_argv(capfd):
    rc = bench.spawn_ranks(4, [sys.executable, "-c", STUB, "--gpus", "4", "--steps", "7"], env=_env())
    assert rc == 0
    lines = sorted(l for l in capfd.readouterr().out.splitlines() if l.startswith("rank"))
    assert len(lines) == 4
    ports = set()
    for r, line in enumerate(lines):
        f = line.split()
        assert f[1] == str(r) and f[2] == str(r) and f[3] == "4" and f[4] == "127.0.0.1"
        assert " ".join(f[6:]) == "--gpus 4 --steps 7"
        ports.add(f[5])
    assert len(ports) == 1  # one rendezvous port for the job


def test_spawn_ranks_propagates_failure_and_stops_the_rest():
    t0 = time.time()
    rc = bench.spawn_ranks(3, [sys.executable, "-c", STUB], env=_env(FAIL_RANK="2", SLEEP_RANK="0"))
    assert rc == 3
    assert time.time() - t0 < 30  # the sleeping rank was terminated, not waited for


def test_spawn_ranks_timeout_terminates_hung_ranks():
    """a rank hung without exiting (here: sleeping) ends the job
    at the timeout with rc 124 and no child left behind"""
    t0 = time.time()
    rc = bench.spawn_ranks(2, [sys.executable, "-c", STUB], env=_env(SLEEP_RANK="1"), timeout_s=2.0)
    assert rc == 124
    assert time.time() - t0 < 30


def test_spawn_ranks_parent_interrupt_terminates_children(monkeypatch):
    """an exception in the parent's wait loop (SIGINT / SIGTERM) terminates
    the children before it propagates"""
    started = []
    real_popen = subprocess.Popen

    def popen(*a, **kw):
        pr = real_popen(*a, **kw)
        started.append(pr)
        return pr

    calls = {"n": 0}

    def sleep(_):
        calls["n"] += 1
        if calls["n"] == 3:
            raise KeyboardInterrupt

    monkeypatch.setattr(bench.subprocess, "Popen", popen)
    monkeypatch.setattr(bench.time, "sleep", sleep)
    try:
        bench.spawn_ranks(2, [sys.executable, "-c", STUB], env=_env(SLEEP_RANK="0"))
    except KeyboardInterrupt:
        pass
    else:
        raise AssertionError("KeyboardInterrupt not propagated")
    assert len(started) == 2 and all(pr.poll() is not None for pr in started)


def test_rank_command_reuses_the_parent_arguments():
    cmd = bench.rank_command(["--gpus", "8", "--steps", "5", "--warmup", "2"])
    assert cmd[0] == sys.executable and os.path.basename(cmd[1]) == "bench.py"
    assert cmd[2:] == ["--gpus", "8", "--steps", "5", "--warmup", "2"]


def test_world_size_must_match_gpus():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=_env(WORLD_SIZE="3"),
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 2
    assert "WORLD_SIZE=3 but --gpus 2" in r.stderr
