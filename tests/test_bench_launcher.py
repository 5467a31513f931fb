"""CPU: `bench.py --gpus N` without a launcher spawns N rank processes itself (before any
GPU call, no re-exec) and reports n_gpus = N; a wrong rank count is an error, never a
silent single rank. The dry-run step replaces the join (no GPU here)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, env=None):
    e = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          timeout=240, env=e, cwd=ROOT)


def test_gpus_2_without_launcher_spawns_two_ranks():
    r = _run("--gpus", "2", "--dry-run", "--steps", "2", "--warmup", "1")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout  # one JSON line (rank 0), nothing else on stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["ranks_reporting"] == 2
    # the ranks joined the spawning parent's listening store, not a port picked by closing
    # a socket
    assert d["rendezvous"] == "parent-store"
    assert d["steps"] == 2 and d["warmup"] == 1
    assert "dry-run" in d["data"]
    # the stage fields the N > 1 lines carry: a measured build span (no literal 0.0) and
    # the host time per step
    assert d["build_ms"] is not None and d["build_ms"] > 0
    assert d["probe_ms"] is not None and d["probe_ms"] > 0
    assert d["host_ms_per_step"] is not None and d["host_ms_per_step"] > 0


def test_no_literal_zero_build_ms():
    """No job in bench.py appends a placeholder build time."""
    with open(os.path.join(ROOT, "bench.py")) as f:
        src = f.read()
    assert "build_ms.append(0.0)" not in src


def test_no_port_picked_by_closing_a_socket():
    """No launcher, test or tool finds a port by binding port 0 and closing the socket."""
    import glob

    files = [os.path.join(ROOT, "bench.py")] + glob.glob(os.path.join(ROOT, "tests", "*.py")) + \
        glob.glob(os.path.join(ROOT, "tools", "*.py")) + \
        glob.glob(os.path.join(ROOT, "datafusion-parallelism_amd", "*.py"))
    for fn in files:
        if os.path.abspath(fn) == os.path.abspath(__file__):
            continue
        with open(fn) as f:
            src = f.read()
        assert "socket.socket(" not in src and ".bind((" not in src, fn


def test_world_size_mismatch_is_an_error():
    r = _run("--gpus", "2", "--dry-run", "--steps", "1", "--warmup", "0",
             env={"RANK": "0", "WORLD_SIZE": "1", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                  "MASTER_PORT": "29591"})
    assert r.returncode != 0
    assert "WORLD_SIZE" in r.stderr
