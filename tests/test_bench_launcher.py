"""bench.py --gpus N as its own launcher (CPU only: the ranks never reach the GPU here).

A rank that never finishes (a hang in a rendezvous or a collective on a first 8-GPU run)
must not leave the driver without a JSON line: after --deadline the launcher stops every
rank and prints one line with status "timeout" and each rank's last phase, exit 124."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_launcher_deadline_stops_hung_ranks():
    env = dict(os.environ, KRR_BENCH_TEST_HANG="1")
    t0 = time.time()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--deadline", "3"],
                       capture_output=True, text=True, env=env, timeout=120)
    assert time.time() - t0 < 60
    assert p.returncode == 124, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    r = json.loads(lines[0])
    assert r["status"] == "timeout" and r["n_gpus"] == 3 and r["ranks_running"] == [0, 1, 2]
    assert r["rank_phases"] == {"0": "init", "1": "init", "2": "init"}
    assert "KRR_PHASE rank=2 init" in p.stderr  # the ranks' stderr is forwarded



def test_rank_watchdog_under_an_external_launcher():
    """Under torchrun (the driver's N > 1 runs: WORLD_SIZE set by the launcher, not by
    bench.py) a hung rank ends itself after --deadline: rank 0 prints the timeout line."""
    env = dict(os.environ, KRR_BENCH_TEST_HANG="1", WORLD_SIZE="2", RANK="0", LOCAL_RANK="0",
               MASTER_ADDR="127.0.0.1", MASTER_PORT="29999")
    env.pop("KRR_BENCH_LAUNCHED", None)
    t0 = time.time()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--deadline", "3"],
                       capture_output=True, text=True, env=env, timeout=120)
    assert time.time() - t0 < 60
    assert p.returncode == 124, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    r = json.loads(lines[0])
    assert r["status"] == "timeout" and r["n_gpus"] == 2 and r["rank_phases"] == {"0": "init"}
