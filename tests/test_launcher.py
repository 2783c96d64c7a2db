"""bench.py's own rank launcher (mpvae_launch.py): `python bench.py --gpus N`
without torchrun starts N rank processes with the rendezvous environment set,
relays rank 0's stdout and fails when any rank fails.  Stub workers stand in
for the bench (no GPU here)."""
import io
import json
import os
import re
import subprocess
import sys
import time

import mpvae_launch as ML

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

STUB = r'''
import json, os, sys, time
r = int(os.environ["RANK"])
if r == int(os.environ.get("STUB_FAIL_RANK", "-1")):
    sys.exit(3)
if os.environ.get("STUB_HANG_OTHERS") and r != int(os.environ.get("STUB_FAIL_RANK", "-1")):
    time.sleep(60)
if r == 0:
    print(json.dumps({k: os.environ[k] for k in
                      ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}))
    print("x" * 200000)   # more than a pipe buffer: the launcher must drain it
print("rank", r, "done", file=sys.stderr)
'''


def _stub(tmp_path):
    p = tmp_path / "stub.py"
    p.write_text(STUB)
    return [sys.executable, str(p)]


def test_needs_spawn():
    assert ML.needs_spawn(2, {}) and ML.needs_spawn(8, {"RANK": "0"})
    assert not ML.needs_spawn(1, {})
    assert not ML.needs_spawn(8, {"WORLD_SIZE": "8"})   # torchrun already did it


def test_launch_sets_rank_env_and_relays_rank0(tmp_path):
    buf = io.StringIO()
    assert ML.launch_ranks(3, _stub(tmp_path), out=buf) == 0
    first = buf.getvalue().splitlines()[0]
    env = json.loads(first)
    assert env["RANK"] == "0" and env["LOCAL_RANK"] == "0" and env["WORLD_SIZE"] == "3"
    assert env["MASTER_ADDR"] == "127.0.0.1" and int(env["MASTER_PORT"]) > 0
    assert len(buf.getvalue()) > 200000


def test_failing_rank_fails_the_job_and_stops_the_others(tmp_path, monkeypatch):
    monkeypatch.setenv("STUB_FAIL_RANK", "1")
    monkeypatch.setenv("STUB_HANG_OTHERS", "1")
    t0 = time.time()
    rc = ML.launch_ranks(3, _stub(tmp_path), out=io.StringIO())
    assert rc == 3
    assert time.time() - t0 < 30   # the sleeping ranks were terminated


def test_bench_spawns_its_ranks(tmp_path):
    """bench.py --gpus 2 (no WORLD_SIZE) goes through the launcher before it
    touches the GPU: with no GPU here the ranks fail, and so does the parent."""
    env = {k: v for k, v in os.environ.items() if k not in ML.RANK_ENV}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--steps", "1", "--warmup", "0", "--config", "c2"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    # the message comes from a rank's setup_dist (whichever fails first)
    assert re.search(r"rank ([01]): LOCAL_RANK \1 but only 0 GPUs visible", r.stderr), \
        r.stderr[-2000:]
