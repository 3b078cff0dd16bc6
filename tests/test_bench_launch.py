"""bench.py's own N-rank launch (`python bench.py --gpus N` without torch.distributed.run): the
parent starts N children with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, relays rank 0's one
JSON line, and fails when any rank fails; a launcher whose WORLD_SIZE disagrees with --gpus is
refused.  CPU only: the children here are a stand-in script, not the GPU bench."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

CHILD = r'''
import json, os, sys, time
r, w = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
assert os.environ["MASTER_ADDR"] == "127.0.0.1" and int(os.environ["MASTER_PORT"]) > 0
assert os.environ["LOCAL_RANK"] == str(r)
mode = sys.argv[1]
if mode == "fail" and r == w - 1:
    sys.exit(3)
if mode == "fail":
    time.sleep(60)          # a rank waiting in a collective for the failed one
if r == 0:
    print("log line to stderr", file=sys.stderr)
    print(json.dumps({"n_gpus": w, "argv": sys.argv[1:]}))
'''


@pytest.fixture()
def child(tmp_path):
    p = tmp_path / "child.py"
    p.write_text(CHILD)
    return str(p)


def test_rank_envs():
    envs = bench.rank_envs(3, {"X": "1"}, 12345)
    assert [e["RANK"] for e in envs] == ["0", "1", "2"]
    assert all(e["WORLD_SIZE"] == "3" and e["MASTER_PORT"] == "12345" and e["X"] == "1" for e in envs)
    assert all(e["MASTER_ADDR"] == "127.0.0.1" for e in envs)


def test_launch_relays_rank0_line(child, capfd):
    rc = bench.launch_ranks(["ok", "--steps", "2"], 4, timeout_s=60, script=child)
    assert rc == 0
    out = capfd.readouterr().out.strip().splitlines()
    assert len(out) == 1
    line = json.loads(out[0])
    assert line == {"n_gpus": 4, "argv": ["ok", "--steps", "2"]}


def test_launch_fails_when_a_rank_fails(child):
    rc = bench.launch_ranks(["fail"], 3, timeout_s=50, script=child)
    assert rc == 3


def test_world_size_mismatch_is_refused():
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, timeout=120)
    assert r.returncode == 2
    assert b"WORLD_SIZE=3" in r.stderr
