"""bench.py's own N-rank launcher (`python bench.py --gpus N` with no
torchrun): each child gets the torchrun environment, the parent never imports
torch (so it never initialises HIP before the ranks take their GPUs), the
worst child status is the parent's, and a rank left waiting on a dead peer is
ended.  Fake workers only: nothing here touches a GPU."""
from __future__ import annotations

import json
import subprocess
import sys
import time

from conftest import ROOT

ENV_KEYS = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")


def _bench():
    if str(ROOT) not in sys.path:
        sys.path.insert(0, str(ROOT))
    import bench

    return bench


def test_children_get_rank_environment(tmp_path):
    bench = _bench()
    code = ("import json, os, sys; "
            f"open(os.path.join({str(tmp_path)!r}, 'r' + os.environ['RANK']), 'w')"
            f".write(json.dumps({{k: os.environ[k] for k in {ENV_KEYS!r}}}))")
    assert bench.launch_ranks(3, [sys.executable, "-c", code]) == 0
    envs = [json.loads((tmp_path / f"r{r}").read_text()) for r in range(3)]
    assert [e["RANK"] for e in envs] == ["0", "1", "2"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2"]
    assert {e["WORLD_SIZE"] for e in envs} == {"3"}
    assert {e["MASTER_ADDR"] for e in envs} == {"127.0.0.1"}
    assert len({e["MASTER_PORT"] for e in envs}) == 1


def test_worst_status_and_stuck_rank_is_ended():
    bench = _bench()
    # rank 1 fails at once; rank 0 would wait "forever" on it (a collective
    # with a dead peer): the launcher ends it after the grace period
    code = "import os, sys, time; r = int(os.environ['RANK']); time.sleep(600) if r == 0 else sys.exit(3)"
    t0 = time.monotonic()
    rc = bench.launch_ranks(2, [sys.executable, "-c", code], grace_s=1.0)
    assert rc == 3 or rc == 128 + 15  # rank 1's 3, or rank 0's SIGTERM, whichever is worse
    assert rc >= 3 and time.monotonic() - t0 < 60


def test_signal_death_reported_as_shell_status():
    bench = _bench()
    code = "import os, signal; os.kill(os.getpid(), signal.SIGKILL)"
    assert bench.launch_ranks(1, [sys.executable, "-c", code]) == 128 + 9


def test_main_spawns_before_touching_torch():
    """`bench.py --gpus 2` without WORLD_SIZE re-runs itself as two ranks; the
    parent must not have imported torch (HIP) by then."""
    probe = f"""
import os, sys
sys.path.insert(0, {str(ROOT)!r})
os.environ.pop('WORLD_SIZE', None)
import bench
seen = {{}}
def fake(n, cmd, grace_s=60.0):
    seen['n'], seen['cmd'] = n, cmd
    seen['torch'] = 'torch' in sys.modules
    return 7
bench.launch_ranks = fake
sys.argv = ['bench.py', '--gpus', '2', '--steps', '3']
try:
    bench.main()
except SystemExit as e:
    seen['rc'] = e.code
import json; print(json.dumps(seen))
"""
    out = subprocess.run([sys.executable, "-c", probe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    seen = json.loads(out.stdout.strip().splitlines()[-1])
    assert seen["n"] == 2 and seen["rc"] == 7 and seen["torch"] is False
    assert seen["cmd"][-4:] == ["--gpus", "2", "--steps", "3"] and seen["cmd"][-5].endswith("bench.py")


def test_world_size_mismatch_is_an_error():
    probe = f"""
import os, sys
sys.path.insert(0, {str(ROOT)!r})
os.environ['WORLD_SIZE'] = '4'
import bench
sys.argv = ['bench.py', '--gpus', '2']
bench.main()
"""
    out = subprocess.run([sys.executable, "-c", probe], capture_output=True, text=True, timeout=120)
    assert out.returncode != 0 and "WORLD_SIZE=4" in out.stderr
