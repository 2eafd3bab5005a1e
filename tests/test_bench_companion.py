"""bench.py's sharded sub-record guard (CPU, no GPU): an exception inside the companion is recorded
in the sub-record, and a companion that never returns is ended by the watchdog, which still prints
the main line (with the sub-record marked as timed out) and exits 124, so launch_ranks and the driver
see the hang."""
import json
import os
import subprocess
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _args(timeout=5.0):
    return types.SimpleNamespace(companion_timeout=timeout, steps=20, warmup=5)


def test_companion_exception_is_recorded(monkeypatch):
    import bench

    def boom(*a, **k):
        raise RuntimeError("RCCL error unhandled system error")
    monkeypatch.setattr(bench, "run", boom)
    sub = bench.sharded_companion(_args(), None, None, 0, 2, None, {"value": 1.0})
    assert sub["error"].startswith("RuntimeError: RCCL error")
    assert bench.LIVE_SHARDS == []


def test_companion_watchdog_prints_line_and_exits_124(tmp_path):
    script = tmp_path / "hang.py"
    script.write_text(
        "import sys, time, types\n"
        "sys.path.insert(0, %r)\n"
        "import bench\n"
        "class Shard:\n"
        "    def abort(self):\n"
        "        sys.stderr.write('aborted\\n')\n"
        "def hang(*a, **k):\n"
        "    bench.LIVE_SHARDS.append(Shard())\n"
        "    time.sleep(600)\n"
        "bench.run = hang\n"
        "args = types.SimpleNamespace(companion_timeout=1.0, steps=20, warmup=5)\n"
        "bench.sharded_companion(args, None, None, 0, 2, None, {'metric': 'm', 'value': 3.0})\n"
        "print('not reached')\n" % ROOT)
    p = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, timeout=60)
    assert p.returncode == 124, p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["value"] == 3.0 and "timed out" in d["models"]["deepfm_sharded"]["error"]
    assert "aborted" in p.stderr
