"""bench.py --gpus N launches its own ranks: the launcher's env / port plumbing,
rank-0 stdout relay and failure propagation, driven with a stand-in rank script (no GPU: the
launcher itself makes no GPU call and imports nothing of librmx)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

RANK_SCRIPT = r'''
import json, os, sys, time
r = int(os.environ["RANK"])
env = {k: os.environ[k] for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
mode = sys.argv[1]
if mode == "gloo":  # a real rendezvous over the launcher's MASTER_ADDR / MASTER_PORT, max over ranks
    import torch, torch.distributed as dist
    dist.init_process_group("gloo")
    t = torch.tensor([float(r + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    env["max"] = t.item()
    g = [None] * dist.get_world_size()
    dist.all_gather_object(g, {"rank": r, "ok": True})
    env["gathered"] = g
    dist.destroy_process_group()
if mode == "fail" and r == int(sys.argv[2]):
    sys.exit(7)
if mode == "fail":
    time.sleep(60)  # the launcher must stop this rank when the other fails
if r == 0:
    print(json.dumps(env), flush=True)
'''


def _script(tmp_path):
    p = tmp_path / "rank.py"
    p.write_text(RANK_SCRIPT)
    return str(p)


def test_launcher_env_and_rank0_line(tmp_path, capfd):
    import bench
    st = bench.launch_ranks(3, ["gloo"], script=_script(tmp_path))
    out = capfd.readouterr().out.strip().splitlines()
    assert st == 0 and out
    d = json.loads(out[-1])  # (this stand-in rank leaves gloo's banner on stdout; bench.py moves it to stderr)
    assert d["RANK"] == "0" and d["LOCAL_RANK"] == "0" and d["WORLD_SIZE"] == "3"
    assert d["MASTER_ADDR"] == "127.0.0.1" and int(d["MASTER_PORT"]) > 0
    assert d["max"] == 3.0 and [g["rank"] for g in d["gathered"]] == [0, 1, 2]


@pytest.mark.parametrize("bad", [0, 1])
def test_launcher_propagates_a_failing_rank(tmp_path, bad):
    import time
    import bench
    t0 = time.time()
    st = bench.launch_ranks(2, ["fail", str(bad)], script=_script(tmp_path), grace_s=2.0)
    assert st == 7
    assert time.time() - t0 < 30  # the surviving rank was stopped, not waited out


def test_bench_cli_launcher_exit_status(tmp_path):
    """The real entry point: `bench.py --gpus 2` with no WORLD_SIZE becomes the launcher; its ranks
    fail here (no GPU / librmx device), and the launcher exits non-zero instead of hanging."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = ""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup",
                        "0", "--no-cpu-baseline", "--settle-ms", "0"], env=env, capture_output=True, timeout=600)
    assert p.returncode != 0
    assert b"exited with status" in p.stderr


def test_launcher_forwards_sigterm_to_its_ranks(tmp_path):
    """A launcher stopped by its caller (the driver's time limit) stops its ranks: none outlives it."""
    import signal
    import time
    script = tmp_path / "rank.py"
    script.write_text("import os, time\nopen(os.environ['OUTDIR'] + '/pid%s' % os.environ['RANK'], 'w')"
                      ".write(str(os.getpid()))\ntime.sleep(120)\n")
    launcher = tmp_path / "launch.py"
    launcher.write_text("import sys\nsys.path.insert(0, %r)\nimport bench\n"
                        "raise SystemExit(bench.launch_ranks(2, [], script=%r))\n" % (ROOT, str(script)))
    env = dict(os.environ, OUTDIR=str(tmp_path))
    p = subprocess.Popen([sys.executable, str(launcher)], env=env)
    t0 = time.time()
    while len(list(tmp_path.glob("pid*"))) < 2 and time.time() - t0 < 60:
        time.sleep(0.1)
    pids = [int(f.read_text()) for f in tmp_path.glob("pid*")]
    assert len(pids) == 2
    p.send_signal(signal.SIGTERM)
    assert p.wait(30) != 0
    time.sleep(1.0)
    for pid in pids:  # gone (or at most a zombie awaiting a reaper other than the launcher)
        try:
            state = [ln for ln in open("/proc/%d/status" % pid) if ln.startswith("State:")][0]
        except (FileNotFoundError, IndexError):
            continue
        assert "Z" in state.split()[1], (pid, state)
