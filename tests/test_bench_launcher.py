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
if mode == "parity":  # every rank checks its rows; rank argv[2] misses -- bench.job_status decides the rc
    import torch.distributed as dist
    sys.path.insert(0, os.environ["BENCH_ROOT"])
    import bench
    dist.init_process_group("gloo")
    bad = int(sys.argv[2])
    pc = {"rows": 512, "max_abs_diff": 1.0 if r == bad else 5.96e-8, "tol": 1e-5, "ok": r != bad}
    if len(sys.argv) > 3:  # the default line's shape: the DeepFM and xDeepFM records of each rank
        pc = {"deepfm": dict(pc, ok=True), "xdeepfm": pc}
    g = [None] * dist.get_world_size()
    dist.all_gather_object(g, pc)
    dist.destroy_process_group()
    st = bench.job_status(g)
    if r == 0:
        print(json.dumps({"parity_ok": all(bench._pc_ok(p) for p in g)}), flush=True)
    sys.exit(st)
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


@pytest.mark.parametrize("bad,shape", [(1, "flat"), (0, "flat"), (1, "models"), (-1, "flat")])
def test_launcher_fails_on_a_rank_parity_miss(tmp_path, bad, shape, monkeypatch, capfd):
    """one rank's rows missing the oracle at N > 1 fail the whole job's exit status
    (bench.STATUS_PARITY_MISS), not only a parity_ok: false inside the line; no miss exits 0."""
    import bench
    monkeypatch.setenv("BENCH_ROOT", ROOT)
    argv = ["parity", str(bad)] + (["models"] if shape == "models" else [])
    st = bench.launch_ranks(3, argv, script=_script(tmp_path), grace_s=2.0)
    out = capfd.readouterr().out.strip().splitlines()
    assert st == (0 if bad < 0 else bench.STATUS_PARITY_MISS)
    assert json.loads(out[-1])["parity_ok"] == (bad < 0)


def test_job_status_companion_and_cpu_records():
    import bench
    ok = {"ok": True}
    assert bench.job_status([ok, ok]) == 0
    assert bench.job_status([ok], {"error": "TimeoutError"}) == bench.STATUS_COMPANION_FAILED
    assert bench.job_status([ok], {"parity_ok": False}) == bench.STATUS_PARITY_MISS
    assert bench.job_status(None, None, {"parity_check": {"ok": False}}) == bench.STATUS_PARITY_MISS
    assert bench.job_status(None, None, {"parity_check": {"ok": True}}, {"value": 1.0}) == 0


def test_record_status_error_is_not_a_parity_miss():
    """an encoder / L-A sub-record that raised (e.g. out of memory at V = 100M) exits with its
    own status and reason, not as a parity miss; a failed check is still a parity miss."""
    import bench
    enc_ok = {"note": "x", "V1M": {"parity_check": {"bitwise_equal": True}}}
    la_ok = {"note": "x", "B100": {"parity_check": {"ok": True}}}
    assert bench.record_status(enc_ok, la_ok) == 0
    assert bench.record_status(None, None) == 0
    assert bench.record_status({"V100M": {"error": "RmxError: out of device memory"}}, la_ok) == \
        bench.STATUS_RECORD_ERROR
    assert bench.record_status(enc_ok, {"B4096": {"error": "x"}}) == bench.STATUS_RECORD_ERROR
    assert bench.record_status({"V1M": {"parity_check": {"bitwise_equal": False}}}, la_ok) == \
        bench.STATUS_PARITY_MISS
    assert bench.record_status(enc_ok, {"B100": {"parity_check": {"ok": False}}}) == bench.STATUS_PARITY_MISS
    assert bench.STATUS_REASON[bench.STATUS_RECORD_ERROR] != bench.STATUS_REASON[bench.STATUS_PARITY_MISS]


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
