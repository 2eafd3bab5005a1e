"""Exit-time teardown and the L-A stage timers.

rmx.shutdown() is an atexit hook: it synchronises every live Context and destroys the live tables, models,
device buffers, exchange groups and contexts in that order while the HIP runtime is still up, instead of
leaving them to __del__ during interpreter teardown.  The subprocess tests exit WITHOUT closing anything and
require a clean exit status.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "recommendation-models_amd")


def _run(code, timeout=120):
    env = dict(os.environ, PYTHONPATH=PKG + os.pathsep + os.environ.get("PYTHONPATH", ""))
    return subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=timeout)


def test_shutdown_host_only_objects_and_closed_model_raises():
    r = _run("""
import rmx
m = rmx.DeepFM(1000, 39, 16, [64, 32])
assert m.getMatsSize()[0] == 624
keep = rmx.XDeepFM(1000, 39, 16, [64], [8])     # left open: the atexit hook destroys it
rmx.shutdown()
try:
    m.setBias(0.1)
    raise SystemExit("a closed model did not raise")
except rmx.RmxError:
    pass
rmx.shutdown()                                  # idempotent
print("done")
""")
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().endswith("done")


@pytest.mark.gpu
def test_exit_with_live_gpu_objects_is_clean():
    """Context, tables (plain, loopback shard, group shard), models, buffers and views all left open at exit."""
    r = _run("""
import numpy as np
import rmx
ctx = rmx.default_context()
t = rmx.EmbeddingTable(ctx, 1000, 16)
t.fill_synthetic(7)
m = rmx.DeepFM(1000, 39, 16, [400, 400, 400], ctx=ctx)
m.setMats(m.initMats(3))
m.setBias(0.01)
ids = rmx.DeviceArray(ctx, 64 * 39, np.int32)
rmx.gen_ids(ctx, 1, 0, 64, 39, 1000, ids)
out = rmx.DeviceArray(ctx, 64, np.float32)
v = out.view(0, 32)
m.forward_ids(t, 64, ids, out)
sh = rmx.ShardedTable(ctx, 1000, 16, 2)        # loopback shard: both partitions in this process
sh.fill_synthetic(7)
m.forward_ids_sharded(sh, 64, ids, out)
g = rmx.ExchangeGroup(1)
gs = rmx.ShardedTable(ctx, 1000, 16, 1, 0, group=g)
x = rmx.XDeepFM(1000, 39, 16, [64], [16], ctx=ctx)
x.setMats(x.initMats(5))
x.setBias(0.01)
x.forward_ids(t, 64, ids, out)                  # queued, not synchronised: the hook syncs first
print("done")
""")
    assert r.returncode == 0, (r.returncode, r.stderr[-3000:])
    assert r.stdout.strip().endswith("done")


@pytest.mark.gpu
def test_la_forward_reports_its_host_transfer_stages():
    """rmx_forward (L-A) with timing on: la_mats (the per-call mats H2D + pack), la_h2d (gathered rows) and
    la_d2h appear beside the kernels' stages, and the result does not depend on the timing."""
    import oracle_ctypes as oc
    import rmx
    B, F, K, V = 100, 39, 16, 1000
    m = rmx.DeepFM(V, F, K, [400, 400, 400])
    mats = m.initMats(11)
    ids = oc.gen_ids(3, 0, B, F, V).astype(np.int64)
    wt, et = oc.gen_table(5, V, K)
    w, e = oc.gather(wt, et, 1, ids)
    index = np.repeat(np.arange(B, dtype=np.int64), F)
    args = (B, (index, ids), np.array([0.01], np.float32), w, e, K, mats, m.getMatsSize())
    p0 = m.forward(*args)
    m.set_timing(True)
    p1 = m.forward(*args)
    p2 = m.forward(*args)
    stages, calls = m.get_timing()
    m.set_timing(False)
    assert calls == 2
    for s in ("la_mats", "la_h2d", "la_d2h"):
        assert s in stages and stages[s] > 0.0, stages
    assert any(not s.startswith("la_") for s in stages), stages
    assert np.array_equal(p0, p1) and np.array_equal(p0, p2)
    m.close()
