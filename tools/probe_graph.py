"""Probe: DeepFM forwards replayed from a HIP graph vs launched one by one (GPU box only).

For each launch batch: N forwards launched directly, then the same forwards captured on the context stream
(hipStreamBeginCapture, relaxed mode) R per graph and replayed N / R times.  Prints ms per forward for both
and whether the replayed outputs are bitwise the direct ones.  Timing: host wall clock over N forwards
between two stream synchronisations (the GPU is the bottleneck: the launches are asynchronous)."""
import ctypes
import sys
import time

import numpy as np

sys.path.insert(0, "recommendation-models_amd")
import rmx  # noqa: E402

F, K, FC = 39, 16, (400, 400, 400)
hip = ctypes.CDLL("libamdhip64.so")
vp = ctypes.c_void_p


def chk(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: hip error {rc}")


def main():
    ctx = rmx.default_context()
    rmx.set_tuning("lazy_fence", 1)  # (no event record per call on the context stream)
    s = vp(ctx.stream)
    V = 1_000_000
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(7)
    for B in [int(x) for x in (sys.argv[1:] or ["1024", "2048", "4096", "65536"])]:
        m = rmx.DeepFM(V, F, K, list(FC))
        m.setMats(m.initMats(3))
        m.setBias(0.01)
        ids = rmx.DeviceArray(ctx, B * F, np.int32)
        rmx.gen_ids(ctx, 11, 0, B, F, V, ids)
        out = rmx.DeviceArray(ctx, B, np.float32)
        m.forward_ids(table, B, ids, out)
        ctx.sync()
        ref = out.numpy().copy()
        N = 4000 if B <= 4096 else 400
        for rep in range(2):
            ctx.sync()
            t0 = time.perf_counter()
            for _ in range(N):
                m.forward_ids(table, B, ids, out)
            ctx.sync()
            t_direct = (time.perf_counter() - t0) / N * 1e3
            res = {}
            for R in (1, 20):
                g, ge = vp(), vp()
                chk(hip.hipStreamBeginCapture(s, 2), "begin capture")
                for _ in range(R):
                    m.forward_ids(table, B, ids, out)
                chk(hip.hipStreamEndCapture(s, ctypes.byref(g)), "end capture")
                chk(hip.hipGraphInstantiate(ctypes.byref(ge), g, None, None, ctypes.c_size_t(0)), "instantiate")
                out.numpy()  # (sync)
                chk(hip.hipGraphLaunch(ge, s), "launch")
                ctx.sync()
                same = bool(np.array_equal(out.numpy(), ref))
                n = N // R
                t0 = time.perf_counter()
                for _ in range(n):
                    chk(hip.hipGraphLaunch(ge, s), "launch")
                ctx.sync()
                res[R] = ((time.perf_counter() - t0) / (n * R) * 1e3, same)
                hip.hipGraphExecDestroy(ge)
                hip.hipGraphDestroy(g)
            print(f"B {B} rep {rep}: direct {t_direct:.4f} ms/fwd; graph R=1 {res[1][0]:.4f} (bitwise {res[1][1]}); "
                  f"graph R=20 {res[20][0]:.4f} (bitwise {res[20][1]})", flush=True)


if __name__ == "__main__":
    main()
