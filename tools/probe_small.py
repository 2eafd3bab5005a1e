"""Timing probes of the small-batch whole-tower kernel (k_small_s3.hip, knob s3_small_diag: 1 no MFMAs, 2 no
weight loads, 4 no row gather; the results of a probe are wrong by construction).  The probe kernels exist only
in a build with -DRMX_SMALL_DIAG=1 (make EXTRA=-DRMX_SMALL_DIAG=1 in csrc/, after a make clean); otherwise every line is the
default kernel.  Prints the stage time per batch and probe.  Usage: python tools/probe_small.py [B ...]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "recommendation-models_amd"))
import numpy as np  # noqa: E402

import rmx  # noqa: E402

F, K, FC, V = 39, 16, (400, 400, 400), 1_000_000


def main():
    ctx = rmx.default_context()
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(0x7AB1E)
    for B in [int(a) for a in sys.argv[1:]] or [1024, 4096]:
        m = rmx.DeepFM(V, F, K, list(FC))
        m.setMats(m.initMats(0x3A75))
        m.setBias(0.01)
        ids = rmx.DeviceArray(ctx, B * F, np.int32)
        rmx.gen_ids(ctx, 0x5A11, 0, B, F, V, ids)
        out = rmx.DeviceArray(ctx, B, np.float32)
        for dg in (0, 1, 2, 3, 4, 7, 0):
            rmx.set_tuning("s3_small_diag", dg)
            for _ in range(50):
                m.forward_ids(table, B, ids, out)
            ctx.sync()
            m.set_timing(True)
            for _ in range(300):
                m.forward_ids(table, B, ids, out)
            ctx.sync()
            stages, calls = m.get_timing()
            m.set_timing(False)
            print("B=%d diag=%d %s" % (B, dg, {k: round(v / max(calls, 1), 4) for k, v in stages.items()}), flush=True)
    rmx.set_tuning("s3_small_diag", None)


if __name__ == "__main__":
    main()
