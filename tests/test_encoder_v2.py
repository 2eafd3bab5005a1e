"""The round-5 encoder kernel (csrc/k_encoder.hip encoder_k16v2_kernel: ids of a 40-field chunk loaded once and
quad-broadcast, rows + first-order weights requested in batches of U = 13 / 20, knob enc_u) against the
oracle and against the round-4 kernel (enc_u 0), bit for bit: gather (ParRecModel.scala:279-306), Scatter
first order (bnn/Scatter.scala:17-36), FM (SecondOrderEncoder.scala:19-34), LR's sigmoid head.

Fields: F = 1, 7, 39 (the bench), 40 (one whole chunk), 41 and 83 (a second chunk, ragged); row and line
tables (table_lines), fp32 and bf16 tables; ragged batch sizes."""
import numpy as np
import pytest

import oracle_ctypes as oc
import rmx

pytestmark = pytest.mark.gpu

K = 16
SEED_IDS, SEED_TAB = 0xE2C0, 0x7AB1E


@pytest.fixture(scope="module")
def ctx():
    return rmx.default_context()


@pytest.fixture(autouse=True)
def _restore():
    yield
    rmx.set_tuning("enc_u", None)
    rmx.set_tuning("table_lines", None)


def _encode(ctx, model, table, B, ids_dev, u):
    rmx.set_tuning("enc_u", u)
    y = rmx.DeviceArray(ctx, B, np.float32)
    model.encoder_ids(table, B, ids_dev, y)
    ctx.sync()
    return y.numpy().copy()


@pytest.mark.parametrize("F", [1, 7, 39, 40, 41, 83])
@pytest.mark.parametrize("B", [1, 1000, 65537])
def test_encoder_v2_bit_exact(ctx, F, B):
    V = 50000
    ids = oc.gen_ids(SEED_IDS, 3, B, F, V)
    wt, et = oc.gen_table(SEED_TAB, V, K)
    table = rmx.EmbeddingTable(ctx, V, K)
    table.upload(wt, et)
    ids_dev = rmx.DeviceArray.from_numpy(ctx, ids.astype(np.int32))
    deepfm = rmx.DeepFM(V, F, K, [32])
    lr = rmx.LR(V, F)  # (a non-DeepFM model: the encoder computes the first order only)
    for model, fm in ((deepfm, True), (lr, False)):
        res = {u: _encode(ctx, model, table, B, ids_dev, u) for u in (0, 13, 20)}
        assert np.array_equal(res[13], res[0]) and np.array_equal(res[20], res[0])
        n = min(B, 4096)
        w, e = oc.gather(wt, et, 1, ids[:n * F].astype(np.int64))
        index = np.repeat(np.arange(n, dtype=np.int64), F)
        ref = oc.first_order(n, index, w) + (oc.fm(n, F, K, e) if fm else 0.0)
        assert np.array_equal(res[20][:n], ref.astype(np.float32))


@pytest.mark.parametrize("B", [1000, 65536])
def test_encoder_v2_line_table_and_bf16(ctx, B):
    F, V = 39, 100_003
    ids_dev = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, ids_dev)
    m = rmx.DeepFM(V, F, K, [32])
    res = {}
    for lines in (0, 1):
        rmx.set_tuning("table_lines", lines)
        t = rmx.EmbeddingTable(ctx, V, K)
        t.fill_synthetic(SEED_TAB)
        for u in (0, 20):
            res[(lines, u)] = _encode(ctx, m, t, B, ids_dev, u)
    assert all(np.array_equal(r, res[(0, 0)]) for r in res.values())
    tb = rmx.EmbeddingTable(ctx, V, K, rmx.DTYPE_BF16)
    tb.fill_synthetic(SEED_TAB)
    assert np.array_equal(_encode(ctx, m, tb, B, ids_dev, 20), _encode(ctx, m, tb, B, ids_dev, 0))


def test_lr_forward_v2_bit_exact(ctx):
    """LR (encoder mode 2: sigmoid(first order + beta)) through the forward: v2 and round-4 kernel agree."""
    F, V, B = 39, 50000, 3001
    m = rmx.LR(V, F)
    m.setBias(0.01)
    t = rmx.EmbeddingTable(ctx, V, 0)
    t.fill_synthetic(SEED_TAB)
    ids_dev = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, ids_dev)
    out = rmx.DeviceArray(ctx, B, np.float32)
    res = []
    for u in (0, 13, 20):
        rmx.set_tuning("enc_u", u)
        m.forward_ids(t, B, ids_dev, out)
        ctx.sync()
        res.append(out.numpy().copy())
    assert np.array_equal(res[0], res[1]) and np.array_equal(res[0], res[2])

