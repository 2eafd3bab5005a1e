"""configs[0] end to end: LR on a 1k-row synthetic Criteo slice (BASELINE.json configs[0]).

The reference path (example/LRLocalExample.scala:13-58, Spark local[.] with batchSize 100):
  LIBSVM text -> SampleParser.parse (data/SampleParser.scala:23-51) -> per 100-line batch: pull +
  makeWeights (ParRecModel.scala:279-284) -> LR.forward = sigma(Scatter(w) + bias) (model/lr/LR.scala:43-59)
  -> AUC over the slice.
Here: the same text from the splitmix generator (rmx.synthetic) -> the native parser at 2 threads
(Spark local[2]) -> LR through librmx, both boundaries (L-A host arrays exactly as RecModel.forward,
L-B ids against the HBM table) -> the device AUC; every stage against the oracle / restatements.
"""
import numpy as np
import pytest

import oracle_ctypes as oc
import ref_parser

F, V, ROWS, BATCH = 39, 1_000_000, 1000, 100
SEED_IDS, SEED_LAB, SEED_TAB = 0x5EED2026, 0x1AB3, 0x7AB1E


def _slice():
    from rmx import synthetic
    return synthetic.libsvm_text(SEED_IDS, SEED_LAB, 0, ROWS, F, V)


def test_host_generator_matches_oracle_and_parsers():
    import rmx
    text, ids, labels = _slice()
    assert np.array_equal(ids.ravel(), oc.gen_ids(SEED_IDS, 0, ROWS, F, V))
    assert 0.15 < labels.mean() < 0.35
    s = rmx.Samples(text, rmx.FORMAT_LIBSVM, 2)
    rows, cols, vals, targets, _ = ref_parser.parse(text.splitlines())
    assert np.array_equal(s.rows, rows) and np.array_equal(s.cols, cols)
    assert np.array_equal(s.values, vals) and np.array_equal(s.targets, targets)
    assert np.array_equal(s.cols, ids.ravel().astype(np.int64)) and np.array_equal(s.targets, labels)
    assert np.array_equal(s.ids(F), ids.ravel())


@pytest.mark.gpu
def test_lr_plumbing_configs0_end_to_end():
    import rmx
    from test_metric import auc_ref
    text, _, labels = _slice()
    s = rmx.Samples(text, rmx.FORMAT_LIBSVM, 2)  # Spark local[2]
    wt, _ = oc.gen_table(SEED_TAB, V, 0)
    bias = np.array([0.01], np.float32)
    lr = rmx.LR(V, F)
    om = oc.make_model(oc.LR)
    # L-A, batch by batch as ParRecModel.predictBiasWeight: makeWeights on the host, RecModel.forward
    p_la = np.zeros(ROWS, np.float32)
    ref = np.zeros(ROWS, np.float32)
    for b0 in range(0, ROWS, BATCH):
        sel = (s.rows >= b0) & (s.rows < b0 + BATCH)
        index, cols = s.rows[sel] - b0, s.cols[sel]
        w = wt[cols]  # makeWeights: w[n] = W1[feats[n]]
        p_la[b0:b0 + BATCH] = lr.forward(BATCH, (index, cols), bias, w)
        ref[b0:b0 + BATCH] = oc.forward(om, BATCH, index, bias, w, None, None, 0, 2)
    assert np.abs(p_la - ref).max() <= 1e-7
    # L-B: the parsed ids against the HBM table, predict loop of 100-row forwards
    ctx = rmx.default_context()
    table = rmx.EmbeddingTable(ctx, V, 0)
    table.fill_synthetic(SEED_TAB)
    lr.setBias(0.01)
    ids = rmx.DeviceArray.from_numpy(ctx, s.ids(F))
    scores = rmx.DeviceArray(ctx, ROWS, np.float32)
    lr.predict_ids(table, ROWS, ids, scores, batch=BATCH)
    ctx.sync()
    p_lb = scores.numpy()
    assert np.array_equal(p_lb, p_la)
    dl = rmx.DeviceArray.from_numpy(ctx, s.targets)
    a = rmx.auc(ctx, dl, scores)
    assert a == pytest.approx(auc_ref(labels, p_la), abs=1e-12)
