"""Independent numpy re-expression of the reference's BigDL module graphs (fp64).

TEST INFRASTRUCTURE ONLY.  It restates each model the way the Scala builds its
BigDL ``Sequential`` (Reshape / Sum / Power / CSubTable / Mean / MM / JoinTable /
Linear / CAddTable / Sigmoid) with whole-tensor numpy ops, as a second,
structurally different restatement to cross-check ``oracle/rmx_oracle.c``.
Paths are relative to /root/reference/src/main/scala/io/yaochi/recommendation/.
"""
import numpy as np


class Mats:
    """Unpacks flat ``mats`` like util/LayerUtil.scala:7-40 at running offsets."""

    def __init__(self, mats):
        self.m = np.asarray(mats, np.float64)
        self.off = 0

    def linear(self, n_in, n_out, with_bias):
        W = self.m[self.off:self.off + n_in * n_out].reshape(n_out, n_in)
        self.off += n_in * n_out
        b = None
        if with_bias:
            b = self.m[self.off:self.off + n_out]
            self.off += n_out
        return W, b

    def bias_layer(self, n):
        b = self.m[self.off:self.off + n]
        self.off += n
        return b


def _linear(x, Wb):
    W, b = Wb
    y = x @ W.T
    return y + b if b is not None else y


def _relu(x):
    return np.where(x > 0, x, 0.0)


def _sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


def scatter(B, index, w):
    """com/intel/analytics/bigdl/nn/Scatter.scala:17-36"""
    y = np.zeros(B)
    np.add.at(y, np.asarray(index), np.asarray(w, np.float64))
    return y


def fm(B, F, k, emb):
    """model/encoder/SecondOrderEncoder.scala:19-34"""
    E = np.asarray(emb, np.float64).reshape(B, F, k)
    square_sum = E.sum(axis=1) ** 2
    sum_square = (E ** 2).sum(axis=1)
    return 0.5 * (square_sum - sum_square).mean(axis=1)


def tower(x, mats, fc_dims, with_output):
    """model/encoder/HigherOrderEncoder.scala:34-59"""
    dim = x.shape[1]
    for d in fc_dims:
        x = _relu(_linear(x, mats.linear(dim, d, True)))
        dim = d
    if with_output:
        x = _linear(x, mats.linear(dim, 1, True))
    return x


def forward(kind, B, F, k, index, bias, weights, emb, mats_flat, fc=(), cin=(), cross_depth=0):
    bias = float(np.asarray(bias).reshape(-1)[0])
    if kind == "lr":  # model/lr/LR.scala:43-59
        return _sigmoid(scatter(B, index, weights) + bias)
    mats = Mats(mats_flat)
    E = np.asarray(emb, np.float64)
    x = E.reshape(B, F * k)
    if kind == "dnn":  # model/dnn/DNN.scala:54-73
        return _sigmoid(tower(x, mats, fc, True)[:, 0] + bias)
    y1 = scatter(B, index, weights)
    if kind == "deepfm":  # model/deepfm/DeepFM.scala:54-80
        y2 = fm(B, F, k, E)
        y3 = tower(x, mats, fc, True)[:, 0]
        return _sigmoid(((y1 + y2) + y3) + bias)
    if kind == "xdeepfm":  # model/xdeepfm/CINEncoder.scala:36-58, 105-176
        d = tower(x, mats, fc, False)
        x0 = E.reshape(B, F, k).transpose(0, 2, 1).reshape(B * k, F)
        u = x0
        pools = []
        hp = F
        for h in cin:
            Z = (x0[:, :, None] * u[:, None, :]).reshape(B * k, F * hp)  # MM(transB) + Reshape
            u = _relu(_linear(Z, mats.linear(F * hp, h, True)))
            pools.append(u.reshape(B, k, h).sum(axis=1))
            hp = h
        Wo, _ = mats.linear(sum(cin) + fc[-1], 1, False)
        y = np.concatenate(pools + [d], axis=1) @ Wo.T
        return _sigmoid((y1 + y[:, 0]) + bias)
    if kind == "dcn":  # model/dcn/CrossEncoder.scala:40-55, 107-185
        D = F * k
        ws = [mats.linear(D, 1, False)[0] for _ in range(cross_depth)]
        betas = [mats.bias_layer(1)[0] for _ in range(cross_depth)]
        xl = x
        for l in range(cross_depth):
            s = xl @ ws[l].T  # (B, 1)
            xl = ((x * s) + xl) + betas[l]
        d = tower(x, mats, fc, False)
        Wo, _ = mats.linear(D + fc[-1], 1, False)
        y = np.concatenate([xl, d], axis=1) @ Wo.T
        return _sigmoid((y1 + y[:, 0]) + bias)
    if kind == "pnn":  # model/pnn/ProductEncoder.scala:34-41, 72-120; PNN.scala:59-87
        D = F * k
        rows = [i for i in range(F) for j in range(i + 1, F)]
        cols = [j for i in range(F) for j in range(i + 1, F)]
        E3 = E.reshape(B, F, k)
        ip = (E3[:, rows, :] * E3[:, cols, :]).sum(axis=2)  # Gather + DotProduct2
        zo = _linear(x, mats.linear(D, fc[0], False))
        zi = _linear(ip, mats.linear(len(rows), fc[0], False))
        bp = mats.bias_layer(1)[0]
        h = _relu((zo + zi) + bp)
        y = tower(h, mats, fc[1:], True)[:, 0]
        return _sigmoid((y1 + y) + bias)
    raise ValueError(kind)
