"""Synthetic Criteo-shaped data on the host, bit-identical to the device generator.

ids[b, f] = f * (V // F) + splitmix64(seed ^ ((row0 + b) * F + f)) % (V // F)   (rmx_gen_ids)
labels[b] = 1 if splitmix64(label_seed ^ (row0 + b)) / 2^64 < positive_rate else 0

libsvm_text() writes them in the reference's input format (one sample per line, "label id:value" with
1-based ids, yr/data/SampleParser.scala:23-51 reads them back as id - 1): the configs[0] plumbing slice.
"""
import numpy as np

_M = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x):
    """Vectorised splitmix64 on uint64 arrays (wrapping arithmetic, as the C / HIP generators)."""
    x = np.asarray(x, np.uint64)
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def gen_ids(seed, row0, rows, n_fields, num_rows):
    """int32 ids [rows, n_fields], the values of rmx_gen_ids (field f owns [f*per, (f+1)*per))."""
    per = np.uint64(num_rows // n_fields)
    c = (np.arange(row0, row0 + rows, dtype=np.uint64)[:, None] * np.uint64(n_fields)
         + np.arange(n_fields, dtype=np.uint64)[None, :])
    h = splitmix64(np.uint64(seed) ^ c)
    return (np.arange(n_fields, dtype=np.uint64)[None, :] * per + h % per).astype(np.int32)


def gen_labels(label_seed, row0, rows, positive_rate=0.25):
    h = splitmix64(np.uint64(label_seed) ^ np.arange(row0, row0 + rows, dtype=np.uint64))
    u = (h >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
    return (u < positive_rate).astype(np.float32)


def libsvm_text(seed, label_seed, row0, rows, n_fields, num_rows):
    """(text, ids [rows, F], labels [rows]): LIBSVM lines "label id+1:1 ..." in field order."""
    ids = gen_ids(seed, row0, rows, n_fields, num_rows)
    labels = gen_labels(label_seed, row0, rows)
    one = (ids.astype(np.int64) + 1).astype(str)
    body = np.char.add(one, ":1")
    lines = ["%d %s" % (int(y), " ".join(r)) for y, r in zip(labels, body)]
    return "\n".join(lines) + "\n", ids, labels
