"""Pure-Python restatement of yr/data/SampleParser.scala:23-85 (TEST INFRASTRUCTURE ONLY).

Follows the Java calls literally: String.split(" ") / split(":") (regex split: trailing empty
strings removed, others kept), Float.parseFloat, Long.parseLong(...) - 1.  Used to check the
native parser (csrc/parse.cpp) on the same text."""
import numpy as np


class ParseError(Exception):
    pass


def java_split(s, sep):
    parts = s.split(sep)
    while len(parts) > 1 and parts[-1] == "":
        parts.pop()
    if parts == [""] and s != "":
        parts = []
    return parts


def _long(t):
    if not t or not (t.lstrip("+-").isdigit()) or t.count("+") + t.count("-") > 1 or t[1:].lstrip("0123456789"):
        raise ParseError("NumberFormatException: " + repr(t))
    return int(t)


def _float(t):
    try:
        if t.strip() != t or t == "":
            raise ValueError
        return np.float32(float(t))
    except ValueError:
        raise ParseError("NumberFormatException: " + repr(t))


def parse(lines, ffm=False):
    rows, cols, fields, vals, targets = [], [], [], [], []
    for i, line in enumerate(lines):
        parts = java_split(line, " ")
        if not parts:
            raise ParseError("NumberFormatException: empty line")
        targets.append(_float(parts[0]))
        for p in parts[1:]:
            kv = java_split(p, ":")
            need = 3 if ffm else 2
            if len(kv) < need:
                raise ParseError("ArrayIndexOutOfBoundsException: " + repr(p))
            if ffm:
                fields.append(_long(kv[0]))
                kv = kv[1:]
            cols.append(_long(kv[0]) - 1)
            vals.append(_float(kv[1]))
            rows.append(i)
    return (np.array(rows, np.int64), np.array(cols, np.int64), np.array(vals, np.float32),
            np.array(targets, np.float32), np.array(fields, np.int64) if ffm else None)
