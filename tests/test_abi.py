"""C-ABI checks that need no GPU: librmx.so loads, exports every function include/rmx.h declares,
and its host-side logic (getMatsSize, mats init, argument validation) matches the reference /
oracle.  No compute call is made here (there is no GPU in the build container)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import oracle_ctypes as oc
import rmx
from rmx import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", f) for f in sorted(os.listdir(os.path.join(ROOT, "include")))
           if f.endswith(".h")]


def declared_functions():
    names = set()
    for h in HEADERS:
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(rmx_\w+)\s*\(", src, flags=re.M):
            names.add(m.group(1))
    return names


def test_headers_declare_functions():
    names = declared_functions()
    assert "rmx_forward" in names and "rmx_forward_ids" in names and len(names) >= 30


def test_library_exports_every_declared_symbol():
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = sorted(declared_functions() - exported)
    assert not missing, missing
    for name in declared_functions():
        assert hasattr(_lib.lib, name)


def test_python_binding_covers_header():
    bound = {name for name, _, _ in _lib.SIGNATURES}
    assert not (declared_functions() - bound), sorted(declared_functions() - bound)


def test_abi_version():
    assert _lib.lib.rmx_abi_version() >= 1


def test_tuning_knob_set_and_reset():
    """rmx_set_tuning stores a knob; RMX_TUNING_DEFAULT (set_tuning(key, None)) removes it."""
    assert rmx.get_tuning("abi_test_knob", 7) == 7
    rmx.set_tuning("abi_test_knob", 3)
    assert rmx.get_tuning("abi_test_knob", 7) == 3
    rmx.set_tuning("abi_test_knob", None)
    assert rmx.get_tuning("abi_test_knob", 7) == 7
    rmx.set_tuning("abi_test_knob", None)  # removing an absent key is a no-op
    assert rmx.get_tuning("abi_test_knob", 5) == 5


KINDS = [
    (rmx.DeepFM, (1000, 39, 16, [400, 400, 400]), oc.DEEPFM, dict(fc=(400, 400, 400))),
    (rmx.DNN, (1000, 39, 16, [64, 32]), oc.DNN, dict(fc=(64, 32))),
    (rmx.XDeepFM, (1000, 39, 16, [400, 400, 400], [200, 200, 200]), oc.XDEEPFM,
     dict(fc=(400, 400, 400), cin=(200, 200, 200))),
    (rmx.XDeepFM, (1000, 39, 16, [64], [200]), oc.XDEEPFM, dict(fc=(64,), cin=(200,))),
    (rmx.DCN, (1000, 39, 16, 3, [400, 400, 400]), oc.DCN, dict(fc=(400, 400, 400), cross_depth=3)),
    (rmx.PNN, (1000, 39, 16, [400, 400, 400]), oc.PNN, dict(fc=(400, 400, 400))),
    (rmx.PNN, (1000, 5, 4, [7]), oc.PNN, dict(fc=(7,))),
]


@pytest.mark.parametrize("cls,args,t,kw", KINDS, ids=lambda x: getattr(x, "__name__", None))
def test_host_metadata_matches_oracle(cls, args, t, kw):
    """getMatsSize / mats length / initMats on a host-only model (no GPU touched)."""
    m = cls(*args)
    F, k = args[1], args[2]
    om = oc.make_model(t, F, k, **kw)
    assert m.getMatsSize() == oc.mats_sizes(om).tolist()
    assert m.matsLength() == oc.mats_len(om)
    assert np.array_equal(m.initMats(0x3A75), oc.init_mats(om, 0x3A75))
    assert m.getEmbeddingDim() == k and m.getInputDim() == args[0]
    assert m.getType() == rmx.RecModelType.BIAS_WEIGHT_EMBEDDING_MATS


def test_lr_metadata():
    m = rmx.LR(123)
    assert m.getMatsSize() == [] and m.getEmbeddingDim() == -1  # LR.scala:15, :19
    assert m.getType() == rmx.RecModelType.BIAS_WEIGHT


@pytest.mark.parametrize("bad", [
    lambda: rmx.DeepFM(10, 3, 4, []),              # "".split(",").map(_.toInt) throws (example/*:21)
    lambda: rmx.DeepFM(10, 0, 4, [8]),
    lambda: rmx.XDeepFM(10, 3, 16, [8], []),
    lambda: rmx.DCN(10, 3, 4, 0, [8]),              # (0 until 0).reduce throws (DCN.scala:17-19)
    lambda: rmx.PNN(10, 1, 4, [8]),
])
def test_model_create_rejects_what_the_reference_rejects(bad):
    with pytest.raises(rmx.RmxError):
        bad()


def test_unknown_model_type_is_type_error():
    h = ctypes.c_void_p()
    st = _lib.lib.rmx_model_create(None, 42, 10, 3, 4, None, 0, None, 0, 0, ctypes.byref(h))
    assert st == _lib.RMX_E_TYPE and b"unknown model type" in _lib.lib.rmx_last_error()


def test_sample_parser_libsvm_libffm():
    """data/SampleParser.scala:23-85: 1-based ids -> id - 1, label per line, row-major COO."""
    coo, fields, y = rmx.SampleParser.parse(["1 3:1 7:0.5", "0 1:1"], rmx.RecModelType.BIAS_WEIGHT)
    assert fields is None and y.tolist() == [1.0, 0.0]
    assert coo.getRowIndices().tolist() == [0, 0, 1] and coo.getColIndices().tolist() == [2, 6, 0]
    assert coo.getValues().tolist() == [1.0, 0.5, 1.0]
    coo, fields, y = rmx.SampleParser.parse(["1 0:5:1 2:9:1"], rmx.RecModelType.BIAS_WEIGHT_EMBEDDING_MATS_FIELD)
    assert fields.tolist() == [0, 2] and coo.getColIndices().tolist() == [4, 8]


def test_wgrad_slice_count_pinned_for_the_bench_shapes():
    """the 208 x 208 dW's slice count S sets the fp32 summation order of the weight gradient.
    It is a pure function of (rows, N, K, CU count) with constants fixed in the source, pinned here for
    DeepFM training at B = 65,536 on the 256-CU MI355X (layer 1 624 x 400: S = 40; the
    400 x 400 layers: S = 64); another CU count may pick another S (documented in include/rmx.h)."""
    from rmx import _lib
    S = _lib.lib.rmx_debug_wgrad_slices
    assert S(65536, 400, 624, 256) == 40
    assert S(65536, 624, 400, 256) == 40
    assert S(65536, 400, 400, 256) == 64
    assert S(32768, 400, 400, 256) == 64
    assert S(65536, 400, 400, 304) % 8 == 0
    assert S(0, 400, 400, 256) == _lib.RMX_E_INVALID
