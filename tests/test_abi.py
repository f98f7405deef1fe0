"""CPU tests of the C ABI: the library builds/loads and exports every symbol
include/d2mi.h declares (no compute calls without a GPU)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "d2mi.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(d2mi_\w+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    import torch  # noqa: F401  (binds the HIP runtime torch ships)
    from detectron2_tensorflow_amd import _C, _build
    _build.build()
    lib = ctypes.CDLL(_C.LIB_PATH)
    syms = declared_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    # and the ctypes table covers exactly the declared API
    assert sorted(_C.EXPORTED) == syms


def test_loader_sets_signatures_and_version():
    from detectron2_tensorflow_amd import _C
    from detectron2_tensorflow_amd import _build
    lib = _C.load()
    assert lib.d2mi_version() == 1
    assert _C.last_error() == ""
    # built from exactly this tree's sources (the loader refuses otherwise)
    assert lib.d2mi_source_hash().decode() == _build.source_hash()


def test_host_side_argument_errors_raise_without_gpu():
    """Argument validation happens on the host before any launch."""
    from detectron2_tensorflow_amd import _C
    lib = _C.load()
    rc = lib.d2mi_nms(None, None, None, 1, 10, 10, 1.5, None, None, None, 0, None)
    assert rc < 0 and "iou_threshold" in _C.last_error()
    rc = lib.d2mi_conv2d_nhwc(None, None, None, None, None, None, 1, 8, 8, 3, 16, 3, 3, 1, 1, 1,
                              0, None)
    assert rc < 0 and "multiple of 4" in _C.last_error()
