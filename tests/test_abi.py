"""C-ABI surface checks (CPU only: load + symbol export, no compute calls)."""
import ctypes
import glob
import os
import re

import pytest

import native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    syms = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        text = open(h).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        syms.update(re.findall(r"\b(ppox_\w+)\s*\(", text))
    return syms


def test_header_declares_entry_points():
    syms = declared_symbols()
    assert {"ppox_version", "ppox_last_error", "ppox_gae", "ppox_gae_dual"} <= syms


def test_library_exports_every_declared_symbol():
    if not os.path.exists(native.LIB_PATH):
        pytest.skip("libppox.so not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(native.LIB_PATH)
    missing = [s for s in sorted(declared_symbols()) if not hasattr(lib, s)]
    assert not missing, missing


def test_python_binding_covers_header():
    bound = set(native.SIGNATURES) | set(native._RESTYPES)
    assert declared_symbols() == bound


def test_version_and_error_channel():
    if not os.path.exists(native.LIB_PATH):
        pytest.skip("libppox.so not built")
    assert native.version().startswith("ppox")
    lib = native.load()
    assert isinstance(lib.ppox_last_error(), bytes)


def test_argument_validation_without_gpu():
    """Argument checks run before any HIP call, so they are testable on CPU."""
    if not os.path.exists(native.LIB_PATH):
        pytest.skip("libppox.so not built")
    lib = native.load()
    rc = lib.ppox_gae(None, None, None, None, None, 0, 4, 0.99, 0.95, None, None, None)
    assert rc == -1000
    assert b"must be positive" in lib.ppox_last_error()


def test_icm_segment_layout_matches_module():
    """icm.supported(): the K9 kernels' parameter segment (ppox_icm_param_elems, include/ppox.h)
    is the module's parameters after state_encoder[0].weight, contiguous in module order."""
    if not os.path.exists(native.LIB_PATH):
        pytest.skip("libppox.so not built")
    import torch

    import icm
    from env import Box, Discrete
    from models import FlatParams, IntrinsicCuriosityModule
    from util import ActionConverter
    K = 2048
    for A in (1, 4, 18, 32):
        m = IntrinsicCuriosityModule(K, ActionConverter(Discrete(A)), 32)
        flat = FlatParams(m, "cpu")
        assert flat.n == 32 * K + native.icm_param_elems(A)
        assert icm.supported(m, flat, (K,), torch.uint8)
        assert not icm.supported(m, flat, (K,), torch.float32)
    assert native.icm_param_elems(33) == -1
    m = IntrinsicCuriosityModule(K, ActionConverter(Discrete(40)), 32)
    assert not icm.supported(m, FlatParams(m, "cpu"), (K,), torch.uint8)
    m = IntrinsicCuriosityModule(K, ActionConverter(Discrete(4)), 64)
    assert not icm.supported(m, FlatParams(m, "cpu"), (K,), torch.uint8)
    m = IntrinsicCuriosityModule(K, ActionConverter(Box((3,))), 32)
    assert not icm.supported(m, FlatParams(m, "cpu"), (K,), torch.uint8)
    m = IntrinsicCuriosityModule(2000, ActionConverter(Discrete(4)), 32)
    assert not icm.supported(m, FlatParams(m, "cpu"), (2000,), torch.uint8)
    assert native.icm_w1_pack_elems(2000) == -1 and native.icm_w1_pack_elems(K) == 2 * 32 * K + 64
    assert native.icm_encode_workspace_bytes(2048, 4 * 84 * 84) > 0
