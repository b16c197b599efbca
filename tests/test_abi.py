"""C-ABI boundary: the library loads (no GPU needed) and exports every symbol
include/gpuflow.h declares; struct sizes match the reference layouts."""
import ctypes as C
import os
import re

from cilium_amd import _lib
from cilium_amd._lib import lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "gpuflow.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(gf_[a-z0-9_]+)\s*\(", txt)))


def test_header_matches_binding_list():
    assert header_symbols() == sorted(_lib.EXPORTED)


def test_library_exports_every_declared_symbol():
    for s in header_symbols():
        assert hasattr(lib, s), s


def test_struct_sizes():
    assert C.sizeof(_lib.gf_l4_allow) == 8
    assert C.sizeof(_lib.gf_pkt_cols) == 8 + 15 * 8
    assert C.sizeof(_lib.gf_xdp_cfg) == 20


def test_version_and_device_count_without_gpu():
    assert b"gfx950" in lib.gf_version()
    assert lib.gf_device_count() >= 0
