"""The C-ABI library loads and exports every symbol include/vina_gpu.h declares
(no compute calls: CPU-only check)."""
import ctypes

import vgpu


def test_header_symbols_exported():
    vgpu.build()
    L = ctypes.CDLL(vgpu.LIB)
    syms = vgpu.header_symbols()
    assert len(syms) >= 10
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing


def test_config_struct_layout_matches_header():
    from vgconfig import CConfig
    # 9 doubles + 4 + 4 + 8 scalars + 4 + 4 ... computed from the header field list
    assert ctypes.sizeof(CConfig) == 8 * (3 + 4 + 4 + 2 + 1 + 4 + 4 + 9 + 3) + 4 * 8
