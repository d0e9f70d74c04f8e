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


def _c_layout(tmp_path, struct, fields):
    """sizeof / offsetof of a header struct, from a C compiler (gcc)."""
    import os
    import subprocess
    inc = os.path.join(os.path.dirname(vgpu.HEADER))
    body = "".join('printf("%%zu\\n", offsetof(%s, %s));' % (struct, f) for f in fields)
    src = tmp_path / "lay.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "vina_gpu.h"\n'
                   'int main(void){printf("%%zu\\n", sizeof(%s));%s return 0;}\n' % (struct, body))
    exe = tmp_path / "lay"
    subprocess.check_call(["gcc", "-I", inc, "-o", str(exe), str(src)])
    out = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    return out[0], out[1:]


def test_config_struct_layout_matches_header(tmp_path):
    """vgconfig.CConfig (the Python binding, also the oracle's orc_config) is
    field-for-field vg_config: same size and offsets (the oracle-only ints sit
    in vg_config's reserved slots)."""
    from vgconfig import CConfig
    names = [f for f, _ in CConfig._fields_]
    hdr = {"use_threads": "reserved0", "vnc_prep": "reserved1"}
    size, offs = _c_layout(tmp_path, "vg_config", [hdr.get(f, f).split("[")[0] for f in names])
    assert ctypes.sizeof(CConfig) == size
    assert [getattr(CConfig, f).offset for f in names] == offs


def test_stats_struct_layout_matches_header(tmp_path):
    names = [f for f, _ in vgpu.Stats._fields_]
    size, offs = _c_layout(tmp_path, "vg_stats", names)
    assert ctypes.sizeof(vgpu.Stats) == size
    assert [getattr(vgpu.Stats, f).offset for f in names] == offs
