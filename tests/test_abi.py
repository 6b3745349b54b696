"""The C ABI: libhga.so loads (no GPU needed) and exports every symbol include/hga.h declares."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "hga.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(hga_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_api():
    syms = declared_symbols()
    for must in ("hga_count_begin", "hga_count_add", "hga_count_run", "hga_count_spec_hist",
                 "hga_count_select", "hga_lookup_load", "hga_lookup_run", "hga_lookup_fetch"):
        assert must in syms


def test_library_exports_every_declared_symbol(hga_mod):
    lib = hga_mod.lib()
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert missing == []
    # the binding table covers the header exactly
    assert sorted(hga_mod.HGA_SYMBOLS) == declared_symbols()


def test_no_compute_without_device(hga_mod):
    # On a box without a GPU the library loads and reports errors instead of crashing.
    lib = hga_mod.lib()
    assert lib.hga_version().decode().startswith("hga-mi355x")
    n = ctypes.c_int(-1)
    st = lib.hga_device_count(ctypes.byref(n))
    assert st in (0, 2)
    if st != 0 or n.value == 0:
        h = ctypes.c_void_p()
        assert lib.hga_ctx_create(ctypes.byref(h), 0) != 0
        assert lib.hga_last_error().decode() != ""
    # a null context is rejected, not dereferenced
    assert lib.hga_count_run(None, 2) == 1


def test_library_is_gfx950_code_object():
    so = os.path.join(ROOT, "hybrid-genome-assembler_amd", "lib", "libhga.so")
    data = open(so, "rb").read()
    assert b"gfx950" in data
