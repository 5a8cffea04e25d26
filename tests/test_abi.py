"""The drop-in boundary without a GPU: libbrickrec loads, exports every entry point that
include/brickrec.h declares, its ctypes mirror has the header's struct layout, and the
product path fails loudly (no CPU fallback) when there is no device."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "brickrec.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^[A-Za-z_][\w\s\*]*?\b(bb_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_the_boundary():
    names = _declared()
    for n in ("bb_create", "bb_upload_items", "bb_search", "bb_finalize", "bb_eval_mask", "bb_destroy"):
        assert n in names


def test_library_exports_every_declared_symbol():
    from brickrec import _lib as L
    lib = L.load()
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing
    assert set(_declared()) == set(L.EXPORTS)
    assert lib.bb_abi_version() == L.ABI_VERSION == 2


def test_exports_are_c_linkage():
    from brickrec import _lib as L
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    syms = {line.split()[-1] for line in out.splitlines() if line.strip()}
    for n in _declared():
        assert n in syms, f"{n} not exported with C linkage"


def _c_layout(structs):
    """Compile a probe against the header with gcc (plain C) and read sizeof/offsetof."""
    lines = ["#include <stdio.h>", "#include <stddef.h>", f'#include "{HEADER}"', "int main(void){"]
    for sname, fields in structs.items():
        lines.append(f'printf("{sname} %zu\\n", sizeof({sname}));')
        for f in fields:
            lines.append(f'printf("{sname}.{f} %zu\\n", offsetof({sname}, {f}));')
    lines.append("return 0;}")
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        c, exe = os.path.join(d, "p.c"), os.path.join(d, "p")
        open(c, "w").write("\n".join(lines))
        subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", c, "-o", exe], check=True)
        out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout
    return {k: int(v) for k, v in (l.split() for l in out.splitlines())}


def test_ctypes_mirror_matches_header_layout():
    from brickrec import _lib as L
    structs = {n: [f[0] for f in getattr(L, n)._fields_]
               for n in ("bb_desc", "bb_predicate", "bb_query", "bb_result", "bb_profile")}
    lay = _c_layout(structs)
    for n, fields in structs.items():
        cls = getattr(L, n)
        assert C.sizeof(cls) == lay[n], n
        for f in fields:
            assert getattr(cls, f).offset == lay[f"{n}.{f}"], f"{n}.{f}"


def test_key_lens_needs_no_device():
    from brickrec import _lib as L
    lib = L.load()
    q = L.bb_query()
    sides, kint = C.c_int32(), C.c_int32()
    for mode, k, ks, want in ((L.BB_MODE_SEMANTIC, 50, 0, (1, 50)), (L.BB_MODE_SIMILAR, 50, 0, (1, 51)),
                              (L.BB_MODE_CF, 20, 0, (1, 20)), (L.BB_MODE_HYBRID, 10, 0, (2, 21)),
                              (L.BB_MODE_HYBRID, 10, 30, (2, 31))):
        q.mode, q.k, q.k_side, q.B = mode, k, ks, 4
        assert lib.bb_key_lens(C.byref(q), C.byref(sides), C.byref(kint)) == L.BB_OK
        assert (sides.value, kint.value) == want
    q.mode, q.k = L.BB_MODE_SIMILAR, 512     # k+1 exceeds the internal list limit
    assert lib.bb_key_lens(C.byref(q), C.byref(sides), C.byref(kint)) == L.BB_E_ARG
    assert lib.bb_last_error()


def test_product_path_fails_loudly_without_device():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a device is present")
    import brickrec
    with pytest.raises(brickrec.BrickrecError):
        brickrec.ItemIndex()


def test_missing_library_is_an_error(monkeypatch):
    from brickrec import _lib as L
    monkeypatch.setattr(L, "LIB_PATH", "/nonexistent/libbrickrec.so")
    monkeypatch.setattr(L, "_lib", None)
    with pytest.raises(L.BrickrecError):
        L.load()


def test_stale_and_foreign_handles_are_errors():
    """every entry point checks its handle against the library's live set
    before touching it — a pointer the library never made (or one it already destroyed: the
    r04 segfault class) returns BB_E_ARG with a message instead of crashing the process.  No
    device is needed: the check comes before any HIP call."""
    from brickrec import _lib as L
    lib = L.load()
    junk = C.create_string_buffer(b"\xab" * 4096)       # bytes that are no bb_index
    gone = C.create_string_buffer(4096)
    gone_addr = C.addressof(gone)
    del gone                                            # freed memory, as after bb_destroy
    q = L.bb_query(mode=L.BB_MODE_SEMANTIC, B=1, k=10, where=L.BB_DEVICE)
    res = L.bb_result(where=L.BB_DEVICE)
    prof = L.bb_profile()
    n, d = C.c_int64(), C.c_int32()
    for addr in (C.addressof(junk), gone_addr):
        h = C.c_void_p(addr)
        calls = {
            "bb_search": lambda: lib.bb_search(h, C.byref(q), C.byref(res)),
            "bb_finalize": lambda: lib.bb_finalize(h, C.byref(q), h, h, 1, C.byref(res)),
            "bb_info": lambda: lib.bb_info(h, C.byref(n), C.byref(d), None, None),
            "bb_set_option": lambda: lib.bb_set_option(h, L.BB_OPT_STREAM, 0),
            "bb_set_profiling": lambda: lib.bb_set_profiling(h, 1),
            "bb_get_profile": lambda: lib.bb_get_profile(h, C.byref(prof)),
            "bb_get_rows": lambda: lib.bb_get_rows(h, h, 1, h, L.BB_HOST),
            "bb_upload_cf": lambda: lib.bb_upload_cf(h, h, 4, L.BB_F32, None),
            "bb_create_view": lambda: lib.bb_create_view(h, C.byref(C.c_void_p())),
            "bb_plan_create": lambda: lib.bb_plan_create(h, C.byref(q), C.byref(res), C.byref(C.c_void_p())),
            "bb_plan_launch": lambda: lib.bb_plan_launch(h),
            "bb_plan_destroy": lambda: lib.bb_plan_destroy(h),
            "bb_destroy": lambda: lib.bb_destroy(h),
        }
        for name, call in calls.items():
            assert call() == L.BB_E_ARG, name
            assert b"stale or foreign" in lib.bb_last_error(), name
    # NULL stays "nothing to destroy"
    assert lib.bb_destroy(None) == L.BB_OK and lib.bb_plan_destroy(None) == L.BB_OK


def test_dual_scan_refuses_24bit_dma_overflow():
    """scan4's LDS-DMA source offsets are 24-bit, so the hybrid dual list
    scan's launcher refuses an item row stride >= 2^23 (BB_E_ARG, the rule named in
    bb_last_error) before any launch instead of faulting; bb_search maps the same check to
    BB_E_ARG.  Runs the launcher's own rule set (scan4_dual_args_ok) on the CPU."""
    from brickrec import _lib as L
    lib = L.load()
    assert lib.bb_check_dual_scan_args(384) == L.BB_OK            # configs[2]'s stride
    assert lib.bb_check_dual_scan_args((1 << 23) - 1) == L.BB_OK
    for bad in (1 << 23, (1 << 23) + 384, 1 << 40, 0, -8):
        assert lib.bb_check_dual_scan_args(bad) == L.BB_E_ARG, bad
        assert b"24-bit" in lib.bb_last_error()
