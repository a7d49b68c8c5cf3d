"""CPU: the C-ABI library loads and exports every entry point include/*.h declares
(no compute calls -- there is no GPU here)."""
import ctypes
import glob
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        text = open(h).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        names |= set(re.findall(r"\b(ik_[a-z0-9_]+)\s*\(", text))
    return names


def test_header_declares_the_reference_surface():
    names = declared_symbols()
    for n in ("ik_decode", "ik_resize", "ik_encode", "ik_transform", "ik_pipeline_run",
              "ik_last_error", "ik_image_free", "ik_buf_free"):
        assert n in names


def test_library_exports_every_declared_symbol():
    from imagekit import _lib
    lib = _lib.load()  # must load without a GPU
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if l.strip()}
    missing = declared_symbols() - exported
    assert not missing, f"declared but not exported: {sorted(missing)}"
    for n in declared_symbols():
        assert isinstance(getattr(lib, n), ctypes._CFuncPtr)


def test_python_binding_covers_header():
    from imagekit import _lib
    bound = {n for n, _, _ in _lib.SIGNATURES}
    assert declared_symbols() <= bound | {"ik_version"}


def test_version_string_without_gpu():
    from imagekit import _lib
    assert b"gfx950" in _lib.load().ik_version()
