"""CPU checks of the drop-in boundary: libasr_amd.so loads and exports every
symbol include/asr_amd.h declares; no compute call is made (no GPU here)."""
import re
import subprocess

from conftest import PKG, ROOT, asr

HEADER = ROOT / "include" / "asr_amd.h"


def declared():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(asr_[a-z0-9_]+)\s*\(", text)))


def test_header_matches_python_mirror():
    assert declared() == sorted(asr.EXPORTS)


def test_library_exports_every_declared_symbol():
    lib = asr.lib()
    for name in declared():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", str(asr.LIB_PATH)], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (asr_[a-z0-9_]+)$", out, flags=re.M))
    assert set(declared()) <= exported


def test_status_strings_and_argument_errors():
    assert asr.status_string(asr.ASR_ERR_BEAM_OVERFLOW).startswith("beam overflow")
    assert asr.status_string(asr.ASR_OK) == "ok"
    L = asr.lib()
    # argument validation happens before any HIP call
    assert L.asr_linear_fwd(None, None, None, None, 1, 1, 1, 0, None) == asr.ASR_ERR_ARG
    assert L.asr_ctc_decode(None, None, 1, 1, 0, None) == asr.ASR_ERR_ARG
    assert L.asr_ctc_get_best(None, None, 0, None, None) == asr.ASR_ERR_ARG


def test_gfx950_code_object():
    """The shared library carries a gfx950 code object (and only gfx950)."""
    out = subprocess.run(["strings", str(asr.LIB_PATH)], capture_output=True, text=True).stdout
    assert "amdgcn-amd-amdhsa--gfx950" in out
    assert "gfx942" not in out and "sm_" not in out.split("amdgcn")[0][-100:]
