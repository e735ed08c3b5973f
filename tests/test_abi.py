"""The C-ABI library builds for gfx950, loads on a CPU-only host and exports
every entry point include/yolomi.h declares (no compute calls without a GPU)."""
import ctypes
import re

from conftest import ROOT, PKG


def declared():
    txt = (ROOT / "include" / "yolomi.h").read_text()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(ym_\w+)\s*\(", txt, re.M)))


def test_header_declares_entry_points():
    names = declared()
    assert "ym_decode_nms" in names and "ym_last_error" in names


def test_library_exports_every_declared_symbol():
    so = PKG / "libyolomi.so"
    assert so.exists(), "build with `make -C yolo-scratch_amd/csrc` (or __graft_entry__.build())"
    L = ctypes.CDLL(str(so))
    missing = [n for n in declared() if not hasattr(L, n)]
    assert not missing, missing


def test_python_signatures_cover_header():
    import yolomi._lib as yl
    assert set(declared()) == set(yl.SIGNATURES), set(declared()) ^ set(yl.SIGNATURES)
    assert yl.lib().ym_version() >= 1


def test_integration_table_matches_header():
    """INTEGRATION.md's entry-point table names every declared entry point and nothing else."""
    doc = (ROOT / "INTEGRATION.md").read_text()
    table = doc[doc.index("| entry point(s) | reference call site |"):]
    table = table[:table.index("\n\n")]
    listed = set()
    for row in table.splitlines()[2:]:
        listed.update(re.findall(r"`(ym_\w+)`", row.split("|")[1]))
    names = set(declared())
    assert listed == names, {"undeclared": sorted(listed - names), "unlisted": sorted(names - listed)}
