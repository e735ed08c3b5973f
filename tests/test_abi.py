"""The C-ABI library builds for gfx950, loads on a CPU-only host and exports
every entry point include/yolomi.h and include/yolomi_experimental.h declare, and
nothing else (no compute calls without a GPU)."""
import ctypes
import re
import subprocess

from conftest import ROOT, PKG

HEADERS = ("yolomi.h", "yolomi_experimental.h")


def declared(header=None):
    names = set()
    for h in ([header] if header else HEADERS):
        txt = (ROOT / "include" / h).read_text()
        # the measurement library's block (libyolomi_exp.so only) is not part of the shipping ABI
        txt = re.sub(r"#ifdef YM_EXPERIMENTS.*?#endif", "", txt, flags=re.S)
        names |= set(re.findall(r"^\s*(?:const\s+|unsigned\s+)?[\w\s\*]+?\b(ym_\w+)\s*\(", txt, re.M))
    return sorted(names)


def test_header_declares_entry_points():
    names = declared()
    assert "ym_decode_nms" in names and "ym_last_error" in names and "ym_policy_generation" in names
    # the policy setters live in the experimental header only
    assert not [n for n in declared("yolomi.h") if "_set_" in n]


def test_library_exports_every_declared_symbol():
    so = PKG / "libyolomi.so"
    assert so.exists(), "build with `make -C yolo-scratch_amd/csrc` (or __graft_entry__.build())"
    L = ctypes.CDLL(str(so))
    missing = [n for n in declared() if not hasattr(L, n)]
    assert not missing, missing


def test_library_exports_nothing_undeclared():
    """The shipping library's dynamic ym_ symbols are exactly the declared ones: no experiment hook (ym_pipe_set_exp
    and the ablation instances are built into libyolomi_exp.so only) and no stray helper."""
    out = subprocess.run(["nm", "-D", "--defined-only", str(PKG / "libyolomi.so")], capture_output=True, text=True,
                         check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if ln.split() and ln.split()[-1].startswith("ym_")}
    assert exported == set(declared()), {"undeclared": sorted(exported - set(declared())),
                                         "missing": sorted(set(declared()) - exported)}


def test_python_signatures_cover_header():
    import yolomi._lib as yl
    assert set(declared()) == set(yl.SIGNATURES), set(declared()) ^ set(yl.SIGNATURES)
    assert yl.lib().ym_version() >= 1
    g0 = yl.lib().ym_policy_generation()
    prev = yl.lib().ym_conv_set_halo(-1)
    yl.lib().ym_conv_set_halo(prev)
    assert yl.lib().ym_policy_generation() == g0 + 2


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
