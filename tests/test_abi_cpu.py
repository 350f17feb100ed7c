"""CPU-side checks of the boundary: the C-ABI library loads, exports exactly the
symbols include/mcgraph.h declares, and the Python binding covers them.
No compute call is made (no GPU here)."""
import ctypes
import os
import re

from conftest import REPO


def declared_functions():
    src = open(os.path.join(REPO, "include", "mcgraph.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mc_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_api():
    names = declared_functions()
    assert "mc_graph_build" in names and "mc_cluster_run" in names and len(names) >= 30


def test_library_exports_every_declared_symbol():
    from maskclustering_amd import _native
    L = ctypes.CDLL(_native.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(L, n)]
    assert not missing, missing


def test_binding_covers_header():
    from maskclustering_amd import _native
    assert sorted(_native.EXPORTED) == declared_functions()
    _native.load()


def test_product_does_not_import_oracle():
    pkg = os.path.join(REPO, "maskclustering_amd")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".inl", ".hpp", ".cpp", ".h")):
                txt = open(os.path.join(root, f)).read()
                assert "from oracle" not in txt and "import oracle" not in txt and "liboracle" not in txt, f
