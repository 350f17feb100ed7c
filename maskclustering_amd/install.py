"""Route the reference's hot-path modules to the MI355X drop-ins, so that the
reference's ``main.py`` / ``run.py`` run unchanged on the device path:

    graph.construction          -> maskclustering_amd.graph.construction
    graph.iterative_clustering  -> maskclustering_amd.graph.iterative_clustering
    graph.node                  -> maskclustering_amd.graph.node
    utils.mask_backprojection   -> maskclustering_amd.utils.mask_backprojection
    utils.post_process          -> maskclustering_amd.utils.post_process
    semantics.open-voc_query    -> maskclustering_amd/semantics/open_voc_query.py
                                   (run.py:102 runs it with ``python -m``: a meta-path finder)

Every other reference module (utils.config, dataset.*, ...)
is imported from the reference as usual.  ``integration/sitecustomize.py`` calls
``install()`` at interpreter start-up.
"""
from __future__ import annotations

import importlib
import sys

ALIASES = {
    "graph.construction": "maskclustering_amd.graph.construction",
    "graph.iterative_clustering": "maskclustering_amd.graph.iterative_clustering",
    "graph.node": "maskclustering_amd.graph.node",
    "utils.mask_backprojection": "maskclustering_amd.utils.mask_backprojection",
    "utils.post_process": "maskclustering_amd.utils.post_process",
}

# scripts the reference runs with ``python -m`` (run.py:102): runpy needs a spec under the
# requested name, so these resolve through a finder to the drop-in's source file instead of a
# sys.modules alias
SCRIPTS = {
    "semantics.open-voc_query": "maskclustering_amd.semantics.open_voc_query",
}


class _ScriptFinder:
    """Meta-path finder: a SCRIPTS name -> a spec that loads the drop-in's file under that name."""

    @staticmethod
    def find_spec(fullname, path=None, target=None):
        if fullname not in SCRIPTS:
            return None
        import importlib.util
        origin = importlib.util.find_spec(SCRIPTS[fullname]).origin
        return importlib.util.spec_from_file_location(fullname, origin)


def install() -> dict:
    """Register the aliases in sys.modules (and on the reference's parent packages when they
    are importable).  Returns {alias: module}."""
    done = {}
    for name, target in ALIASES.items():
        mod = importlib.import_module(target)
        sys.modules[name] = mod
        parent, child = name.rsplit(".", 1)
        try:
            setattr(importlib.import_module(parent), child, mod)
        except ImportError:
            pass
        done[name] = mod
    if not any(isinstance(f, _ScriptFinder) for f in sys.meta_path):
        sys.meta_path.insert(0, _ScriptFinder())
    return done
