"""Route the reference's hot-path modules to the MI355X drop-ins, so that the
reference's ``main.py`` / ``run.py`` run unchanged on the device path:

    graph.construction          -> maskclustering_amd.graph.construction
    graph.iterative_clustering  -> maskclustering_amd.graph.iterative_clustering
    graph.node                  -> maskclustering_amd.graph.node
    utils.mask_backprojection   -> maskclustering_amd.utils.mask_backprojection
    utils.post_process          -> maskclustering_amd.utils.post_process

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
    return done
