"""Drop-in modules for the reference's ``graph/`` package (graph/construction.py,
graph/iterative_clustering.py, graph/node.py)."""
