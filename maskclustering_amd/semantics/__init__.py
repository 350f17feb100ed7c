"""Drop-ins for the reference's ``semantics/`` scripts that run on the clustering's output."""
