"""Drop-in modules for the reference's ``utils/`` package (the hot-path subset)."""
