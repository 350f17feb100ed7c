"""Host-side helpers of the drop-in modules."""
from __future__ import annotations

import contextlib
import gc


@contextlib.contextmanager
def no_gc():
    """Pause CPython's cyclic collector while the drop-ins build the reference's containers (tens
    of thousands of nodes, sets and tuples per scene): the allocations would otherwise trigger
    full-heap collections that cost more than the building itself.  Nested uses are safe; the
    collector is re-enabled only if it was enabled on entry."""
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()
