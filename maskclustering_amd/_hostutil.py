"""Host-side helpers of the drop-in modules."""
from __future__ import annotations

import contextlib
import gc


@contextlib.contextmanager
def no_gc():
    """Pause CPython's cyclic collector while the drop-ins build the reference's containers (tens
    of thousands of nodes, sets and tuples per scene): the allocations would otherwise trigger
    full-heap collections that cost more than the building itself.  Nested uses are safe; the
    collector is re-enabled only if it was enabled on entry.

    On the way out the objects made inside are moved to the oldest generation (``gc.freeze()`` then
    ``gc.unfreeze()``: two list splices, and the young generations' counts start again from zero), as
    a collection would move them after finding them alive, instead of letting the first allocation
    after ``gc.enable()`` scan the whole block's allocations in one young-generation pass (measured
    19 ms of a 66 ms C2 reference-API scene).  They are then looked at by full collections only, as
    any long-lived object is."""
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.freeze()
            gc.unfreeze()
            gc.enable()
