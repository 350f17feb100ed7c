"""MI355X-native view-consensus graph path of MaskClustering."""
import os
import sys
import warnings

# S1's denoise runs its size classes side by side on their own HIP streams; HIP maps streams onto
# GPU_MAX_HW_QUEUES hardware queues (default 4), and two classes that share a queue run one after
# the other (docs/experiments.md: C3 E2E 224 ms with 8 queues against 415 ms with 4).  Ask for 8 unless
# more are set.  HIP reads the variable once, when the process first initialises the runtime, so
# the setting does nothing if that already happened: warn then (torch.cuda initialised before this
# import is the case that can be seen from here).
try:
    _queues = int(os.environ.get("GPU_MAX_HW_QUEUES") or 4)
except ValueError:
    _queues = None
if _queues is not None and _queues < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"
    _torch = sys.modules.get("torch")
    if _torch is not None and getattr(getattr(_torch, "cuda", None), "is_initialized", lambda: False)():
        warnings.warn("maskclustering_amd: the HIP runtime was initialised before this import, so "
                      f"GPU_MAX_HW_QUEUES={_queues} stays in effect and S1's denoise classes share hardware "
                      "queues (slower, results unchanged); import maskclustering_amd first or export "
                      "GPU_MAX_HW_QUEUES=8", RuntimeWarning, stacklevel=2)
