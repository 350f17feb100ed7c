"""MI355X-native view-consensus graph path of MaskClustering."""
import os

# S1's denoise runs its size classes side by side on their own HIP streams; HIP maps streams onto
# GPU_MAX_HW_QUEUES hardware queues (default 4), and two classes that share a queue run one after
# the other.  Ask for 8 unless more are set (effective before the process's first HIP call).
try:
    if int(os.environ.get("GPU_MAX_HW_QUEUES") or 4) < 8:
        os.environ["GPU_MAX_HW_QUEUES"] = "8"
except ValueError:
    pass
