"""Start-up hook: with this directory and the repository root on PYTHONPATH,
every Python process (the reference's run.py and the main.py subprocesses it
starts) imports the MI355X drop-ins under the reference's module names.
Set MASKCLUSTERING_AMD=0 to disable.  See INTEGRATION.md."""
import os
import sys

if os.environ.get("MASKCLUSTERING_AMD", "1") != "0":
    try:
        from maskclustering_amd.install import install

        install()
    except Exception as e:  # the reference must still start; the first device call reports the cause
        print(f"[maskclustering_amd] drop-in modules not installed: {e}", file=sys.stderr)
