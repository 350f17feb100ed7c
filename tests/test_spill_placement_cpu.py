"""The gfx950 code of the S1 kernels (release and the MC_DBG_CHECK diagnostics build) holds no VGPR
spill store placed where EXEC can be partial (scripts/spill_exec_check.py; docs/experiments.md: the round-4
diagnostics build lost the inactive lanes' values of such spills).  Cross-compiles on the CPU."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
@pytest.mark.parametrize("defs", [[], ["-DMC_DBG_CHECK=1"]], ids=["release", "diagnostics"])
def test_no_spill_stores_before_exec_restore(defs):
    r = subprocess.run([sys.executable, os.path.join(REPO, "scripts", "spill_exec_check.py"), "--build", *defs, "k_"],
                       cwd=REPO, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]


def test_checker_flags_the_failure_pattern(tmp_path):
    """The checker itself: a spill store in an execz-branch target before the block's EXEC restore is
    flagged; the same store after the restore is not."""
    sys.path.insert(0, os.path.join(REPO, "scripts"))
    import spill_exec_check as c
    bad = """  s_and_saveexec_b64 s[4:5], vcc
  s_cbranch_execz .LBB0_2
  v_add_u32 v1, v1, v2
.LBB0_2:
  scratch_store_dwordx4 off, v[48:51], off offset:176 ; 16-byte Folded Spill
  s_or_b64 exec, exec, s[4:5]
""".splitlines()
    good = """  s_and_saveexec_b64 s[4:5], vcc
  s_cbranch_execz .LBB0_2
  v_add_u32 v1, v1, v2
.LBB0_2:
  s_or_b64 exec, exec, s[4:5]
  scratch_store_dwordx4 off, v[48:51], off offset:176 ; 16-byte Folded Spill
""".splitlines()
    assert len(c.check(bad)[0]) == 1
    assert c.check(good) == ([], [])
