"""div_rn (maskclustering_amd/csrc/mc_bp_kernels.inl): S1's per-pixel divisions (the unprojection by
fx / fy, the voxel index by the voxel size) are a reciprocal multiply and two FMAs whose result must be
the IEEE quotient bit for bit, since the voxel partition and the voxel means are Open3D's exact
arithmetic (oracle/s1_oracle.c divides).  The identity (Markstein) is checked here on
2*10^7 operand pairs of those ranges, near-integer quotients included, with the host's fma; the GPU
parity tests check the kernels' outputs against the oracle's divisions."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_reciprocal_fma_division_equals_ieee_quotient(tmp_path):
    exe = tmp_path / "div_check"
    subprocess.check_call(["gcc", "-O2", "-o", str(exe), os.path.join(REPO, "scripts", "div_check.c"), "-lm"])
    r = subprocess.run([str(exe), "20000000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "bad=0" in r.stdout, r.stdout
