"""Which kernels' machine code differs between two builds of mc_api.hip (gfx950 device assembly from
`hipcc -S --offload-device-only`).  The S1 class kernels have shown build-dependent results (DESIGN.md
§4, round-4 investigation), so a source change is validated against the GPU runs of the build whose
code it reproduces: an unchanged kernel list means the tested machine code ships.

    python scripts/isa_diff.py <git-rev> [kernel-substring]   # <git-rev>'s source against the working tree
"""
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-S", "--offload-device-only"]


def device_asm(src_dir, out):
    subprocess.check_call(["/opt/rocm/bin/hipcc", *FLAGS, os.path.join(src_dir, "mc_api.hip"), "-o", out],
                          stderr=subprocess.DEVNULL)
    s = open(out).read()
    funcs = {}
    for m in re.finditer(r"^(_ZN2mc[^\s:]*):", s, re.M):
        end = s.find(".Lfunc_end", m.end())
        funcs[m.group(1)] = [l for l in s[m.end():end].splitlines()
                             if l.strip() and not l.strip().startswith((".loc", ";", ".Ltmp", ".cfi"))]
    return funcs


def main():
    rev = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else "k_bp"
    with tempfile.TemporaryDirectory() as tmp:
        wt = os.path.join(tmp, "wt")
        subprocess.check_call(["git", "-C", REPO, "worktree", "add", "-f", "-q", wt, rev])
        try:
            a = device_asm(os.path.join(wt, "maskclustering_amd", "csrc"), os.path.join(tmp, "a.s"))
        finally:
            subprocess.call(["git", "-C", REPO, "worktree", "remove", "--force", wt])
        b = device_asm(os.path.join(REPO, "maskclustering_amd", "csrc"), os.path.join(tmp, "b.s"))
    names = sorted(k for k in set(a) | set(b) if sub in k)
    diff = [k for k in names if a.get(k) != b.get(k)]
    for k in diff:
        print("differs:", k, len(a.get(k, [])), len(b.get(k, [])))
    print(f"{len(names) - len(diff)} of {len(names)} kernels matching '{sub}' identical")


if __name__ == "__main__":
    main()
