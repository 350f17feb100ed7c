"""Find VGPR spill stores that the compiler placed where EXEC can be partial ("the
diagnostics-build failure").

On gfx9 a `scratch_store` writes only the lanes active in EXEC.  The round-4 diagnostics build of the
denoise classes lost values this way: the register allocator put the spills of values live across a
call (`mn[]` among them) into the exit block of a per-thread loop, *before* the `s_or_b64 exec, exec,
s[..]` that re-enables the lanes which had left the loop, so the stores ran with EXEC = the lanes still
in the loop (none, at that exit); the reloads later returned stale scratch.

This check flags a `... Folded Spill` store (and any `scratch_store` of a spill slot) that sits in a
block entered by `s_cbranch_execz` (a loop or if exit whose EXEC restore has not run yet) before that
block's first `s_or_b64 exec, exec, ...`, and a spill store inside a block that starts after
`s_and_saveexec` / `s_andn2_b64 exec` with no restore between.  The second pattern is legitimate only
when the spilled value is dead in the inactive lanes, which the assembly alone cannot tell, so it is
reported as "divergent" (informational); the first is the failure pattern and fails the check.

    python scripts/spill_exec_check.py [asm.s | --build [-Dflags...]] [kernel-substring]
"""
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-S", "--offload-device-only"]


def device_asm(defs, out):
    subprocess.check_call(["/opt/rocm/bin/hipcc", *FLAGS, *defs,
                           os.path.join(REPO, "maskclustering_amd", "csrc", "mc_api.hip"), "-o", out],
                          stderr=subprocess.DEVNULL)
    return open(out).read()


def functions(asm):
    for m in re.finditer(r"^(_ZN2mc[^\s:]*):", asm, re.M):
        end = asm.find(".Lfunc_end", m.end())
        yield m.group(1), asm[m.end():end].splitlines()


def check(lines):
    """-> (bad, divergent): lists of (line number, text) of spill stores after an execz-branch target
    before its EXEC restore, and of spill stores under a saveexec mask."""
    execz_targets = set(re.findall(r"s_cbranch_execz (\.\w+)", "\n".join(lines)))
    bad, div = [], []
    state = "full"  # "exit": in an execz target block before its restore; "masked": after saveexec
    for i, raw in enumerate(lines):
        l = raw.strip()
        if not l or l.startswith((".loc", ";", ".Ltmp", ".cfi")):
            continue
        lab = re.match(r"^(\.\w+):", l)
        if lab:
            state = "exit" if lab.group(1) in execz_targets else ("masked" if state == "masked" else state)
            if state == "exit":
                continue
            continue
        if re.match(r"s_or_b64 exec, exec, ", l) or re.match(r"s_mov_b64 exec, -1", l):
            state = "full"
            continue
        if re.match(r"s_(and|or|xor)_saveexec_b64 |s_andn2_b64 exec, exec|s_and_b64 exec, exec|s_mov_b64 exec, s", l):
            state = "masked" if state == "full" else state
        spill = "Folded Spill" in raw or (l.startswith("scratch_store") and "Spill" in raw)
        if spill and state == "exit":
            bad.append((i, l))
        elif spill and state == "masked":
            div.append((i, l))
    return bad, div


def main():
    args = sys.argv[1:]
    sub = "k_bp"
    if args and args[0] == "--build":
        defs = [a for a in args[1:] if a.startswith("-D")]
        rest = [a for a in args[1:] if not a.startswith("-D")]
        if rest:
            sub = rest[0]
        with tempfile.TemporaryDirectory() as tmp:
            asm = device_asm(defs, os.path.join(tmp, "a.s"))
    else:
        asm = open(args[0]).read()
        if len(args) > 1:
            sub = args[1]
    nbad = 0
    for name, lines in functions(asm):
        if sub not in name:
            continue
        bad, div = check(lines)
        if bad or div:
            print(f"{name[:90]}: {len(bad)} spill stores before an exec restore, {len(div)} under a saveexec mask")
            for i, l in bad[:6]:
                print(f"    line {i}: {l}")
        nbad += len(bad)
    print(f"{nbad} spill stores placed before their block's EXEC restore")
    sys.exit(1 if nbad else 0)


if __name__ == "__main__":
    main()
