#!/usr/bin/env python3
"""Find vector writes that run before a divergent region's EXEC restore (gfx950 code objects).

    python3 tools/exec_join_check.py [lib.so ...] [--verbose]

A divergent `if` compiles to `s_and_saveexec_b64 sX, cond; s_cbranch_execz JOIN; <then>;
JOIN: s_or_b64 exec, exec, sX`. The join block must restore EXEC before any vector
instruction: an instruction placed between JOIN and the restore runs only for the lanes
that took the branch (and for none when the branch was skipped). The same holds for the
exit of a divergent loop (the fall-through after `s_cbranch_execnz HEADER`).

ROCm 7.2's AMDGPU greedy register allocator can put such instructions there: when a live
range is split at the top of a join block whose EXEC restore is preceded by SGPR copies
(left by PHI elimination), the split's COPY goes to the block top, before the restore,
because only a *leading* run of EXEC-writing instructions counts as the block's prologue.
The copy then moves the value for the branch's lanes only; every other lane keeps the
register's stale contents. This is what broke C1 under some code layouts:
in start_sample's last Philox draw, the copies that carry the Rng buffer (r0, r2) out of
`if ((d & 3) == 0) philox_block(..)` ran for the lanes that called only, so the other lanes
left with r0 = d and r2 = a dead float, and their first in_unit_sphere() draw was wrong.

This tool reads the library's offload bundles (tools/kernel_resources.py), disassembles
each gfx950 code object with llvm-objdump, and lists every vector-register write between
an `s_cbranch_execz` target (or the fall-through of an `s_cbranch_execnz`) and the next
EXEC write. tests/test_exec_join.py runs it on the product library, so a build that the
allocator miscompiles this way fails in the CPU suite before it reaches a GPU.
"""
from __future__ import annotations

import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from kernel_resources import DEFAULT_LIB, bundles, readable  # noqa: E402

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
LINE = re.compile(r"^\t(\S+)\s*(.*?)\s*// ([0-9A-F]{12}):")
FUNC = re.compile(r"^([0-9a-f]{16}) <(.+)>:$")
# first operand of a vector instruction that writes VGPRs / AGPRs
VDST = re.compile(r"^(v\d+|v\[\d+:\d+\]|a\d+|a\[\d+:\d+\])\b")
LOADS = ("global_load", "flat_load", "scratch_load", "buffer_load", "ds_read", "ds_load", "global_atomic",
         "flat_atomic", "buffer_atomic", "ds_")


def writes_exec(mn: str, ops: str) -> bool:
    if "saveexec" in mn or mn.startswith("v_cmpx"):
        return True
    if mn.startswith("s_") and re.match(r"^exec\b", ops):
        return True
    return mn.startswith(("s_setpc", "s_swappc", "s_branch", "s_cbranch", "s_endpgm"))


def narrows_exec(mn: str, ops: str) -> bool:
    """An EXEC write that can turn lanes off (the if / loop masks), as opposed to a restore."""
    if mn.startswith(("s_or_", "s_cbranch", "s_branch")):
        return False
    return writes_exec(mn, ops) and not mn.startswith(("s_setpc", "s_swappc", "s_endpgm"))


def writes_vgpr(mn: str, ops: str) -> bool:
    if mn.startswith("v_"):
        if mn.startswith(("v_readlane", "v_readfirstlane", "v_cmp", "v_writelane")):
            return False
        return bool(VDST.match(ops))
    if mn.startswith(LOADS):
        return bool(VDST.match(ops))
    return False


def parse(dis: str):
    """[(addr, function, mnemonic, operands)] of a disassembly."""
    out, fn = [], None
    for line in dis.splitlines():
        m = FUNC.match(line)
        if m:
            fn = m.group(2)
            continue
        m = LINE.match(line)
        if m:
            out.append((int(m.group(3), 16), fn, m.group(1), m.group(2)))
    return out


def disassemble(co: bytes) -> str:
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(co)
        f.flush()
        return subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", "--mcpu=gfx950", f.name], capture_output=True,
                              text=True, check=True).stdout


def check_code_object(co: bytes):
    """Yields (function, join address, offending instruction) for one code object."""
    yield from check_disassembly(disassemble(co))


def check_disassembly(dis: str):
    """Yields (function, join address, offending instruction) for llvm-objdump -d text
    (tests/golden/exec_join_*.s hold excerpts with and without the split copies)."""
    ins = parse(dis)
    index = {a: i for i, (a, _, _, _) in enumerate(ins)}
    starts = []
    for i, (a, fn, mn, ops) in enumerate(ins):
        # only the branches that skip or leave a divergent region: EXEC was just narrowed (an
        # execz test after a restore is a wave-empty check, not a region boundary)
        prev = ins[i - 1] if i else None
        if not (prev and narrows_exec(prev[2], prev[3])):
            continue
        if mn == "s_cbranch_execz":
            off = int(ops.split()[0])
            t = a + 4 + 4 * (off - 65536 if off > 32767 else off)
            if t in index:
                starts.append(index[t])
        elif mn == "s_cbranch_execnz" and i + 1 < len(ins):
            starts.append(i + 1)
    seen = set()
    for s in starts:
        if s in seen:
            continue
        seen.add(s)
        for a, fn, mn, ops in ins[s:s + 64]:
            if writes_exec(mn, ops):
                break
            if writes_vgpr(mn, ops):
                yield fn, ins[s][0], f"{a:#x}: {mn} {ops}"


def check_library(path: str):
    data = open(path, "rb").read()
    found = []
    for triple, co in bundles(data):
        if "gfx950" in triple and co:
            found.extend(check_code_object(co))
    return found


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="*", default=[DEFAULT_LIB])
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args()
    bad = 0
    for lib in a.libs:
        found = check_library(lib)
        bad += len(found)
        per = {}
        for fn, join, what in found:
            per.setdefault(readable(fn), []).append((join, what))
        print(f"{os.path.basename(lib)}: {len(found)} vector writes before an EXEC restore"
              + "".join(f"\n  {fn}: {len(v)}" for fn, v in sorted(per.items())))
        if a.verbose:
            for fn, v in sorted(per.items()):
                for join, what in v:
                    print(f"    {fn} join {join:#x} -> {what}")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
