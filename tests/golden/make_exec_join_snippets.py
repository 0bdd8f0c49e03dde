#!/usr/bin/env python3
"""Cut the two disassembly excerpts tests/test_exec_join.py feeds to tools/exec_join_check.py.

    python3 tests/golden/make_exec_join_snippets.py

exec_join_bad.s: from librtamd_rngdiv.so (the EXEC-join regression fixture, make rngdiv), the
divergent region of trace_samples<0, 3, 1> whose join carries the Rng buffer's two split copies
ahead of the EXEC restore, from the EXEC-narrowing instruction to a few lines past
the restore. exec_join_good.s: the same time-draw region of the product library's instance, whose
join restores EXEC first. Both are llvm-objdump text (the format check_disassembly parses), so the
checker's logic is pinned by fixed inputs whatever a later compiler does with the live fixture.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import exec_join_check as ejc  # noqa: E402
import kernel_resources as kr  # noqa: E402

LIB = os.path.join(ROOT, "raytracinginoneweekendinrust_amd", "_lib")
INSTANCE = "trace_samples<0, 3, 1>"


def dis_of(path):
    for triple, co in kr.bundles(open(path, "rb").read()):
        if "gfx950" in triple and co:
            text = ejc.disassemble(co)
            if any(kr.readable(fn) == INSTANCE for _, fn, _, _ in ejc.parse(text)):
                return text
    raise SystemExit(f"{INSTANCE} not in {path}")


def excerpt(text, join_addr, tail=8):
    """Lines of the function holding join_addr, from the branch to join_addr back to the
    EXEC-narrowing instruction before it, through `tail` lines past the join."""
    lines = text.splitlines()
    head, func_line, idx = None, None, {}
    for i, line in enumerate(lines):
        m = ejc.FUNC.match(line)
        if m:
            head = i
        m = ejc.LINE.match(line)
        if m:
            idx[int(m.group(3), 16)] = (i, head)
    j, head = idx[join_addr]
    # the execz branch whose target is the join
    b = None
    for i in range(j - 1, head, -1):
        m = ejc.LINE.match(lines[i])
        if m and m.group(1) == "s_cbranch_execz":
            off = int(m.group(2).split()[0])
            a = int(m.group(3), 16)
            if a + 4 + 4 * (off - 65536 if off > 32767 else off) == join_addr:
                b = i
                break
    assert b is not None, hex(join_addr)
    return "\n".join([lines[head]] + lines[b - 1:j + tail + 1]) + "\n"


def main():
    bad_text = dis_of(os.path.join(LIB, "librtamd_rngdiv.so"))
    found = [(fn, j) for fn, j, _ in ejc.check_disassembly(bad_text) if kr.readable(fn) == INSTANCE]
    assert found, "the live fixture shows no split copies in " + INSTANCE
    with open(os.path.join(HERE, "exec_join_bad.s"), "w") as f:
        f.write(excerpt(bad_text, found[0][1]))
    # the product's region: the first execz branch in the same instance whose join restores EXEC
    # at once and whose narrowing instruction is an s_and_saveexec (a plain `if`)
    good_text = dis_of(kr.DEFAULT_LIB)
    ins = ejc.parse(good_text)
    for i, (a, fn, mn, ops) in enumerate(ins):
        if kr.readable(fn) != INSTANCE or mn != "s_cbranch_execz" or "saveexec" not in ins[i - 1][2]:
            continue
        off = int(ops.split()[0])
        t = a + 4 + 4 * (off - 65536 if off > 32767 else off)
        if 8 < (t - a) // 4 < 60:
            with open(os.path.join(HERE, "exec_join_good.s"), "w") as f:
                f.write(excerpt(good_text, t))
            break
    print("wrote exec_join_bad.s and exec_join_good.s")


if __name__ == "__main__":
    main()
