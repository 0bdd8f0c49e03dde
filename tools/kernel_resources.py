#!/usr/bin/env python3
"""Register / scratch resources of the gfx950 kernels inside a HIP shared library.

    python3 tools/kernel_resources.py [lib.so] [--filter trace_samples] [--json]

Reads the library's clang offload bundles (.hip_fatbin: one per translation unit),
takes each gfx950 code object, and decodes its NT_AMDGPU_METADATA note (msgpack,
amdhsa.kernels): per kernel the VGPR / AGPR / SGPR counts, the VGPR and SGPR spill
counts, the scratch (private segment) size and the LDS (group segment) size. No GPU
and no external tool needed; tests/test_kernel_resources.py compares the trace_samples
instances against the committed table tests/golden/kernel_resources.json, so a compiler
bump or an unrelated edit that makes an instance spill more fails in the CPU suite.
"""
from __future__ import annotations

import argparse
import json
import os
import struct
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT_LIB = os.path.join(ROOT, "raytracinginoneweekendinrust_amd", "_lib", "librtamd.so")
BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
NT_AMDGPU_METADATA = 32


def bundles(data: bytes):
    """Yields (triple, code object bytes) of every offload bundle in `data`."""
    pos = data.find(BUNDLE_MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", data, pos + 24)[0]
        p = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24: p + 24 + tlen].decode()
            p += 24 + tlen
            yield triple, data[pos + off: pos + off + size]
        pos = data.find(BUNDLE_MAGIC, pos + 1)


def notes(elf: bytes):
    """Yields (type, name, desc) of every note in a 64-bit little-endian ELF's PT_NOTE segments."""
    if elf[:4] != b"\x7fELF":
        return
    phoff = struct.unpack_from("<Q", elf, 0x20)[0]
    phentsize, phnum = struct.unpack_from("<HH", elf, 0x36)
    for i in range(phnum):
        ptype, _flags, off, _va, _pa, filesz = struct.unpack_from("<IIQQQQ", elf, phoff + i * phentsize)
        if ptype != 4:  # PT_NOTE
            continue
        p, end = off, off + filesz
        while p + 12 <= end:
            namesz, descsz, ntype = struct.unpack_from("<III", elf, p)
            name = elf[p + 12: p + 12 + namesz].rstrip(b"\0").decode()
            d0 = p + 12 + ((namesz + 3) & ~3)
            yield ntype, name, elf[d0: d0 + descsz]
            p = d0 + ((descsz + 3) & ~3)


def kernel_resources(lib_path: str = DEFAULT_LIB) -> dict:
    """{kernel symbol: resources} over every gfx950 code object of the library."""
    import msgpack
    data = open(lib_path, "rb").read()
    out = {}
    for triple, co in bundles(data):
        if "gfx950" not in triple:
            continue
        for ntype, name, desc in notes(co):
            if name != "AMDGPU" or ntype != NT_AMDGPU_METADATA:
                continue
            md = msgpack.unpackb(desc, raw=False)
            for k in md.get("amdhsa.kernels", []):
                out[k[".symbol"].removesuffix(".kd")] = {
                    "name": k.get(".name"),
                    "vgpr_count": k.get(".vgpr_count"),
                    "agpr_count": k.get(".agpr_count"),
                    "sgpr_count": k.get(".sgpr_count"),
                    "vgpr_spill_count": k.get(".vgpr_spill_count"),
                    "sgpr_spill_count": k.get(".sgpr_spill_count"),
                    "private_segment_fixed_size": k.get(".private_segment_fixed_size"),
                    "group_segment_fixed_size": k.get(".group_segment_fixed_size"),
                    "uses_dynamic_stack": k.get(".uses_dynamic_stack"),
                }
    return out


def readable(symbol: str) -> str:
    """trace_samples<kKind, kWaves, kF> for a mangled trace_samples instance; the symbol otherwise."""
    import re
    m = re.search(r"trace_samplesILi(\d+)ELi(\d+)ELj(\d+)E", symbol)
    return f"trace_samples<{m.group(1)}, {m.group(2)}, {m.group(3)}>" if m else symbol


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?", default=DEFAULT_LIB)
    ap.add_argument("--filter", default="trace_samples")
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args()
    res = {k: v for k, v in kernel_resources(a.lib).items() if a.filter in k}
    names = {k: readable(k) for k in res}
    if a.json:
        json.dump({names[k]: v for k, v in sorted(res.items(), key=lambda kv: names[kv[0]])}, sys.stdout, indent=1)
        print()
        return
    for k in sorted(res, key=lambda s: names[s]):
        v = res[k]
        print(f"{names[k]:32s} vgpr {v['vgpr_count']:4d} sgpr {v['sgpr_count']:4d} spill v{v['vgpr_spill_count']:4d} "
              f"s{v['sgpr_spill_count']:4d} scratch {v['private_segment_fixed_size']:6d} B lds {v['group_segment_fixed_size']}")


if __name__ == "__main__":
    main()
