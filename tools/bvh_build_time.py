#!/usr/bin/env python3
"""Time Bvh::new's leaf ordering: rt_bvh_build_order on the device (synchronous call,
keys already in HBM) vs the single-threaded C restatement (oracle_bvh_order, the same
stable-merge-sort recursion the host lowering runs). Prints one JSON line per size.

    python3 tools/bvh_build_time.py [n ...]
"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import raytracinginoneweekendinrust_amd as rt  # noqa: E402
from oracle import oracle_ffi  # noqa: E402


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [16384, 262144, 1 << 20, 1 << 22]
    for n in sizes:
        keys = np.random.default_rng(n).uniform(-500, 500, size=(n, 3)).astype(np.float32)
        dk = torch.from_numpy(keys.reshape(-1)).to("cuda:0")
        out = torch.empty(n, dtype=torch.int32, device="cuda:0")
        st = torch.cuda.current_stream(0).cuda_stream

        def run():
            rt.check(rt.lib.rt_bvh_build_order(C.c_void_p(dk.data_ptr()), n, 20231, C.c_void_p(out.data_ptr()),
                                               C.c_void_p(st or None)), "rt_bvh_build_order")
        run()
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            run()
        dev_ms = (time.perf_counter() - t0) / reps * 1e3
        t0 = time.perf_counter()
        want = oracle_ffi.bvh_order(keys, 20231)
        cpu_ms = (time.perf_counter() - t0) * 1e3
        same = bool(np.array_equal(out.cpu().numpy().view(np.uint32), want))
        print(json.dumps({"items": n, "device_ms": round(dev_ms, 3), "cpu_1thread_ms": round(cpu_ms, 3),
                          "speedup": round(cpu_ms / dev_ms, 2), "identical": same}), flush=True)


if __name__ == "__main__":
    main()
