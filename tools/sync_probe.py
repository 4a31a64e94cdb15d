"""Cost of torch.cuda.synchronize() (hipDeviceSynchronize) under the HIP
device scheduling flags: auto (default), spin, yield, blocking.  The flag is
set through the HIP runtime torch itself loads, before torch creates its
context.  Prints one JSON line: idle-sync us (median of 200), and the wall
time of 20 back-to-back 10 us spin kernels + a synchronize.

    python tools/sync_probe.py auto|spin|yield|block
"""
import ctypes
import json
import os
import sys
import time

import torch

FLAGS = {"auto": 0, "spin": 1, "yield": 2, "block": 4}


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "auto"
    hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    rc_set = None
    if mode != "auto":
        rc_set = hip.hipSetDeviceFlags(ctypes.c_uint(FLAGS[mode]))
    torch.cuda.init()
    x = torch.zeros(1, device="cuda")
    torch.cuda.synchronize()
    flags = ctypes.c_uint(0)
    rc_get = hip.hipGetDeviceFlags(ctypes.byref(flags))
    ts = []
    for _ in range(200):
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    walls = []
    for _ in range(20):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            torch.cuda._sleep(20000)  # ~10 us of GPU time per kernel
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t0)
    walls.sort()
    print(json.dumps(dict(mode=mode, set_rc=rc_set, get_rc=rc_get, device_flags=flags.value,
                          idle_sync_us_median=round(ts[100] * 1e6, 2), idle_sync_us_p10=round(ts[20] * 1e6, 2),
                          k20_wall_us_median=round(walls[10] * 1e6, 1))), flush=True)


if __name__ == "__main__":
    main()
