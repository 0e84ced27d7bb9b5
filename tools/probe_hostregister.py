#!/usr/bin/env python3
"""Feasibility probe: H2D straight out of a page-cache file mapping
(mmap + hipHostRegister) against pread into pinned staging + H2D. One JSON
line per method. Not part of the product path."""
import ctypes
import json
import mmap
import os
import sys
import tempfile
import time


def main():
    import numpy as np
    import torch
    size = int(sys.argv[1]) if len(sys.argv) > 1 else (2 << 30)
    d = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
    path = os.path.join(d, "cap.bin")
    with open(path, "wb") as f:
        chunk = np.random.default_rng(0).integers(0, 256, 1 << 26, dtype=np.uint8).tobytes()
        for _ in range(size >> 26):
            f.write(chunk)
    hip = ctypes.CDLL("libamdhip64.so")
    dev = torch.empty(size, dtype=torch.uint8, device="cuda")
    # (1) pread into pinned staging, then H2D
    pinned = torch.empty(size, dtype=torch.uint8, pin_memory=True)
    fd = os.open(path, os.O_RDONLY)
    pv = memoryview(pinned.numpy())
    for rep in range(3):
        t0 = time.perf_counter()
        got = 0
        while got < size:
            got += os.preadv(fd, [pv[got:got + (1 << 26)]], got)
        t1 = time.perf_counter()
        dev.copy_(pinned, non_blocking=True)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
    print(json.dumps({"method": "pread->pinned->H2D", "bytes": size, "read_gbs": round(size / (t1 - t0) / 1e9, 2),
                      "h2d_gbs": round(size / (t2 - t1) / 1e9, 2), "total_gbs": round(size / (t2 - t0) / 1e9, 2)}),
          flush=True)
    # (2) mmap (page cache) + hipHostRegister, H2D straight from the mapping
    mm = mmap.mmap(fd, size, prot=mmap.PROT_READ)
    arr = np.frombuffer(mm, np.uint8)
    host_ptr = arr.ctypes.data
    for flags, name in ((0, "default"), (8, "readonly")):  # hipHostRegisterReadOnly = 0x08
        t0 = time.perf_counter()
        rc = hip.hipHostRegister(ctypes.c_void_p(host_ptr), ctypes.c_size_t(size), ctypes.c_uint(flags))
        t1 = time.perf_counter()
        if rc != 0:
            print(json.dumps({"method": f"mmap+hipHostRegister({name})", "rc": rc}), flush=True)
            continue
        for rep in range(3):
            t2 = time.perf_counter()
            rc2 = hip.hipMemcpy(ctypes.c_void_p(dev.data_ptr()), ctypes.c_void_p(host_ptr), ctypes.c_size_t(size), 1)
            t3 = time.perf_counter()
        ok = bool((dev[:1 << 20].cpu().numpy() == arr[:1 << 20]).all())
        print(json.dumps({"method": f"mmap+hipHostRegister({name})->H2D", "rc": rc2, "register_s": round(t1 - t0, 3),
                          "h2d_gbs": round(size / (t3 - t2) / 1e9, 2), "bytes_equal": ok}), flush=True)
        hip.hipHostUnregister(ctypes.c_void_p(host_ptr))
    del arr
    mm.close()
    os.close(fd)
    os.remove(path)


if __name__ == "__main__":
    main()
