"""Round 5: host-memory costs behind similarity.main's fetch and teardown on the GPU box.
Times (ms): pinned host allocation (hipHostMalloc) and free, pageable and pinned device-to-host
copies of the config-2 fetch size, first-touch of fresh pages, and munmap of a large numpy array.
Direct HIP runtime calls through ctypes (no libblp)."""
import ctypes
import json
import os
import sys
import time

import numpy as np

hip = ctypes.CDLL("libamdhip64.so")
vp = ctypes.c_void_p
MB = 1 << 20
SIZE = int(sys.argv[1]) * MB if len(sys.argv) > 1 else 600 * MB
out = {"bytes": SIZE}


def ms(t):
    return round((time.perf_counter() - t) * 1e3, 2)


def ck(rc, what):
    if rc:
        raise RuntimeError("%s: %d" % (what, rc))


for f in ("/sys/kernel/mm/transparent_hugepage/enabled", "/sys/kernel/mm/transparent_hugepage/defrag"):
    try:
        out[os.path.basename(os.path.dirname(f)) + "/" + os.path.basename(f)] = open(f).read().strip()
    except OSError as e:
        out[f] = str(e)
ck(hip.hipSetDevice(0), "hipSetDevice")
d = vp()
ck(hip.hipMalloc(ctypes.byref(d), ctypes.c_size_t(SIZE)), "hipMalloc")
ck(hip.hipMemset(d, 1, ctypes.c_size_t(SIZE)), "hipMemset")
ck(hip.hipDeviceSynchronize(), "sync")
D2H = 2
for rep in range(2):
    r = {}
    t = time.perf_counter()
    a = np.empty(SIZE, np.uint8)
    ck(hip.hipMemcpy(vp(a.ctypes.data), d, ctypes.c_size_t(SIZE), D2H), "memcpy")
    r["pageable_fresh_d2h"] = ms(t)
    t = time.perf_counter()
    ck(hip.hipMemcpy(vp(a.ctypes.data), d, ctypes.c_size_t(SIZE), D2H), "memcpy")
    r["pageable_touched_d2h"] = ms(t)
    t = time.perf_counter()
    del a
    r["numpy_free"] = ms(t)
    t = time.perf_counter()
    b = np.empty(SIZE, np.uint8)
    b[::4096] = 0
    r["first_touch_1thread"] = ms(t)
    del b
    h = vp()
    t = time.perf_counter()
    ck(hip.hipHostMalloc(ctypes.byref(h), ctypes.c_size_t(SIZE), 0), "hipHostMalloc")
    r["hipHostMalloc"] = ms(t)
    t = time.perf_counter()
    ck(hip.hipMemcpy(h, d, ctypes.c_size_t(SIZE), D2H), "memcpy")
    r["pinned_d2h"] = ms(t)
    t = time.perf_counter()
    ck(hip.hipMemcpy(h, d, ctypes.c_size_t(SIZE), D2H), "memcpy")
    r["pinned_d2h_2"] = ms(t)
    t = time.perf_counter()
    ck(hip.hipHostFree(h), "hipHostFree")
    r["hipHostFree"] = ms(t)
    # register an existing (touched) numpy buffer
    c = np.empty(SIZE, np.uint8)
    c[::4096] = 0
    t = time.perf_counter()
    ck(hip.hipHostRegister(vp(c.ctypes.data), ctypes.c_size_t(SIZE), 0), "hipHostRegister")
    r["hipHostRegister"] = ms(t)
    t = time.perf_counter()
    ck(hip.hipMemcpy(vp(c.ctypes.data), d, ctypes.c_size_t(SIZE), D2H), "memcpy")
    r["registered_d2h"] = ms(t)
    t = time.perf_counter()
    ck(hip.hipHostUnregister(vp(c.ctypes.data)), "hipHostUnregister")
    r["hipHostUnregister"] = ms(t)
    del c
    out["rep%d" % rep] = r
print(json.dumps(out))
