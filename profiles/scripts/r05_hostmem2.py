"""Round 5: transparent huge pages (the box runs THP in madvise mode) for the large host buffers
of similarity.main. Times (ms) for SIZE bytes: anonymous mmap with and without
madvise(MADV_HUGEPAGE) -- first touch (1 and 16 threads), pageable device-to-host copy into
fresh and into touched pages, munmap."""
import ctypes
import json
import sys
import threading
import time

import numpy as np

libc = ctypes.CDLL("libc.so.6", use_errno=True)
libc.mmap.restype = ctypes.c_void_p
libc.mmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long]
libc.munmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
libc.madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
hip = ctypes.CDLL("libamdhip64.so")
vp = ctypes.c_void_p
PROT_RW, MAP_PRIV_ANON, MADV_HUGEPAGE = 3, 0x22, 14
MB = 1 << 20
SIZE = int(sys.argv[1]) * MB if len(sys.argv) > 1 else 600 * MB


def ms(t):
    return round((time.perf_counter() - t) * 1e3, 2)


def region(huge):
    p = libc.mmap(None, SIZE + 2 * MB, PROT_RW, MAP_PRIV_ANON, -1, 0)
    a = (p + 2 * MB - 1) // (2 * MB) * (2 * MB)
    if huge:
        assert libc.madvise(a, SIZE, MADV_HUGEPAGE) == 0
    return p, a


def touch(a, nt):
    def work(t):
        lo, hi = SIZE * t // nt // 4096 * 4096, SIZE * (t + 1) // nt
        buf = np.ctypeslib.as_array((ctypes.c_uint8 * (hi - lo)).from_address(a + lo))
        buf[::4096] = 0  # numpy's strided fill (no GIL held)
    th = [threading.Thread(target=work, args=(t,)) for t in range(nt)]
    [x.start() for x in th]
    [x.join() for x in th]


huge_mode = [False]
assert hip.hipSetDevice(0) == 0
d = vp()
assert hip.hipMalloc(ctypes.byref(d), ctypes.c_size_t(SIZE)) == 0
assert hip.hipMemset(d, 1, ctypes.c_size_t(SIZE)) == 0
hip.hipDeviceSynchronize()
out = {"bytes": SIZE}
for rep in range(2):
    for huge in (False, True):
        huge_mode[0] = huge
        r = {}
        p, a = region(huge)
        t = time.perf_counter()
        touch(a, 1)
        r["first_touch_1t"] = ms(t)
        t = time.perf_counter()
        assert hip.hipMemcpy(vp(a), d, ctypes.c_size_t(SIZE), 2) == 0
        r["d2h_touched"] = ms(t)
        t = time.perf_counter()
        libc.munmap(p, SIZE + 2 * MB)
        r["munmap"] = ms(t)
        p, a = region(huge)
        t = time.perf_counter()
        assert hip.hipMemcpy(vp(a), d, ctypes.c_size_t(SIZE), 2) == 0
        r["d2h_fresh"] = ms(t)
        libc.munmap(p, SIZE + 2 * MB)
        p, a = region(huge)
        t = time.perf_counter()
        touch(a, 16)
        r["first_touch_16t"] = ms(t)
        libc.munmap(p, SIZE + 2 * MB)
        out["rep%d_%s" % (rep, "huge" if huge else "4k")] = r
print(json.dumps(out))
