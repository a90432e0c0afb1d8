"""r06: hipMalloc / first kernel touch / hipFree cost by size on the box (the drop-in cold crawl's regrowths)."""
import ctypes
import json
import time

hip = ctypes.CDLL("libamdhip64.so")
out = {}
for gb in (0.25, 1, 4, 16):
    n = int(gb * (1 << 30))
    p = ctypes.c_void_p()
    hip.hipDeviceSynchronize()
    t0 = time.perf_counter()
    rc = hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(n))
    t1 = time.perf_counter()
    hip.hipMemset(p, 0, ctypes.c_size_t(n))
    hip.hipDeviceSynchronize()
    t2 = time.perf_counter()
    hip.hipMemset(p, 1, ctypes.c_size_t(n))
    hip.hipDeviceSynchronize()
    t3 = time.perf_counter()
    hip.hipFree(p)
    t4 = time.perf_counter()
    out[f"{gb}GB"] = {"rc": rc, "malloc_ms": (t1 - t0) * 1e3, "first_memset_ms": (t2 - t1) * 1e3,
                      "second_memset_ms": (t3 - t2) * 1e3, "free_ms": (t4 - t3) * 1e3}
print(json.dumps(out))
