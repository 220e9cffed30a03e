"""Time hipMalloc / hipMemset / hipFree of large device buffers on the GPU box (does the generated
path's per-run allocation of its state store cost seconds?).   python scripts/hipmalloc_time.py GIB ..."""
import ctypes
import sys
import time

hip = ctypes.CDLL("libamdhip64.so")
hip.hipSetDevice(0)
hip.hipDeviceSynchronize()
for gib in [int(x) for x in sys.argv[1:]] or [16, 64, 200]:
    p = ctypes.c_void_p()
    t0 = time.time()
    rc = hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(gib << 30))
    t1 = time.time()
    hip.hipMemset(p, 0, ctypes.c_size_t(1 << 30))
    hip.hipDeviceSynchronize()
    t2 = time.time()
    hip.hipFree(p)
    t3 = time.time()
    print("hipMalloc %d GiB rc=%d: malloc %.3f s, memset 1 GiB %.3f s, free %.3f s" % (gib, rc, t1 - t0, t2 - t1, t3 - t2), flush=True)
