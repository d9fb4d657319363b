#!/usr/bin/env python3
"""Does the HIP runtime as loaded in a Python process (with or without torch imported first) run a
D2H copy into hipHostMalloc memory as a blit kernel?  Run under `rocprofv3 --kernel-trace`:
__amd_rocclr_copyBuffer in the trace = blit.  Usage: d2h_py.py [torch|plain] [hostptr|devptr]"""
import ctypes as C
import sys

mode = sys.argv[1] if len(sys.argv) > 1 else "plain"
dst_kind = sys.argv[2] if len(sys.argv) > 2 else "hostptr"
if mode == "torch":
    import torch
    torch.cuda.init()
    torch.zeros(1, device="cuda")
hip = C.CDLL("libamdhip64.so", mode=C.RTLD_GLOBAL)
d, h, s = C.c_void_p(), C.c_void_p(), C.c_void_p()
n = 64 << 20
assert hip.hipMalloc(C.byref(d), C.c_size_t(n)) == 0
assert hip.hipHostMalloc(C.byref(h), C.c_size_t(n), C.c_uint(0x1)) == 0  # hipHostMallocPortable
assert hip.hipStreamCreateWithFlags(C.byref(s), C.c_uint(1)) == 0
dst = h
if dst_kind == "devptr":
    class Attr(C.Structure):  # hipPointerAttribute_t prefix: type, device, devicePointer, hostPointer
        _fields_ = [("type", C.c_int), ("device", C.c_int), ("devicePointer", C.c_void_p), ("hostPointer", C.c_void_p),
                    ("pad", C.c_char * 64)]
    a = Attr()
    assert hip.hipPointerGetAttributes(C.byref(a), h) == 0
    dst = C.c_void_p(a.devicePointer)
kind = 2 if dst_kind == "hostptr" else 1024  # hipMemcpyDeviceToHost / hipMemcpyDeviceToDeviceNoCU
for _ in range(10):
    assert hip.hipMemcpyAsync(dst, d, C.c_size_t(n), C.c_int(kind), s) == 0
assert hip.hipStreamSynchronize(s) == 0
print(f"{mode} {dst_kind}: 10 copies of 64 MB done")
