"""Probe: HIP event-record nodes inside a torch.cuda.graph capture (return codes of each call),
through the HIP runtime torch itself loaded (torch/lib/libamdhip64.so)."""
import ctypes
import os
import torch

hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
v = ctypes.c_int()
hip.hipRuntimeGetVersion(ctypes.byref(v))
print("runtime", v.value)
vp = ctypes.c_void_p
s = torch.cuda.Stream()
x = torch.zeros(1 << 20, device="cuda")
ev = [vp() for _ in range(4)]
for e in ev:
    hip.hipEventCreate(ctypes.byref(e))


def manual(e):
    st, cid, g, deps, nd = ctypes.c_int(), ctypes.c_ulonglong(), vp(), ctypes.POINTER(vp)(), ctypes.c_size_t()
    r1 = hip.hipStreamGetCaptureInfo_v2(vp(s.cuda_stream), ctypes.byref(st), ctypes.byref(cid), ctypes.byref(g),
                                        ctypes.byref(deps), ctypes.byref(nd))
    node = vp()
    r2 = hip.hipGraphAddEventRecordNode(ctypes.byref(node), g, deps, nd, e)
    r3 = hip.hipStreamUpdateCaptureDependencies(vp(s.cuda_stream), ctypes.byref(node), ctypes.c_size_t(1), 1)
    return r1, r2, r3, st.value, nd.value


for mode in ("flags", "manual", "torch_external"):
    g = torch.cuda.CUDAGraph()
    te = [torch.cuda.Event(enable_timing=True, external=True) for _ in range(2)]
    try:
        with torch.cuda.graph(g, stream=s):
            if mode == "flags":
                print(mode, "rec0", hip.hipEventRecordWithFlags(ev[0], vp(s.cuda_stream), 1))
                hip.hipGetLastError()
            elif mode == "manual":
                print(mode, "rec0", manual(ev[2]))
            else:
                te[0].record(s)
            for _ in range(50):
                x.mul_(1.0001)
            if mode == "flags":
                print(mode, "rec1", hip.hipEventRecordWithFlags(ev[1], vp(s.cuda_stream), 1))
                hip.hipGetLastError()
            elif mode == "manual":
                print(mode, "rec1", manual(ev[3]))
            else:
                te[1].record(s)
    except Exception as exc:
        print(mode, "capture failed:", str(exc).splitlines()[0])
        hip.hipGetLastError()
        continue
    for r in range(3):
        g.replay()
        torch.cuda.synchronize()
        if mode == "torch_external":
            print(mode, "replay", r, te[0].elapsed_time(te[1]))
        else:
            ms = ctypes.c_float(-1)
            a, b = (ev[0], ev[1]) if mode == "flags" else (ev[2], ev[3])
            print(mode, "replay", r, hip.hipEventElapsedTime(ctypes.byref(ms), a, b), ms.value)
