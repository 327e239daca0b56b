"""GPU probe: timing event-record nodes inside a torch-captured HIP graph, two ways
(hipEventRecordWithFlags(External) during capture; hipGraphAddEventRecordNode spliced into the capture
with hipStreamGetCaptureInfo_v2 / hipStreamUpdateCaptureDependencies)."""
import ctypes

import torch

hip = ctypes.CDLL("libamdhip64.so.7")
vp = ctypes.c_void_p
hip.hipGetErrorName.restype = ctypes.c_char_p


def chk(r, what):
    print(f"{what}: {r} {hip.hipGetErrorName(r).decode() if r else ''}", flush=True)
    return r


def mk(flags=0):
    e = vp()
    chk(hip.hipEventCreateWithFlags(ctypes.byref(e), ctypes.c_uint(flags)), "hipEventCreateWithFlags")
    return e


def ms(a, b):
    t = ctypes.c_float()
    r = hip.hipEventElapsedTime(ctypes.byref(t), a, b)
    return t.value if r == 0 else f"err {r} {hip.hipGetErrorName(r).decode()}"


def splice(ev, st):
    """Add an event-record node after the capture's current dependencies and make it the new one."""
    status = ctypes.c_int()
    cid = ctypes.c_ulonglong()
    graph = vp()
    deps = ctypes.POINTER(vp)()
    nd = ctypes.c_size_t()
    r = hip.hipStreamGetCaptureInfo_v2(vp(st.cuda_stream), ctypes.byref(status), ctypes.byref(cid), ctypes.byref(graph),
                                       ctypes.byref(deps), ctypes.byref(nd))
    if r:
        return chk(r, "hipStreamGetCaptureInfo_v2")
    node = vp()
    darr = (vp * max(1, nd.value))(*[deps[i] for i in range(nd.value)])
    r = hip.hipGraphAddEventRecordNode(ctypes.byref(node), graph, darr, nd, ev)
    if r:
        return chk(r, "hipGraphAddEventRecordNode")
    narr = (vp * 1)(node)
    r = hip.hipStreamUpdateCaptureDependencies(vp(st.cuda_stream), narr, ctypes.c_size_t(1), ctypes.c_uint(1))
    if r:
        return chk(r, "hipStreamUpdateCaptureDependencies")
    return 0


def main():
    dev = torch.device("cuda", 0)
    a = torch.randn(4096, 4096, device=dev)
    b = torch.randn(4096, 4096, device=dev)
    st = torch.cuda.Stream()
    c = a @ b
    torch.cuda.synchronize()
    evs = [mk() for _ in range(3)]
    import sys
    for mode in sys.argv[1:]:
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=st):
            s = torch.cuda.current_stream()
            for i in range(3):
                if mode == "flags":
                    r = chk(hip.hipEventRecordWithFlags(evs[i], vp(s.cuda_stream), ctypes.c_uint(1)), f"{mode} record {i}")
                else:
                    r = chk(splice(evs[i], s), f"{mode} splice {i}")
                if i < 2:
                    c = a @ b
        for _ in range(3):
            g.replay()
            torch.cuda.synchronize()
            print(mode, "elapsed", ms(evs[0], evs[1]), ms(evs[1], evs[2]), flush=True)
        del c


if __name__ == "__main__":
    main()
