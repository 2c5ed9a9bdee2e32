"""Probe: can a captured hipGraph carry timing events (external event-record
nodes), and do they time a kernel?  Prints each HIP call's status.

    python tools/probe_graph_events.py
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hyperopt_amd import _lib as L  # noqa: E402


def main():
    hip = L.hip()
    s = torch.cuda.Stream()
    sp = ctypes.c_void_p(s.cuda_stream)
    x = torch.zeros(1 << 24, device="cuda")
    torch.cuda.synchronize()
    evs = []
    for _ in range(2):
        h = ctypes.c_void_p()
        print("create", hip.hipEventCreateWithFlags(ctypes.byref(h), 0))
        evs.append(h)
    # event-record nodes added to the capture's graph by hand
    P = ctypes.c_void_p
    for name, args in (("hipStreamGetCaptureInfo_v2", [P, ctypes.POINTER(ctypes.c_int),
                                                      ctypes.POINTER(ctypes.c_ulonglong),
                                                      ctypes.POINTER(P),
                                                      ctypes.POINTER(ctypes.POINTER(P)),
                                                      ctypes.POINTER(ctypes.c_size_t)]),
                       ("hipGraphAddEventRecordNode", [ctypes.POINTER(P), P, ctypes.POINTER(P),
                                                      ctypes.c_size_t, P]),
                       ("hipStreamUpdateCaptureDependencies", [P, ctypes.POINTER(P),
                                                              ctypes.c_size_t, ctypes.c_uint])):
        fn = getattr(hip, name)
        fn.restype = ctypes.c_int
        fn.argtypes = args

    def node(ev):
        st, cid, gr = ctypes.c_int(), ctypes.c_ulonglong(), P()
        deps, nd = ctypes.POINTER(P)(), ctypes.c_size_t()
        print(" info", hip.hipStreamGetCaptureInfo_v2(sp, ctypes.byref(st), ctypes.byref(cid),
                                                     ctypes.byref(gr), ctypes.byref(deps),
                                                     ctypes.byref(nd)), st.value, nd.value)
        n = P()
        print(" add", hip.hipGraphAddEventRecordNode(ctypes.byref(n), gr, deps, nd.value, ev))
        print(" upd", hip.hipStreamUpdateCaptureDependencies(sp, ctypes.byref(n), 1, 1))

    print("begin manual", hip.hipStreamBeginCapture(sp, L.CAPTURE_RELAXED))
    node(evs[0])
    with torch.cuda.stream(s):
        x.mul_(1.0001)
    node(evs[1])
    g = ctypes.c_void_p()
    print("end", hip.hipStreamEndCapture(sp, ctypes.byref(g)))
    e = ctypes.c_void_p()
    print("inst", hip.hipGraphInstantiate(ctypes.byref(e), g, None, None, 0))
    for _ in range(3):
        print("launch", hip.hipGraphLaunch(e, sp))
        print("sync", hip.hipStreamSynchronize(sp))
        ms = ctypes.c_float()
        print("elapsed", hip.hipEventElapsedTime(ctypes.byref(ms), evs[0], evs[1]), ms.value)
    for mode, flags in (("plain", 0),):
        print("begin", mode, hip.hipStreamBeginCapture(sp, L.CAPTURE_RELAXED))
        print("record0", hip.hipEventRecordWithFlags(evs[0], sp, flags))
        with torch.cuda.stream(s):
            x.mul_(1.0001)
        print("record1", hip.hipEventRecordWithFlags(evs[1], sp, flags))
        g = ctypes.c_void_p()
        print("end", hip.hipStreamEndCapture(sp, ctypes.byref(g)))
        e = ctypes.c_void_p()
        print("inst", hip.hipGraphInstantiate(ctypes.byref(e), g, None, None, 0))
        for _ in range(3):
            print("launch", hip.hipGraphLaunch(e, sp))
            print("sync", hip.hipStreamSynchronize(sp))
            ms = ctypes.c_float()
            print("elapsed", hip.hipEventElapsedTime(ctypes.byref(ms), evs[0], evs[1]), ms.value)
        hip.hipGraphExecDestroy(e)
        hip.hipGraphDestroy(g)
    # plain event records outside a graph around a graph launch
    h = ctypes.c_void_p()
    print("plain-around", hip.hipEventRecord(evs[0], sp))


if __name__ == "__main__":
    main()
