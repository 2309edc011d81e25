"""Host CPU time of hipEventSynchronize on a ~5 ms kernel with event flags 0, blocking-sync,
and of a nap-then-spin poll on hipEventQuery (round 5, tools/archive/r05/spin_probe.py follow-up)."""
import ctypes as C
import resource
import time

import torch

hip = C.CDLL("libamdhip64.so")


def cpu_s():
    r = resource.getrusage(resource.RUSAGE_SELF)
    return r.ru_utime + r.ru_stime


torch.cuda.init()
torch.cuda._sleep(1000)
torch.cuda.synchronize()
stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
for name, flags in (("default", 0x2), ("blocking", 0x2 | 0x1)):
    ev = C.c_void_p()
    assert hip.hipEventCreateWithFlags(C.byref(ev), flags) == 0
    for mode in ("sync", "query-nap"):
        res = []
        for _ in range(5):
            torch.cuda._sleep(10_000_000)
            assert hip.hipEventRecord(ev, stream) == 0
            c0, t0 = cpu_s(), time.perf_counter()
            if mode == "sync":
                assert hip.hipEventSynchronize(ev) == 0
            else:
                while hip.hipEventQuery(ev) != 0:
                    time.sleep(50e-6)
            res.append(((time.perf_counter() - t0) * 1e3, (cpu_s() - c0) * 1e3))
        print(f"{name:9s} {mode:10s} wall/cpu ms: " + " ".join(f"{w:.2f}/{c:.2f}" for w, c in res), flush=True)
