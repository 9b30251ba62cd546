"""D2H copy engine under torch's bundled HIP runtime: hipMemcpyAsync device -> pinned host (hipHostMalloc)
33 MB on a plain stream, after a kernel on the same stream. Run under rocprofv3 --kernel-trace
--memory-copy-trace: a DMA copy shows in the copy trace, a blit as __amd_rocclr_copyBuffer."""
import ctypes
import time

import torch

hip = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)  # torch's copy (already loaded)
n = 3840 * 2160 * 4
d = torch.ones(n // 4, dtype=torch.int32, device="cuda")
h = ctypes.c_void_p()
assert hip.hipHostMalloc(ctypes.byref(h), ctypes.c_size_t(n), 0) == 0
s = torch.cuda.Stream()
for with_kernel in (False, True):
    best = 1e9
    for _ in range(3):
        with torch.cuda.stream(s):
            if with_kernel:
                d.add_(1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            if with_kernel:
                d[:64].add_(1)
        assert hip.hipMemcpyAsync(h, ctypes.c_void_p(d.data_ptr()), ctypes.c_size_t(n), 2, ctypes.c_void_p(s.cuda_stream)) == 0
        s.synchronize()
        best = min(best, time.perf_counter() - t0)
    print(f"kernel before: {with_kernel}  {best * 1e3:.3f} ms  {n / best / 1e9:.1f} GB/s", flush=True)
