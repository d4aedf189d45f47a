import time, torch, ctypes
dev = torch.device("cuda", 0)
s = torch.cuda.Stream(device=dev)
big = torch.randn(64 * 1024 * 1024, device=dev)
hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
for mib in (1, 2, 3, 4, 8, 16):
    n = mib * 262144
    src = torch.ones(n, device=dev)
    dst = torch.empty(n, pin_memory=True)
    for mode in ("torch", "hip"):
        torch.cuda.synchronize()
        with torch.cuda.stream(s):
            for _ in range(20):
                big.mul_(1.0001)  # ~ several ms of GPU work queued ahead
            t0 = time.perf_counter()
            if mode == "torch":
                dst.copy_(src, non_blocking=True)
            else:
                hip.hipMemcpyAsync(ctypes.c_void_p(dst.data_ptr()), ctypes.c_void_p(src.data_ptr()), n * 4, 2, ctypes.c_void_p(s.cuda_stream))
            t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"{mib} MiB {mode}: enqueue {1e3*(t1-t0):.3f} ms, total {1e3*(t2-t0):.3f} ms", flush=True)
