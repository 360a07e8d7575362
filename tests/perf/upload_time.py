"""Host -> device upload of the cfg5 descriptor set (500 x 4096 x 128 u8 = 262 MB, a pageable
numpy array): torch .to(device) against registering the numpy buffer in place (hipHostRegister
through torch's cudart binding) and an async copy.  python tests/perf/upload_time.py"""
import time

import numpy as np
import torch


def main():
    dev = torch.device("cuda", 0)
    a = np.random.default_rng(0).integers(0, 256, (500, 4096, 128), dtype=np.uint8)
    t = torch.from_numpy(a)
    for _ in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d = t.to(dev)
        torch.cuda.synchronize()
        print("pageable .to(dev) ms", round((time.perf_counter() - t0) * 1e3, 2), flush=True)
    rt = torch.cuda.cudart()
    for _ in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rc = rt.cudaHostRegister(t.data_ptr(), t.numel(), 0)
        t1 = time.perf_counter()
        d2 = torch.empty_like(t, device=dev)
        d2.copy_(t, non_blocking=True)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        rt.cudaHostUnregister(t.data_ptr())
        t3 = time.perf_counter()
        print("register rc", rc, "register ms", round((t1 - t0) * 1e3, 2), "copy ms",
              round((t2 - t1) * 1e3, 2), "unregister ms", round((t3 - t2) * 1e3, 2), flush=True)
        assert torch.equal(d2, d)


if __name__ == "__main__":
    main()
