"""Host -> HBM upload of the cfg5 / cfg4 descriptor array (500 x 4096 x 128 u8, 262 MB), the first
thing GraphBuilder does: a pageable torch copy, the same after pin_memory() (the host copy
included), and the caller's own pages registered in place (hipHostRegister via torch.cuda.cudart)
then one DMA copy (registration + copy + unregistration timed).  ms per upload, best of 3.
python tests/perf/upload_time.py"""
import json
import time

import numpy as np
import torch


def best(fn, reps=3):
    out = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        out.append((time.perf_counter() - t) * 1e3)
    return min(out)


def main():
    desc = np.random.default_rng(0).integers(0, 256, (500, 4096, 128), dtype=np.uint8)
    dev = torch.device("cuda", 0)
    dst = torch.empty(desc.shape, dtype=torch.uint8, device=dev)
    ref = torch.from_numpy(desc).to(dev)
    rt = torch.cuda.cudart()

    def pageable():
        dst.copy_(torch.from_numpy(desc))

    def pinned_copy():
        dst.copy_(torch.from_numpy(desc).pin_memory(), non_blocking=True)

    def registered():
        h = torch.from_numpy(desc)
        assert int(rt.cudaHostRegister(h.data_ptr(), h.numel(), 0)) == 0
        try:
            dst.copy_(h, non_blocking=True)
            torch.cuda.synchronize()
        finally:
            rt.cudaHostUnregister(h.data_ptr())

    res = {"bytes": int(desc.nbytes)}
    for name, fn in (("pageable", pageable), ("pin_memory_then_copy", pinned_copy),
                     ("register_in_place", registered)):
        ms = best(fn)
        res[name] = {"ms": ms, "GBs": desc.nbytes / ms / 1e6, "same": bool(torch.equal(dst, ref))}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
