"""Host-to-device copy rate on the box: pinned and pageable torch tensors of
frame size (1080p luma, 2.07 MB) and 64 MB, copied back to back on one stream
and on two streams (two DMA engines?), HIP events around each run."""
import torch

dev = torch.device("cuda", 0)
for nbytes in (1920 * 1080, 64 << 20):
    for pin in (True, False):
        src = torch.empty(nbytes, dtype=torch.uint8).pin_memory() if pin else torch.empty(nbytes, dtype=torch.uint8)
        dst = [torch.empty(nbytes, dtype=torch.uint8, device=dev) for _ in range(2)]
        reps = 64 if nbytes < (8 << 20) else 8
        for nstreams in (1, 2):
            streams = [torch.cuda.Stream(device=dev) for _ in range(nstreams)]
            for _ in range(2):
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                import time
                t0 = time.perf_counter()
                for i in range(reps):
                    s = streams[i % nstreams]
                    with torch.cuda.stream(s):
                        dst[i % 2].copy_(src, non_blocking=True)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
            print(f"{nbytes/1e6:.2f} MB pinned={pin} streams={nstreams}: {reps*nbytes/dt/1e9:.1f} GB/s "
                  f"({dt/reps*1e6:.1f} us per copy)", flush=True)
