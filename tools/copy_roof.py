"""Device-to-device copy ceiling on this GPU (the deterministic re-walk copy's yardstick): torch's
copy_ of an N-GiB u32 buffer, and a read-only reduction over it, timed with HIP events.
   python tools/copy_roof.py [GiB]"""
import sys

import torch

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 6.7
n = int(gib * 2 ** 30) // 4
a = torch.randint(0, 1 << 30, (n,), dtype=torch.int32, device="cuda")
b = torch.empty_like(a)
for name, fn, traffic in (("copy", lambda: b.copy_(a), 2 * n * 4), ("read_sum", lambda: a.sum(), n * 4)):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ms = []
    for _ in range(8):
        s.record()
        fn()
        e.record()
        e.synchronize()
        ms.append(s.elapsed_time(e))
    best = min(ms)
    print(f'{{"op": "{name}", "GiB": {gib}, "ms_best": {best:.3f}, "ms_median": {sorted(ms)[4]:.3f}, '
          f'"TBps_best": {traffic / best / 1e9:.3f}}}')
