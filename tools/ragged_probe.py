import sys, time
sys.path.insert(0, '.')
import torch
from eigen_value_amd import device as dev
s = dev.DeviceSolver("cuda:0")
for dt, sizes in ((torch.float64, (8192, 8191, 16384, 16385, 32768, 32767)),
                  (torch.float32, (8192, 8190, 23168, 23171))):
    for n in sizes:
        a0 = dev.generate("random", n, dt, seed=0, device="cuda:0")
        for every in (True, False):
            best = 1e9
            for rep in range(3):
                a = a0.clone()
                torch.cuda.synchronize()
                _, _, it, st = s.solve(a, inplace=True, eps=0.0, max_itr=24, write_every_round=every)
                best = min(best, st["loop_ms"] / 24)
                del a
            print(f"{str(dt)[6:]} n={n} every={every}: {best:.4f} ms/round "
                  f"({2*n*n*a0.element_size()/best/1e6:.0f} GB/s on 2N^2b)", flush=True)
        del a0
        torch.cuda.empty_cache()
