import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from eigen_value_amd import device as dev
s = dev.DeviceSolver("cuda:0")
for n in (4096, 16384, 32768):
    for eps, mi in ((None, 0), (0.0, 4)):
        a = dev.generate("random", n, torch.float64, seed=0)
        l1, v1, i1, st1 = s.solve(a, eps=eps, max_itr=mi)
        a.mul_(2.0)
        l2, v2, i2, st2 = s.solve(a, eps=eps, max_itr=mi)
        print(n, eps, mi, "|", i1, repr(l1), "|", i2, repr(l2 / 2), "| vequal", torch.equal(v1, v2),
              "maxdiff", (v1 - v2).abs().max().item(), st1["rounds"], st2["rounds"], flush=True)
        del a
        torch.cuda.empty_cache()
