"""Quick BlazeFace (config 5) timing: B images per call, kernel-by-kernel events via rocprof."""
import sys, time, os
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'head-pose-estimation-model_amd')); sys.path.insert(0, os.path.join(ROOT, 'tests'))
from hpe import blazeface as B
from util import fixture
mc, w = fixture('reg1-stoqa9pt-reg2-hrchr82r-selected')
bf = B.BlazeFace(mc, w)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
x = torch.empty((n, 128, 128, 3), device='cuda').uniform_(-1, 1)
for _ in range(3):
    bf.forward(x)
torch.cuda.synchronize()
t0 = time.perf_counter()
K = 20
for _ in range(K):
    bf.forward(x)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / K
print('B=%d  %.3f ms/batch  %.0f img/s' % (n, dt * 1e3, n / dt))
