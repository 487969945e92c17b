"""Bit-for-bit comparison of the configs[1] inference outputs between two library builds:
python scripts/chain_bitcmp.py save <out.npy>  (run once per HPE_LIB), then
python scripts/chain_bitcmp.py cmp <a.npy> <b.npy>."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'head-pose-estimation-model_amd'))

if sys.argv[1] == 'cmp':
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    print('identical' if np.array_equal(a, b) else 'DIFFER max %g' % np.abs(a - b).max())
    sys.exit(0 if np.array_equal(a, b) else 1)
import torch  # noqa: E402
import bench  # noqa: E402
import hpe  # noqa: E402
import json  # noqa: E402
gdir = os.path.join(ROOT, 'tests', 'golden', 'models')
mc = json.load(open(os.path.join(gdir, 'hrchr82r.json')))['model_config']
wts = dict(np.load(os.path.join(gdir, 'hrchr82r.npz')))
ie = hpe.model_from_config(mc, wts)._eng()
dev = torch.device('cuda', 0)
xi, _ = bench.synth(16, 99, dev)
P = bench.H * bench.W
yo = torch.empty((16 * P, 3), device=dev)
ie.forward(xi, P, out=yo)
torch.cuda.synchronize()
np.save(sys.argv[2], yo.cpu().numpy())
print('saved', yo.shape)
